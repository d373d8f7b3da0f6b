// host_math.hpp -- host-side number theory for the engine: parameter selection
// (binfhecontext.cpp:42-181), negacyclic NTT tables, Shoup companions, and the
// one-time BSK/KSK conversion into the device layout.  Pure C++ (no HIP), so it
// is unit-testable without a GPU (tfhe_host_selftest).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "tfhe_hip.h"

namespace tfhe {

// Host worker count: hardware threads, capped (TFHE_HOST_THREADS overrides; the
// GPU box grants 16 CPUs per GPU although nproc reports the whole machine).
inline unsigned host_threads() {
    if (const char* e = std::getenv("TFHE_HOST_THREADS")) {
        int v = std::atoi(e);
        if (v > 0) return (unsigned)v;
    }
    unsigned h = std::thread::hardware_concurrency();
    return std::max(1u, std::min(h ? h : 1u, 16u));
}

// Static-partition parallel loop over [0, n) with std::thread.
template <typename F>
void parallel_for(size_t n, F&& f) {
    const size_t T = std::min<size_t>(host_threads(), n ? n : 1);
    if (T <= 1) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + T - 1) / T;
    for (size_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            const size_t lo = t * per, hi = std::min(n, lo + per);
            for (size_t i = lo; i < hi; ++i) f(i);
        });
    for (auto& x : th) x.join();
}

// Persistent worker pool for large host memcpy (pinned staging of the host-array API):
// creating threads per 8 MiB block would cost as much as the copy.  Thread-safe (one
// copy at a time); workers are created on first use and live until process exit.
void parallel_memcpy(void* dst, const void* src, size_t bytes);
// On the same pool: OR of n words, and the host side of the narrow PCIe wire format: u64 <-> u16 /
// u32 (wb = 2 or 4 bytes per word); parallel_narrow returns the OR of the words it narrowed (the
// caller falls back to u64 when a value did not fit).
uint64_t parallel_or(const uint64_t* src, size_t n);
uint64_t parallel_narrow(void* dst, const uint64_t* src, size_t n, int wb);
void parallel_widen(uint64_t* dst, const void* src, size_t n, int wb);
// Wire bytes per word for values below 2^bits(max_or): 2, 4 or 8.
inline int wire_bytes(uint64_t max_or) { return max_or < (1ull << 16) ? 2 : (max_or < (1ull << 32) ? 4 : 8); }

// A host array of records of w u64 words, held either flat ([records][w]) or as row pointers: record
// s is rows[s k] ... rows[s k + k - 1] (rw words each) followed, when tail is set, by tail[s]
// (w = k rw + 1).  The row form lets a caller whose ciphertexts live in separate allocations (the
// drop-in shim: one NativeVector per polynomial) hand them to the PCIe staging directly, with no
// flat copy on either side.  P is const uint64_t (inputs) or uint64_t (outputs).
template <typename P>
struct HostRows {
    P* flat = nullptr;
    P* const* rows = nullptr;
    P* tail = nullptr;
    size_t k = 1, rw = 0, w = 0;
    bool empty() const { return !flat && !rows; }
    HostRows sub(size_t s) const {  // the view from record s on
        HostRows v = *this;
        if (flat) v.flat = flat + s * w;
        if (rows) v.rows = rows + s * k;
        if (tail) v.tail = tail + s;
        return v;
    }
    // f(p, at, len): words [lo + at, lo + at + len) of the view are p[0 .. len)
    template <typename F>
    void walk(size_t lo, size_t hi, F&& f) const {
        if (flat) {
            if (hi > lo) f(flat + lo, (size_t)0, hi - lo);
            return;
        }
        for (size_t i = lo; i < hi;) {
            const size_t s = i / w, r = i % w, j = r / rw;
            if (j < k) {
                const size_t in = r - j * rw, len = std::min(rw - in, hi - i);
                f(rows[s * k + j] + in, i - lo, len);
                i += len;
            } else {
                f(tail + s, i - lo, (size_t)1);
                i += 1;
            }
        }
    }
};
using HostIn = HostRows<const uint64_t>;
using HostOut = HostRows<uint64_t>;
template <typename P>
HostRows<P> flat_rows(P* p, size_t w) {
    HostRows<P> v;
    v.flat = p;
    v.rw = v.w = w;
    return v;
}
template <typename P>
HostRows<P> ptr_rows(P* const* rows, size_t k, size_t rw, P* tail) {
    HostRows<P> v;
    v.rows = rows;
    v.k = k;
    v.rw = rw;
    v.tail = tail;
    v.w = k * rw + (tail ? 1 : 0);
    return v;
}
// The staging operations over views: words [off, off + n) of v <-> dst / src[0 .. n).
void parallel_memcpy_in(uint64_t* dst, const HostIn& v, size_t off, size_t n);
uint64_t parallel_narrow_in(void* dst, const HostIn& v, size_t off, size_t n, int wb);
void parallel_memcpy_out(const HostOut& v, size_t off, const uint64_t* src, size_t n);
void parallel_widen_out(const HostOut& v, size_t off, const void* src, size_t n, int wb);

using u128 = unsigned __int128;

inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)(((u128)a * b) % m); }
inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t m) {
    uint64_t r = a + b;
    return r >= m ? r - m : r;
}
inline uint64_t submod(uint64_t a, uint64_t b, uint64_t m) { return a >= b ? a - b : a + (m - b); }
// Contiguous shard g of D over B units: [lo, lo + cnt), sizes differing by at most one (the first
// B mod D shards one larger).  The engine's multi-device split (for_each_shard) and the one-process-
// per-GPU split of tfhe_amd.dist.shard_range are this function (tfhe_shard_range).  The reference
// deals SM_count-sized chunks round-robin instead (bootstrapping.cu:1617).
inline void shard_span(size_t B, size_t D, size_t g, size_t* lo, size_t* cnt) {
    const size_t base = B / D, extra = B % D;
    *lo = g * base + (g < extra ? g : extra);
    *cnt = base + (g < extra ? 1 : 0);
}

uint64_t powmod(uint64_t b, uint64_t e, uint64_t m);
bool is_prime(uint64_t x);
uint32_t ilog2(uint64_t x);
uint32_t bitrev(uint32_t x, uint32_t bits);

// Shoup companion: floor(w * 2^bits / Q), bits = 32 or 64
inline uint64_t shoup_companion(uint64_t w, uint64_t Q, int bits) {
    return (uint64_t)(((u128)w << bits) / Q);
}

tfhe_status params_from_set(int set, tfhe_params* p);
tfhe_status params_from_logq(int set, int arb_func, uint32_t logQ, int64_t N, uint32_t baseG, uint32_t thr,
                             tfhe_params* p);
tfhe_status params_finish(tfhe_params* p, std::string* err);

// Word width chosen for the blind rotation: 32 when every lazy sum fits a u32
// (2*dG2*Q < 2^32, Q < 2^31), else 64 (needs Q < 2^58 for the lazy sums).
int word_bits_for(const tfhe_params& p);

// NTT tables for one (Q, N): psi = primitive 2N-th root; forward CT twiddles in
// bit-reversed order (Longa-Naehrig), inverse GS twiddles, monomial table
// psi^k - 1 (k < 2N) and the exponent e_x of the forward-NTT output slot x
// (NTT(X)[x] = psi^(e_x)).
struct NttTables {
    uint32_t N = 0, logN = 0;
    uint64_t Q = 0, psi = 0, Ninv = 0;
    std::vector<uint64_t> psi_br, ipsi_br;  // [N]
    std::vector<uint64_t> mono;             // [2N] psi^k - 1
    std::vector<uint32_t> eidx;             // [N]
};
NttTables make_ntt_tables(uint64_t Q, uint32_t N);
void host_ntt_fwd(const NttTables& t, uint64_t* a);
void host_ntt_inv(const NttTables& t, uint64_t* a, bool scale);

// BSK [n][2][dG2][2][N] -> NTT domain, scaled by N^-1 (so the device INTT needs no final
// scaling), same layout; parallel over polynomials.  eval = the input is already in
// OpenFHE's EVALUATION format (= this NTT, see make_ntt_tables): scaling only, and false is
// returned when an entry is not reduced mod Q.
bool bsk_to_ntt_scaled(const tfhe_params& p, const NttTables& t, const uint64_t* bsk, bool eval, uint64_t* out);

}  // namespace tfhe
