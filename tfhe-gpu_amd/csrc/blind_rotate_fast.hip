// blind_rotate_fast.hip -- host side and key packing of the specialised N = 1024, Q < 2^27
// blind rotation (STD128, STD128_OPT and the other digit shapes fast4_shape_supported lists:
// logQ = 11 contexts, STD128_AP).  The kernel is the four-wavefront one of blind_rotate_fast4.hip
// (DESIGN.md 3.1); this file derives its key rows and constants from the generic arena and
// launches it.  (Round 3 removed the superseded two-wavefront kernel k_blind_rotate_fast2.)
//
// Same math as the generic kernel and the oracle (rgsw-acc-cggi.cpp:246-307, rgsw-acc.cpp:57-111).
// Signed Montgomery arithmetic (R = 2^32): constants centred (|w| <= Q/2) in Montgomery form.
//
// Top digit folded into the key rows (DESIGN.md 3.1 idea 1): OpenFHE's signed digits of a centred
// coefficient c satisfy c = sum_l d_l G^l exactly when no digit is thrown and the top digit never
// wraps, so D_top = G^-top (NTT(c) - sum_{l<top} G^l D_l) and
//     sum_l D_{p,l} W[2l+p] = sum_{l<top} D_{p,l} (W[2l+p] - G^(l-top) W[2top+p]) + C_p N G^-top W[2top+p]
// with C = N^-1 NTT(acc), kept by the kernel next to the accumulator.  k_pack_fast writes those rows.
#include <atomic>
#include <cstdlib>

#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {
namespace {

constexpr uint32_t FN = 1024;
// the fast key buffer: [four-wavefront kernel tables (blind_rotate_fast4.hip)][key rows]
constexpr uint32_t T4W = 5416, TB_WORDS = T4W;

struct FastConst {  // = f4::FastConst (blind_rotate_fast4.hip)
    int32_t Q, nQ, qinv, rM;  // rM = R mod Q (centred): smul(x, rM) reduces x
    uint32_t Q2, Q4, h1, kacc;  // 2Q, 4Q, (Q>>1)+1, (Q>>1)+1+4Q
    int32_t ninv;               // N^-1 (centred Montgomery form)
    uint32_t bm;                // floor(2^32 / Q) (the Barrett accumulator update)
};

// generic (plain, N^-1-scaled) BSK -> centred Montgomery key rows, the top digit folded in when
// M.fold (hc[l] = G^(l - top), hc[top] = N G^-top mod Q; STD128: 2^(7l-21) and N 2^-21), else plain
struct PackMode {
    uint32_t hc[8];
    uint32_t rw;    // key rows per (key, column) = dG2
    uint32_t fold;  // top digit eliminated
};
__global__ void k_pack_fast(uint32_t Q, const uint32_t* __restrict__ bsk, size_t words, int32_t* __restrict__ out,
                            PackMode M) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto mont = [Q](uint32_t v) {
        const uint32_t m = (uint32_t)(((uint64_t)v << 32) % Q);
        return m > Q / 2 ? (int32_t)m - (int32_t)Q : (int32_t)m;
    };
    if (idx < words) {
        // idx = (((i * 2 + k) * rw + row) * 2 + j) * N + slot; row = 2l + p
        const uint32_t row = (uint32_t)((idx / (2 * FN)) % M.rw), l = row >> 1, p = row & 1, top = M.rw / 2 - 1;
        uint32_t v = bsk[idx] % Q;
        if (M.fold) {
            const size_t it = idx + ((size_t)(2 * top + p) - row) * 2 * FN;  // row 2 top + p, same k, j, slot
            const uint64_t wt = (uint64_t)(bsk[it] % Q) * M.hc[l] % Q;
            v = l < top ? (uint32_t)(((uint64_t)v + Q - wt) % Q) : (uint32_t)wt;
        }
        out[TB_WORDS + idx] = mont(v);
    }
}

}  // namespace

// The digit shape of P for the 4-wavefront kernel; fold when no digit is thrown and the top
// digit of every centred coefficient c in [-(Q>>1)-1, Q>>1) stays in [-G/2, G/2) (no wrap), so
// that c = sum_l d_l G^l exactly (DESIGN.md 3.1 idea 1).
static Fast4Shape fast_shape(const BRParams& P) {
    Fast4Shape sh{(int)P.digits, (int)P.logG, (int)P.thr, false};
    if (P.thr == 0 && P.digits >= 2 && P.logG >= 1 && P.logG * P.digits <= 40) {
        const int64_t G = (int64_t)1 << P.logG, Qh = (int64_t)(P.Q >> 1);
        const uint32_t top = P.digits - 1;
        int64_t K = 0;
        for (uint32_t z = 0; z < top; ++z) K = K * G + G / 2;  // (G/2)(G^top - 1)/(G - 1)
        const int64_t lo = (-Qh - 1 + K) >> (P.logG * top), hi = (Qh - 1 + K) >> (P.logG * top);
        sh.fold = lo >= -G / 2 && hi < G / 2;
    }
    return sh;
}

bool fast_path_supported(const BRParams& P, int word_bits) {
    return word_bits == 32 && P.N == FN && P.dG2 == 2 * P.digits && P.Q < (1ull << 27) && P.n > 0 &&
           fast4_shape_supported(fast_shape(P));
}

size_t bsk_fast_bytes(const BRParams& P) { return ((size_t)P.n * 2 * P.dG2 * 2 * FN + TB_WORDS) * 4; }

namespace {
// TFHE_FAST_VARIANT / tfhe_set_kernel_variant select the build of the four-wavefront kernel:
// 60 = default; 70 (two ciphertexts per wavefront) and 86 (four per workgroup) are kept as
// cross-checks of the multi-ciphertext paths (tests/test_gpu_kernel_variants.py).  The other
// round-1/2 builds were removed in round 3.
constexpr int kDefaultVariant = 60;
bool known_variant(int v) { return v == 60 || v == 70 || v == 86; }
std::atomic<int> g_variant{-1};
int fast_variant() {
    int v = g_variant.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = std::getenv("TFHE_FAST_VARIANT");
        v = e && e[0] ? std::atoi(e) : kDefaultVariant;
        if (!known_variant(v)) v = kDefaultVariant;
        g_variant.store(v, std::memory_order_relaxed);
    }
    return v;
}
uint64_t powmod(uint64_t b, uint64_t e, uint64_t m) {
    uint64_t r = 1 % m;
    for (b %= m; e; e >>= 1, b = (unsigned __int128)b * b % m)
        if (e & 1) r = (unsigned __int128)r * b % m;
    return r;
}
int32_t mont_centred(uint64_t v, uint32_t Q) {
    const uint32_t m = (uint32_t)(((unsigned __int128)(v % Q) << 32) % Q);
    return m > Q / 2 ? (int32_t)m - (int32_t)Q : (int32_t)m;
}
}  // namespace

bool set_fast_variant(int v) {
    if (v == 0) v = kDefaultVariant;
    if (!known_variant(v)) return false;
    g_variant.store(v, std::memory_order_relaxed);
    return true;
}
int get_fast_variant() { return fast_variant(); }

hipError_t launch_pack_bsk_fast(const BRParams& P, const DevTables& T, const void* bsk, void* bsk_fast,
                                hipStream_t s) {
    const size_t words = (size_t)P.n * 2 * P.dG2 * 2 * FN;
    const Fast4Shape sh = fast_shape(P);
    if (P.dG2 > 16 || !fast4_shape_supported(sh)) return hipErrorNotSupported;
    PackMode M{};
    M.rw = P.dG2;
    M.fold = sh.fold;
    const uint32_t top = P.digits - 1;
    const uint64_t Q = P.Q, igt = powmod(2, Q - 1 - (uint64_t)P.logG * top, Q);  // G^-top (Q prime)
    for (uint32_t l = 0; l < top; ++l) M.hc[l] = (uint32_t)((unsigned __int128)powmod(2, (uint64_t)P.logG * l, Q) * igt % Q);
    M.hc[top] = (uint32_t)((unsigned __int128)FN * igt % Q);
    hipLaunchKernelGGL(k_pack_fast, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, (uint32_t)P.Q,
                       (const uint32_t*)bsk, words, (int32_t*)bsk_fast, M);
    if (fast4_table_words() != T4W) return hipErrorInvalidValue;
    return launch_pack_tables_fast4((uint32_t)P.Q, T, (int32_t*)bsk_fast, s);
}

hipError_t launch_blind_rotate_fast(const BRParams& P, const DevTables&, const void* bsk_fast, const uint64_t* a,
                                    uint64_t amod, uint64_t* acc, size_t B, hipStream_t s, BRDone* dn, int split_max) {
    if (B == 0) return hipSuccess;
    if (amod == 0 || (amod & (amod - 1)) || amod > 2 * FN) return hipErrorNotSupported;
    uint32_t loga = 0;
    while ((1ull << loga) < amod) ++loga;
    const uint32_t Q = (uint32_t)P.Q;
    uint32_t inv = 1;  // Q^-1 mod 2^32 by Newton iteration
    for (int it = 0; it < 5; ++it) inv *= 2u - Q * inv;
    FastConst K;
    K.Q = (int32_t)Q;
    K.nQ = -(int32_t)Q;
    K.qinv = (int32_t)inv;
    const uint32_t rm = (uint32_t)((1ull << 32) % Q);
    K.rM = rm > Q / 2 ? (int32_t)rm - (int32_t)Q : (int32_t)rm;
    K.Q2 = 2 * Q;
    K.Q4 = 4 * Q;
    K.h1 = (Q >> 1) + 1;
    K.kacc = K.h1 + 4 * Q;
    K.ninv = mont_centred(Q - (Q - 1) / FN, Q);  // N (Q-1)/N = -1 mod Q
    K.bm = (uint32_t)((1ull << 32) / Q);
    const int32_t* tabs = (const int32_t*)bsk_fast;
    return launch_blind_rotate_fast4(fast_variant(), fast_shape(P), &K, P.n, loga, tabs, tabs + TB_WORDS, a, acc, B, s,
                                     dn, split_max);
}

}  // namespace tfhe
