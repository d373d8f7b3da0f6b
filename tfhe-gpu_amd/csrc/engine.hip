// engine.hip -- tfhe_ctx: key ingest (GPUSetup), device pipelines for every batch
// operation, multi-GPU sharding, and the extern "C" entry points of tfhe_hip.h.
//
// Design (MI355X-first):
//  * keys live in one per-device "key arena" (tables + NTT-domain BSK with Shoup
//    companions + packed KSK) so a whole key image is one device-to-device copy
//    (peer copy over xGMI in-process, RCCL broadcast across processes);
//  * every bootstrap of a fused op (gate, EvalFunc, EvalFloor, EvalSign,
//    EvalDecomp) stays in HBM: test vector -> blind rotation -> extraction ->
//    MKM -> LWE glue, one stream per device, host sees only LWE ciphertexts;
//  * a batch is split into contiguous shards, one host thread + stream per
//    device (the reference interleaves SM_count-sized chunks, bootstrapping.cu:1617).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "host_math.hpp"
#include "kernels.hpp"
#include "tfhe_hip.h"

using namespace tfhe;

namespace {

thread_local std::string g_last_error;

tfhe_status fail(tfhe_status s, const std::string& msg) {
    g_last_error = msg;
    return s;
}

#define HCHECK(expr)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return fail(e_ == hipErrorOutOfMemory ? TFHE_ERR_OUT_OF_MEMORY : TFHE_ERR_DEVICE,          \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                            \
    } while (0)

#define SCHECK(expr)                        \
    do {                                    \
        tfhe_status s_ = (expr);            \
        if (s_ != TFHE_OK) return s_;       \
    } while (0)

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

int ksk_bits_for(uint64_t qKS) {
    if (qKS <= (1ull << 16)) return 16;
    if (qKS <= (1ull << 32)) return 32;
    return 64;
}

// Byte offsets of everything inside the key arena; a pure function of the params,
// so an importing process can locate the sections of a broadcast image.
struct ArenaLayout {
    size_t psi, psi_sh, ipsi, ipsi_sh, mono, mono_sh, eidx, bsk, bsk_sh, ksk, kskb, total;
    size_t bsk_words, ksk_words, ksk_rows, n_pad;
};

ArenaLayout arena_layout(const tfhe_params& p, int word_bits) {
    ArenaLayout L{};
    const size_t wb = word_bits / 8, N = p.N;
    const size_t kb = ksk_bits_for(p.qKS) / 8;
    L.bsk_words = (size_t)p.n * 2 * p.dG2 * 2 * N;
    L.ksk_rows = (size_t)N * p.baseKS * p.dKS;
    const size_t vec = 16 / kb;  // KSK row padded to a multiple of 16 bytes
    L.n_pad = (p.n + vec - 1) / vec * vec;
    L.ksk_words = L.ksk_rows * (p.n + 1);  // caller's layout (B at index n)
    size_t o = 0;
    L.psi = o; o = align_up(o + N * wb);
    L.psi_sh = o; o = align_up(o + N * wb);
    L.ipsi = o; o = align_up(o + N * wb);
    L.ipsi_sh = o; o = align_up(o + N * wb);
    L.mono = o; o = align_up(o + 2 * N * wb);
    L.mono_sh = o; o = align_up(o + 2 * N * wb);
    L.eidx = o; o = align_up(o + N * 4);
    L.bsk = o; o = align_up(o + L.bsk_words * wb);
    L.bsk_sh = o; o = align_up(o + L.bsk_words * wb);
    L.ksk = o; o = align_up(o + L.ksk_rows * L.n_pad * kb);
    L.kskb = o; o = align_up(o + L.ksk_rows * kb);
    L.total = o;
    return L;
}

struct Scratch {
    uint64_t* acc = nullptr;  // [cap][2][N]
    uint64_t* a = nullptr;    // [cap][n]
    uint64_t* ext = nullptr;  // [cap][N+1]
    uint64_t* lwe[6] = {};    // [cap][n+1] each
    void* ks = nullptr;       // tiled key switch: digit planes (ks_tiled_scratch_bytes) for ks_cap
    size_t ks_cap = 0;
    size_t cap = 0;
    uint64_t* io = nullptr;   // host-array staging: in1 | in2 | out
    size_t io_words = 0;
    void* pk = nullptr;       // the same arrays in the narrow wire format (u16 / u32 words)
    size_t pk_bytes = 0;
};

// A device has a compute stream (`stream`, scratch `sc`) and a copy stream (`stream2`):
// host-array calls pipeline their sub-batches' PCIe copies on the copy stream against the
// kernels on the compute stream, through two device I/O sets (sc.io, sc2.io).  Device-pointer
// entry points use the compute scratch on the caller's stream (or `stream`).
struct Device {
    int id = 0;
    hipStream_t stream = nullptr;
    unsigned char* arena = nullptr;
    void* bsk_fast = nullptr;
    void* keys_f64 = nullptr;  // exact-FP64 path: centred double tables + BSK
    void* keys_sf = nullptr;   // special-form path: W1 = w 2^32 mod Q of the arena's tables and BSK, factor rows
    void* ks40 = nullptr;      // split-word key-switch records of 8-byte keys (ks_tiled.hip k_pack_ks40)
    DuoDev duo;                // two-workgroup forms (sf2duo, f64wduo): exchange buffers, wait deadline, co-resident
                               // pairs, launch fence (kernels.hpp DuoDev; alloc_duo)
    Scratch sc;
    DevTables tables{};
    hipStream_t stream2 = nullptr;  // copy stream of the host-array runner
    Scratch sc2;                    // only its io set is used
    void* pin[2] = {};               // pinned staging blocks for the host-array API
    hipEvent_t pin_ev[2] = {};       // last DMA that used each block
    // Lane 0's scratch (sc) is shared by the host-array path (on `stream`) and the
    // device-resident entry points (on the caller's stream): every user of sc waits on
    // this event before its first kernel and records it after its last one, so work
    // queued on different streams never overlaps on the same scratch.
    hipEvent_t sc_fence = nullptr;
    hipEvent_t h2d_ev[2] = {};  // host-array runner: input of I/O set k landed
    hipEvent_t k_ev[2] = {};    // host-array runner: kernels that use I/O set k done
    // Completion flags of the host-array EvalAcc (d2h_flagged): pinned host words, 4 per ciphertext,
    // set by the blind rotation's waves; br_done.flags is non-null only while such a call queues its op.
    uint32_t* flags = nullptr;
    size_t flags_words = 0;
    BRDone br_done{};
};

// hipMalloc'd buffer owned by one scope (error paths free it too)
struct DevBuf {
    void* p = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) hipFree(p);
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

constexpr size_t kStageBytes = (size_t)8 << 20;

}  // namespace

struct tfhe_ctx;
namespace {
void free_device(Device& d);
}

struct tfhe_ctx {
    tfhe_params p{};
    int word_bits = 64;
    int ksk_bits = 64;
    bool use_fast = false;
    bool use_f64 = false;
    bool f64_fold = false;  // exact-FP64 kernel with the top digit's transforms eliminated
    bool use_sf = false;    // special-form u64 kernel (logQ / arbFunc contexts, default)
    BRParams br{};
    KSParams ks{};
    ArenaLayout layout{};
    std::vector<Device> devs;
    std::atomic<uint64_t> bootstraps{0};
    int replicate_method = TFHE_REPLICATE_NONE;
    double replicate_ms = 0;
    size_t max_chunk = 65536;  // the reference's max_bootstapping_num, bootstrapping.cuh:140
    Knobs kn{};                // launch choices: environment at setup, tfhe_set_knobs afterwards
    std::string rccl_lib;      // TFHE_RCCL_LIB at setup ("" = the system librccl)
    ~tfhe_ctx();  // frees every device's arena, scratch, streams (error paths included)
};

namespace {

// ---------------------------------------------------------------------------
// setup helpers
// ---------------------------------------------------------------------------
// Launch knobs from the environment, once per context (tfhe_setup*): the A/B switches of earlier rounds'
// measurements.  Afterwards only tfhe_set_knobs changes them; no launch reads the environment.
// The range every knob must lie in (tfhe_set_knobs and the environment alike); nullptr when valid.
const char* knob_out_of_range(const Knobs& k) {
    if (k.ks_tiled_min < -1) return "ks_tiled_min (TFHE_KS_TILED_MIN) < -1";
    if (k.ks_cts < 0 || k.ks_cts > 4 || k.ks_cts == 3) return "ks_cts (TFHE_KS_CTS) not 0, 1, 2 or 4";
    if (k.ks_split < 1) return "ks_split (TFHE_KS_SPLIT) < 1";
    if (k.host_parts < 1) return "host_parts (TFHE_HOST_PARTS) < 1";
    if (k.generic < 0 || k.generic > 2) return "generic (TFHE_GENERIC) not in 0..2";
    if (k.duo < 0 || k.duo > 256) return "duo (TFHE_DUO) not in 0..256";
    if (k.split4 < 0) return "split4 (TFHE_SPLIT4) < 0";
    if (k.f64w != 1) return "f64w (TFHE_F64W): the slot-layout FP64 kernel it selected was retired in round 5 (must be 1)";
    for (int32_t v : {k.ks_pk, k.wire, k.acc_flags, k.sf2, k.sf2p, k.trace, k.ks40})
        if (v < 0 || v > 1) return "a 0/1 knob (TFHE_KS_PK, TFHE_WIRE, TFHE_ACC_FLAGS, TFHE_SF2, TFHE_SF2P, TFHE_KS40) "
                                   "not 0 or 1";
    if (k.probe < 0) return "probe < 0";
    return nullptr;
}

// bad: the first variable that is not a whole number, or whose value is out of range
Knobs knobs_from_env(std::string& bad) {
    Knobs k;
    auto num = [&bad](const char* name, int32_t& dst) {
        const char* e = std::getenv(name);
        if (!e || !e[0]) return;
        char* end = nullptr;
        const long v = std::strtol(e, &end, 10);
        if (*end != '\0' || v < INT32_MIN || v > INT32_MAX) {
            if (bad.empty()) bad = std::string(name) + "=" + e + " is not a whole number";
            return;
        }
        dst = (int32_t)v;
    };
    num("TFHE_KS_TILED_MIN", k.ks_tiled_min);
    num("TFHE_KS_CTS", k.ks_cts);
    num("TFHE_KS_SPLIT", k.ks_split);
    num("TFHE_KS_PK", k.ks_pk);
    num("TFHE_HOST_PARTS", k.host_parts);
    num("TFHE_WIRE", k.wire);
    num("TFHE_ACC_FLAGS", k.acc_flags);
    {  // retired (round 5): scripts of earlier rounds export TFHE_F64W=0 / 1; accepted and ignored with a
       // warning rather than failing contexts that never touch the FP64 kernel.  tfhe_set_knobs
       // still requires 1.
        int32_t f = 1;
        num("TFHE_F64W", f);
        if (f != 1 && bad.empty())
            std::fprintf(stderr, "[tfhe] TFHE_F64W=%d ignored: the slot-layout FP64 kernel it selected was retired in "
                                 "round 5 (f64w is the only FP64 form)\n", (int)f);
    }
    num("TFHE_SF2", k.sf2);
    num("TFHE_DUO", k.duo);
    num("TFHE_SF2P", k.sf2p);
    num("TFHE_SPLIT4", k.split4);
    num("TFHE_KS40", k.ks40);
    num("TFHE_GENERIC", k.generic);
    if (const char* e = std::getenv("TFHE_GENERIC_V1"); e && e[0] == '1') k.generic = 1;    // round-3 names
    if (const char* e = std::getenv("TFHE_GENERIC_GEN3"); e && e[0] == '0') k.generic = 2;
    k.trace = std::getenv("TFHE_TRACE") != nullptr;
    if (const char* why = knob_out_of_range(k); why && bad.empty()) bad = why;
    return k;
}

tfhe_status init_derived(tfhe_ctx* c) {
    const tfhe_params& p = c->p;
    std::string bad;
    c->kn = knobs_from_env(bad);
    if (!bad.empty()) return fail(TFHE_ERR_INVALID_ARGUMENT, "launch knob from the environment: " + bad);
    c->word_bits = word_bits_for(p);
    c->ksk_bits = ksk_bits_for(p.qKS);
    c->layout = arena_layout(p, c->word_bits);
    c->br.N = p.N;
    c->br.logN = ilog2(p.N);
    c->br.n = p.n;
    c->br.dG2 = p.dG2;
    c->br.digits = p.digitsG - p.numDigitsToThrow;
    c->br.thr = p.numDigitsToThrow;
    c->br.logG = ilog2(p.baseG);
    c->br.Q = p.Q;
    c->br.r1 = c->word_bits == 32 ? (uint64_t)((((u128)1) << 32) / p.Q) : (uint64_t)((((u128)1) << 64) / p.Q);
    c->ks.N = p.N;
    c->ks.n = p.n;
    c->ks.baseKS = p.baseKS;
    c->ks.dKS = p.dKS;
    c->ks.Q = p.Q;
    c->ks.qKS = p.qKS;
    c->ks.n_pad = (uint32_t)c->layout.n_pad;
    const char* force = std::getenv("TFHE_FORCE_GENERIC");
    c->use_fast = fast_path_supported(c->br, c->word_bits) && !(force && force[0] == '1');
    c->use_f64 = f64_path_supported(c->br, c->word_bits) && !(force && force[0] == '1');
    c->f64_fold = c->use_f64 && f64_fold_enabled(c->br);
    if (c->use_f64 && !f64_instance_available(c->br, c->f64_fold)) c->f64_fold = false;
    if (c->use_f64 && !f64_instance_available(c->br, c->f64_fold)) c->use_f64 = false;
    // Q = 2^54 - c: the special-form kernel (TFHE_SF=0 keeps the Shoup gen3 kernel)
    const char* sfe = std::getenv("TFHE_SF");
    c->use_sf = !c->use_fast && !c->use_f64 && sf_path_supported(c->br, c->word_bits) &&
                !(force && force[0] == '1') && !(sfe && sfe[0] == '0');
    if (p.Q >= (1ull << 58) || (c->word_bits == 64 && (u128)2 * p.dG2 * p.Q >= ((u128)1 << 64)))
        return fail(TFHE_ERR_UNSUPPORTED, "modulus too large for lazy accumulation");
    if (p.baseKS > 256) return fail(TFHE_ERR_UNSUPPORTED, "baseKS > 256 not supported");
    return TFHE_OK;
}

template <typename W>
void fill_words(std::vector<unsigned char>& host, size_t off, const uint64_t* src, size_t count) {
    W* dst = reinterpret_cast<W*>(host.data() + off);
    const size_t blk = 1 << 16;
    parallel_for((count + blk - 1) / blk, [&](size_t b) {
        for (size_t i = b * blk; i < std::min(count, (b + 1) * blk); ++i) dst[i] = (W)src[i];
    });
}

template <typename W>
void fill_companions(std::vector<unsigned char>& host, size_t off, const uint64_t* src, size_t count, uint64_t Q) {
    W* dst = reinterpret_cast<W*>(host.data() + off);
    const int bits = sizeof(W) * 8;
    const size_t blk = 1 << 14;
    parallel_for((count + blk - 1) / blk, [&](size_t b) {
        for (size_t i = b * blk; i < std::min(count, (b + 1) * blk); ++i) dst[i] = (W)shoup_companion(src[i], Q, bits);
    });
}

// KSK [rows][n+1] -> A part [rows][n_pad] (zero padded) + B part [rows]
template <typename W>
void pack_ksk(std::vector<unsigned char>& img, const ArenaLayout& L, uint32_t n, const uint64_t* ksk) {
    W* A = reinterpret_cast<W*>(img.data() + L.ksk);
    W* Bp = reinterpret_cast<W*>(img.data() + L.kskb);
    const size_t blk = 4096;
    parallel_for((L.ksk_rows + blk - 1) / blk, [&](size_t b) {
        for (size_t r = b * blk; r < std::min(L.ksk_rows, (b + 1) * blk); ++r) {
            const uint64_t* src = ksk + r * (n + 1);
            W* dst = A + r * L.n_pad;
            for (uint32_t k = 0; k < n; ++k) dst[k] = (W)src[k];
            for (size_t k = n; k < L.n_pad; ++k) dst[k] = 0;
            Bp[r] = (W)src[n];
        }
    });
}

// Build the whole key image on the host (one-time, GPUSetup_core's job in the
// reference, bootstrapping.cu:874-1083).
tfhe_status build_host_image(tfhe_ctx* c, const uint64_t* bsk, bool bsk_eval, const uint64_t* ksk,
                             std::vector<unsigned char>& img) {
    const tfhe_params& p = c->p;
    const ArenaLayout& L = c->layout;
    img.assign(L.total, 0);
    NttTables t = make_ntt_tables(p.Q, p.N);
    std::vector<uint64_t> bsk_ntt(L.bsk_words);
    if (!bsk_to_ntt_scaled(p, t, bsk, bsk_eval, bsk_ntt.data()))
        return fail(TFHE_ERR_INVALID_ARGUMENT, "evaluation-format BSK entry >= Q");
    auto put = [&](auto tag, size_t off, size_t off_sh, const uint64_t* v, size_t count) {
        using W = decltype(tag);
        fill_words<W>(img, off, v, count);
        if (off_sh != (size_t)-1) fill_companions<W>(img, off_sh, v, count, p.Q);
    };
    if (c->word_bits == 32) {
        put(uint32_t{}, L.psi, L.psi_sh, t.psi_br.data(), p.N);
        put(uint32_t{}, L.ipsi, L.ipsi_sh, t.ipsi_br.data(), p.N);
        put(uint32_t{}, L.mono, L.mono_sh, t.mono.data(), 2ull * p.N);
        put(uint32_t{}, L.bsk, L.bsk_sh, bsk_ntt.data(), L.bsk_words);
    } else {
        put(uint64_t{}, L.psi, L.psi_sh, t.psi_br.data(), p.N);
        put(uint64_t{}, L.ipsi, L.ipsi_sh, t.ipsi_br.data(), p.N);
        put(uint64_t{}, L.mono, L.mono_sh, t.mono.data(), 2ull * p.N);
        put(uint64_t{}, L.bsk, L.bsk_sh, bsk_ntt.data(), L.bsk_words);
    }
    std::memcpy(img.data() + L.eidx, t.eidx.data(), sizeof(uint32_t) * p.N);
    if (c->use_fast)  // the fast kernel derives e_x = 2 bitrev(x) + 1 in registers
        for (uint32_t x = 0; x < p.N; ++x)
            if (t.eidx[x] != 2 * bitrev(x, t.logN) + 1) return fail(TFHE_ERR_INTERNAL, "eidx is not 2 bitrev(x) + 1");
    // KSK: packed to the narrowest word holding qKS (reference keeps u64, bootstrapping.cu:963)
    const uint64_t qks = p.qKS;
    std::atomic<bool> bad{false};
    const size_t blk = 1 << 16;
    parallel_for((L.ksk_words + blk - 1) / blk, [&](size_t b) {
        for (size_t i = b * blk; i < std::min(L.ksk_words, (b + 1) * blk); ++i)
            if (ksk[i] >= qks) bad = true;
    });
    if (bad) return fail(TFHE_ERR_INVALID_ARGUMENT, "KSK entry >= qKS");
    if (c->ksk_bits == 16) pack_ksk<uint16_t>(img, L, p.n, ksk);
    else if (c->ksk_bits == 32) pack_ksk<uint32_t>(img, L, p.n, ksk);
    else pack_ksk<uint64_t>(img, L, p.n, ksk);
    return TFHE_OK;
}

void bind_tables(tfhe_ctx* c, Device& d) {
    const ArenaLayout& L = c->layout;
    d.tables.psi = d.arena + L.psi;
    d.tables.psi_sh = d.arena + L.psi_sh;
    d.tables.ipsi = d.arena + L.ipsi;
    d.tables.ipsi_sh = d.arena + L.ipsi_sh;
    d.tables.mono = d.arena + L.mono;
    d.tables.mono_sh = d.arena + L.mono_sh;
    d.tables.eidx = reinterpret_cast<const uint32_t*>(d.arena + L.eidx);
}

// The duo state of a device: the exchange buffer, the partner-wait deadline (kDuoWaitMs of the wall clock
// s_memrealtime reads), the pairs it holds co-resident (one duo workgroup per CU) and the launch fence
tfhe_status alloc_duo(Device& d) {
    HCHECK(hipMalloc(&d.duo.base, duo_bytes()));
    HCHECK(hipMemsetAsync(d.duo.base, 0, duo_bytes(), d.stream));
    int khz = 0, cus = 0;
    HCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d.id));
    HCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d.id));
    d.duo.wait_ticks = (uint64_t)(khz > 0 ? khz : 100000) * kDuoWaitMs;
    d.duo.resident_pairs = (uint32_t)std::max(0, cus / 2);
    HCHECK(hipEventCreateWithFlags(&d.duo.fence, hipEventDisableTiming));
    d.duo.mu = new std::mutex;
    return TFHE_OK;
}

tfhe_status finish_device(tfhe_ctx* c, Device& d) {
    bind_tables(c, d);
    if (c->use_fast) {
        HCHECK(hipMalloc(&d.bsk_fast, bsk_fast_bytes(c->br)));
        HCHECK(launch_pack_bsk_fast(c->br, d.tables, d.arena + c->layout.bsk, d.bsk_fast, d.stream));
        HCHECK(hipStreamSynchronize(d.stream));
    }
    if (c->use_f64) {
        HCHECK(hipMalloc(&d.keys_f64, bsk_f64_bytes(c->br)));
        HCHECK(launch_pack_bsk_f64(c->br, d.tables, d.arena + c->layout.bsk, c->f64_fold, d.keys_f64, d.stream));
        if (f64_duo_form(c->br, c->f64_fold)) SCHECK(alloc_duo(d));
        HCHECK(hipStreamSynchronize(d.stream));
    }
    if (c->ksk_bits == 64 && ks40_bytes(c->ks) > 0) {  // the logQ contexts' KSK (qKS = 2^35) as split words
        HCHECK(hipMalloc(&d.ks40, ks40_bytes(c->ks)));
        HCHECK(launch_pack_ks40(c->ks, d.arena + c->layout.ksk, d.ks40, d.stream));
        HCHECK(hipStreamSynchronize(d.stream));
    }
    if (c->use_sf) {
        HCHECK(hipMalloc(&d.keys_sf, sf_bytes(c->br)));
        HCHECK(launch_pack_sf(c->br, d.tables, d.arena + c->layout.bsk, d.keys_sf, d.stream));
        if (c->br.digits == 1 || c->br.digits == 2) SCHECK(alloc_duo(d));  // sfduo<1> / sf2duo
        HCHECK(hipStreamSynchronize(d.stream));
    }
    return TFHE_OK;
}

void free_device(Device& d) {
    if (d.id < 0) return;
    hipSetDevice(d.id);
    if (d.sc_fence) hipEventSynchronize(d.sc_fence), hipEventDestroy(d.sc_fence);
    if (d.stream) hipStreamSynchronize(d.stream);
    hipFree(d.arena);
    hipFree(d.bsk_fast);
    hipFree(d.keys_f64);
    hipFree(d.keys_sf);
    hipFree(d.ks40);
    hipFree(d.duo.base);
    if (d.duo.fence) hipEventDestroy(d.duo.fence);
    delete d.duo.mu;
    d.duo = DuoDev{};
    if (d.stream2) hipStreamSynchronize(d.stream2);
    for (Scratch* sc : {&d.sc, &d.sc2}) {
        hipFree(sc->acc);
        hipFree(sc->a);
        hipFree(sc->ext);
        for (auto* p : sc->lwe) hipFree(p);
        hipFree(sc->ks);
        hipFree(sc->io);
        hipFree(sc->pk);
    }
    if (d.flags) hipHostFree(d.flags);
    for (int k = 0; k < 2; ++k) {
        if (d.pin_ev[k]) hipEventSynchronize(d.pin_ev[k]), hipEventDestroy(d.pin_ev[k]);
        if (d.pin[k]) hipHostFree(d.pin[k]);
        if (d.h2d_ev[k]) hipEventDestroy(d.h2d_ev[k]);
        if (d.k_ev[k]) hipEventDestroy(d.k_ev[k]);
    }
    if (d.stream) hipStreamDestroy(d.stream);
    if (d.stream2) hipStreamDestroy(d.stream2);
    d = Device{};
    d.id = -1;
}

tfhe_status create_streams(Device& d) {
    HCHECK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    HCHECK(hipStreamCreateWithFlags(&d.stream2, hipStreamNonBlocking));
    HCHECK(hipEventCreateWithFlags(&d.sc_fence, hipEventDisableTiming));
    return TFHE_OK;
}

// Order `s` after every earlier user of lane 0's scratch (see Device::sc_fence).
tfhe_status sc_acquire(Device& d, hipStream_t s) {
    HCHECK(hipStreamWaitEvent(s, d.sc_fence, 0));
    return TFHE_OK;
}
tfhe_status sc_release(Device& d, hipStream_t s) {
    HCHECK(hipEventRecord(d.sc_fence, s));
    return TFHE_OK;
}

// The context device holding device buffer p (the _device entry points' device index).
tfhe_status device_for(tfhe_ctx* c, const void* p, Device*& out) {
    if (c->devs.size() == 1) {  // nothing to choose: skip the query
        out = &c->devs[0];
        return TFHE_OK;
    }
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return fail(TFHE_ERR_INVALID_ARGUMENT, "not a device buffer");
    }
    for (Device& d : c->devs)
        if (d.id == at.device) {
            out = &d;
            return TFHE_OK;
        }
    return fail(TFHE_ERR_INVALID_ARGUMENT, "buffer is on a device this context does not use");
}

tfhe_status ensure_scratch(tfhe_ctx* c, Device& d, size_t B) {
    if (B <= d.sc.cap) return TFHE_OK;
    const tfhe_params& p = c->p;
    if (d.sc_fence) HCHECK(hipEventSynchronize(d.sc_fence));  // no queued kernel still uses the old buffers
    const size_t cap = std::max(B, std::min(c->max_chunk, (size_t)1024));
    hipFree(d.sc.acc);
    hipFree(d.sc.a);
    hipFree(d.sc.ext);
    for (auto*& q : d.sc.lwe) hipFree(q), q = nullptr;
    hipFree(d.sc.ks);
    uint64_t* io = d.sc.io;
    const size_t io_words = d.sc.io_words;
    void* pk = d.sc.pk;
    const size_t pk_bytes = d.sc.pk_bytes;
    d.sc = Scratch{};
    d.sc.io = io, d.sc.io_words = io_words, d.sc.pk = pk, d.sc.pk_bytes = pk_bytes;
    HCHECK(hipMalloc(&d.sc.acc, cap * 2 * p.N * sizeof(uint64_t)));
    HCHECK(hipMalloc(&d.sc.a, cap * p.n * sizeof(uint64_t)));
    HCHECK(hipMalloc(&d.sc.ext, cap * (p.N + 1) * sizeof(uint64_t)));
    for (auto*& q : d.sc.lwe) HCHECK(hipMalloc(&q, cap * (p.n + 1) * sizeof(uint64_t)));
    if (ks_tiled_supported(c->ks)) {
        HCHECK(hipMalloc(&d.sc.ks, ks_tiled_scratch_bytes(c->ks, cap)));
        d.sc.ks_cap = cap;
    }
    d.sc.cap = cap;
    return TFHE_OK;
}

size_t ks_tiled_min(const tfhe_ctx* c);

// The tiled key switch's digit planes alone, for the device-resident key switch (which needs
// none of the bootstrap scratch): grown to B only when the tiled form will run.
tfhe_status ensure_ks_scratch(tfhe_ctx* c, Device& d, size_t B) {
    const size_t tmin = ks_tiled_min(c);
    if (!ks_tiled_supported(c->ks) || tmin == 0 || B < tmin || B <= d.sc.ks_cap) return TFHE_OK;
    if (d.sc_fence) HCHECK(hipEventSynchronize(d.sc_fence));
    hipFree(d.sc.ks);
    d.sc.ks = nullptr, d.sc.ks_cap = 0;
    HCHECK(hipMalloc(&d.sc.ks, ks_tiled_scratch_bytes(c->ks, B)));
    d.sc.ks_cap = B;
    return TFHE_OK;
}

// ---------------------------------------------------------------------------
// device pipelines (one device, one stream, B <= scratch capacity)
// ---------------------------------------------------------------------------
tfhe_status dev_blind_rotate(tfhe_ctx* c, Device& d, const uint64_t* a, uint64_t amod, uint64_t* acc, size_t B) {
    if (amod == 0 || (2ull * c->p.N) % amod != 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "a-modulus must divide 2N");
    const ArenaLayout& L = c->layout;
    if (c->use_fast && (amod & (amod - 1)) == 0) {
        HCHECK(launch_blind_rotate_fast(c->br, d.tables, d.bsk_fast, a, amod, acc, B, d.stream,
                                        d.br_done.flags ? &d.br_done : nullptr, c->kn.split4));
    } else if (c->use_f64) {
        HCHECK(launch_blind_rotate_f64(c->br, d.tables, d.keys_f64, c->f64_fold, a, amod, acc, B, d.stream, c->kn,
                                       d.duo.base ? &d.duo : nullptr));
    } else if (c->use_sf) {
        HCHECK(launch_blind_rotate_sf(c->br, d.tables, d.arena + L.bsk, d.keys_sf, a, amod, acc, B, d.stream, c->kn,
                                      d.duo.base ? &d.duo : nullptr));
    } else {
        HCHECK(launch_blind_rotate_generic(c->word_bits, c->br, d.tables, d.arena + L.bsk, d.arena + L.bsk_sh, a,
                                           amod, acc, B, d.stream, c->kn));
    }
    c->bootstraps += B;
    return TFHE_OK;
}

// Smallest batch that takes the tiled key switch (knob ks_tiled_min / TFHE_KS_TILED_MIN; 0 = never).
// Round 2 set it at 4096 (u16 keys) / 256 (wider keys): the tiled workgroups each swept all N dKS rows
// (~1 ms for STD128 at any batch up to 8192).
size_t ks_tiled_min(const tfhe_ctx* c) {
    if (c->kn.ks_tiled_min >= 0) return (size_t)c->kn.ks_tiled_min;  // knob (TFHE_KS_TILED_MIN)
    // round 4 (profiles/r04b/ks_sweep.log): with the steps split up to 16 ways at small batches, the tiled
    // form beats the gather at every batch from 1 to 1024 and every key width (STD128Q B = 128: 0.33 vs
    // 6.3 ms; logQ = 23: 1.68 vs 9.3 ms; STD128 B = 1: 0.105 vs 0.64 ms); the gather stays for key
    // shapes the tiled form does not support
    return 1;
}

// the tiled form runs when d.sc.ks holds B ciphertexts (ensure_scratch / ensure_ks_scratch)
tfhe_status dev_mkm(tfhe_ctx* c, Device& d, const uint64_t* ext, uint64_t fmod, uint64_t* out, size_t B) {
    if (fmod < 2) return fail(TFHE_ERR_INVALID_ARGUMENT, "fmod < 2");
    const size_t tmin = ks_tiled_min(c);
    if (tmin && B >= tmin && d.sc.ks && B <= d.sc.ks_cap) {
        const hipError_t e = launch_ks_tiled(c->ks, c->ksk_bits, d.arena + c->layout.ksk, d.arena + c->layout.kskb,
                                             ext, fmod, out, B, d.sc.ks, d.stream, c->kn, d.ks40);
        if (e != hipErrorNotSupported) {
            HCHECK(e);
            return TFHE_OK;
        }
    }
    HCHECK(launch_mkm(c->ks, c->ksk_bits, d.arena + c->layout.ksk, d.arena + c->layout.kskb, ext, fmod, out, B,
                      d.stream));
    return TFHE_OK;
}

// BootstrapFunc / BootstrapGate on device: ct[B][n+1] mod tv.ctmod -> out mod fmod
tfhe_status dev_bootstrap(tfhe_ctx* c, Device& d, TvParams tv, uint64_t b_add, const uint64_t* ct, uint64_t* out,
                          size_t B) {
    tv.N = c->p.N;
    tv.n = c->p.n;
    tv.Q = c->p.Q;
    tv.Q8 = c->p.Q / 8 + 1;
    if ((2ull * c->p.N) % tv.ctmod != 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "ciphertext modulus must divide 2N");
    HCHECK(launch_build_testvector(tv, ct, d.sc.acc, d.sc.a, B, d.stream));
    SCHECK(dev_blind_rotate(c, d, d.sc.a, tv.ctmod, d.sc.acc, B));
    HCHECK(launch_extract(c->p.N, c->p.Q, b_add, d.sc.acc, d.sc.ext, B, d.stream));
    return dev_mkm(c, d, d.sc.ext, tv.fmod, out, B);
}

uint64_t gate_const(int gate, uint64_t q) {  // rgsw-cryptoparameters.h:130-137
    static const uint64_t k[] = {5, 7, 1, 3, 5, 1};
    return k[gate] * (q >> 3);
}

// vector EvalBinGate, binfhe-base-scheme.cpp:598-677.  Uses lwe[0..2] + lwe[5].
tfhe_status dev_gate(tfhe_ctx* c, Device& d, int gate, const uint64_t* ct1, const uint64_t* ct2, uint64_t q,
                     uint64_t* out, size_t B) {
    const uint32_t n = c->p.n;
    hipStream_t s = d.stream;
    if (gate == TFHE_XOR || gate == TFHE_XNOR) {
        uint64_t *n1 = d.sc.lwe[3], *n2 = d.sc.lwe[4], *t1 = d.sc.lwe[5];
        HCHECK(launch_lwe_op(LWE_NOT, n, q, 0, ct1, nullptr, n1, B, s));
        HCHECK(launch_lwe_op(LWE_NOT, n, q, 0, ct2, nullptr, n2, B, s));
        SCHECK(dev_gate(c, d, TFHE_AND, ct1, n2, q, t1, B));   // AND(ct1, NOT ct2)
        SCHECK(dev_gate(c, d, TFHE_AND, n1, ct2, q, n2, B));   // AND(NOT ct1, ct2)
        SCHECK(dev_gate(c, d, TFHE_OR, t1, n2, q, out, B));
        if (gate == TFHE_XNOR) HCHECK(launch_lwe_op(LWE_NOT, n, q, 0, out, nullptr, out, B, s));
        return TFHE_OK;
    }
    uint64_t* prep = d.sc.lwe[0];
    HCHECK(launch_lwe_op((gate == TFHE_XOR_FAST || gate == TFHE_XNOR_FAST) ? LWE_DOUBLE_SUB : LWE_ADD, n, q, 0, ct1,
                         ct2, prep, B, s));
    TvParams tv{};
    tv.mode = TV_GATE;
    tv.ctmod = q;
    tv.fmod = q;
    tv.q1 = gate_const(gate, q);
    tv.q2 = addmod(tv.q1, q >> 1, q);
    return dev_bootstrap(c, d, tv, c->p.Q / 8 + 1, prep, out, B);
}

// binfhe-base-scheme.cpp:162-186
int check_input_function(const uint64_t* lut, uint64_t len, uint64_t mod) {
    const uint64_t h = len / 2;
    if (lut[0] == mod - lut[h]) {
        for (uint64_t i = 1; i < h; ++i)
            if (lut[i] != mod - lut[h + i]) return 2;
        return 0;
    }
    if (lut[0] == lut[h]) {
        for (uint64_t i = 1; i < h; ++i)
            if (lut[i] != lut[h + i]) return 2;
        return 1;
    }
    return 2;
}

// vector EvalFunc, binfhe-base-scheme.cpp:679-924.  d_lut is a device LUT ([q] or [B][q]).
tfhe_status dev_func(tfhe_ctx* c, Device& d, int prop, const uint64_t* ct, uint64_t q, const uint64_t* d_lut,
                     uint64_t lut_stride, uint64_t* out, size_t B) {
    const uint32_t n = c->p.n;
    const uint64_t beta = 128;
    hipStream_t s = d.stream;
    uint64_t *ct1 = d.sc.lwe[0], *ct2 = d.sc.lwe[1], *ct3 = d.sc.lwe[2];
    TvParams tv{};
    tv.lut = d_lut;
    tv.lut_stride = lut_stride;
    tv.lut_len = q;
    if (prop == 0) {  // negacyclic: one bootstrap
        HCHECK(launch_lwe_op(LWE_ADD_CONST, n, q, beta, ct, nullptr, ct1, B, s));
        tv.mode = TV_LUT;
        tv.ctmod = q;
        tv.fmod = q;
        return dev_bootstrap(c, d, tv, 0, ct1, out, B);
    }
    if (prop == 2) {  // arbitrary: raise to 2q, two bootstraps
        if (q > c->p.N) return fail(TFHE_ERR_UNSUPPORTED, "arbitrary function needs q <= N");
        const uint64_t dq = q << 1;
        HCHECK(launch_lwe_op(LWE_ADD_CONST, n, dq, beta, ct, nullptr, ct2, B, s));
        tv.mode = TV_HALF;
        tv.ctmod = dq;
        tv.fmod = dq;
        SCHECK(dev_bootstrap(c, d, tv, 0, ct2, ct3, B));
        HCHECK(launch_lwe_op(LWE_SUB, n, dq, 0, ct, ct3, ct3, B, s));  // EvalSubEq2(ct1, ct3)
        HCHECK(launch_lwe_op(LWE_ADD_CONST, n, dq, beta, ct3, nullptr, ct3, B, s));
        HCHECK(launch_lwe_op(LWE_SUB_CONST, n, dq, q >> 1, ct3, nullptr, ct3, B, s));
        tv.mode = TV_LUT2;
        SCHECK(dev_bootstrap(c, d, tv, 0, ct3, out, B));
        HCHECK(launch_lwe_op(LWE_SET_MOD, n, q, 0, out, nullptr, out, B, s));
        return TFHE_OK;
    }
    // periodic
    HCHECK(launch_lwe_op(LWE_ADD_CONST, n, q, beta, ct, nullptr, ct1, B, s));
    tv.mode = TV_HALF;
    tv.ctmod = q;
    tv.fmod = q;
    SCHECK(dev_bootstrap(c, d, tv, 0, ct1, ct2, B));
    HCHECK(launch_lwe_op(LWE_SUB, n, q, 0, ct, ct2, ct2, B, s));  // EvalSubEq2(ct, ct2)
    HCHECK(launch_lwe_op(LWE_ADD_CONST, n, q, beta, ct2, nullptr, ct2, B, s));
    HCHECK(launch_lwe_op(LWE_SUB_CONST, n, q, q >> 2, ct2, nullptr, ct2, B, s));
    tv.mode = TV_LUT1;
    return dev_bootstrap(c, d, tv, 0, ct2, out, B);
}

// vector EvalFloor, binfhe-base-scheme.cpp:926-987.  out may alias nothing; uses lwe[3], lwe[4].
tfhe_status dev_floor(tfhe_ctx* c, Device& d, const uint64_t* ct, uint64_t mod, uint32_t roundbits, uint64_t* out,
                      size_t B) {
    const uint32_t n = c->p.n;
    const uint64_t beta = 128;
    const uint64_t q = roundbits == 0 ? c->p.q : beta * 2 * (1ull << roundbits);
    hipStream_t s = d.stream;
    uint64_t *ctq = d.sc.lwe[3], *t = d.sc.lwe[4];
    HCHECK(launch_lwe_op(LWE_ADD_CONST, n, mod, beta, ct, nullptr, out, B, s));  // ct1
    HCHECK(launch_lwe_op(LWE_SET_MOD, n, q, 0, out, nullptr, ctq, B, s));
    TvParams tv{};
    tv.mode = TV_HALF;
    tv.ctmod = q;
    tv.fmod = mod;
    SCHECK(dev_bootstrap(c, d, tv, 0, ctq, t, B));
    HCHECK(launch_lwe_op(LWE_SUB, n, mod, 0, out, t, out, B, s));
    HCHECK(launch_lwe_op(LWE_SET_MOD, n, q, 0, out, nullptr, ctq, B, s));
    tv.mode = TV_FLOOR2;
    SCHECK(dev_bootstrap(c, d, tv, 0, ctq, t, B));
    HCHECK(launch_lwe_op(LWE_SUB, n, mod, 0, out, t, out, B, s));
    return TFHE_OK;
}

// vector EvalSign, binfhe-base-scheme.cpp:989-1037 (in: lwe[1] holds the input copy)
tfhe_status dev_sign(tfhe_ctx* c, Device& d, const uint64_t* ct, uint64_t mod, uint64_t* out, size_t B) {
    const uint32_t n = c->p.n;
    const uint64_t beta = 128, q = c->p.q;
    hipStream_t s = d.stream;
    uint64_t *tmp = d.sc.lwe[1], *fl = d.sc.lwe[2];
    HCHECK(hipMemcpyAsync(tmp, ct, B * (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    while (mod > q) {
        SCHECK(dev_floor(c, d, tmp, mod, 0, fl, B));
        const uint64_t nm = mod / q * 2 * beta;
        HCHECK(launch_lwe_op(LWE_MODSWITCH, n, nm, mod, fl, nullptr, tmp, B, s));
        mod = nm;
    }
    HCHECK(launch_lwe_op(LWE_ADD_CONST, n, mod, beta, tmp, nullptr, tmp, B, s));
    TvParams tv{};
    tv.mode = TV_SIGN3;
    tv.ctmod = mod;
    tv.fmod = q;
    SCHECK(dev_bootstrap(c, d, tv, 0, tmp, out, B));
    HCHECK(launch_lwe_op(LWE_SUB_CONST, n, q, q >> 2, out, nullptr, out, B, s));
    return TFHE_OK;
}

// ---------------------------------------------------------------------------
// host-array front ends: shard over devices, chunk to scratch, H2D/D2H
// ---------------------------------------------------------------------------
// One host thread per device, each on a contiguous shard (shard_span).  select(g) makes device g
// current on the calling thread (hipSetDevice; a no-op in tfhe_host_shard_selftest); body(g, lo, cnt)
// queues and waits for that shard.  Every thread's status and thread-local error message is
// collected; the first failing device's is returned as "device g: ...".
template <typename Select, typename Body>
tfhe_status run_shards(size_t D, size_t B, Select&& select, Body&& body) {
    if (D == 1 || B < 2 * D) {
        SCHECK(select(0));
        return body((size_t)0, (size_t)0, B);
    }
    std::vector<tfhe_status> st(D, TFHE_OK);
    std::vector<std::string> msg(D);
    std::vector<std::thread> th;
    for (size_t g = 0; g < D; ++g) {
        size_t lo, cnt;
        shard_span(B, D, g, &lo, &cnt);
        th.emplace_back([&, g, lo, cnt] {
            try {  // an exception must not leave a worker thread (std::terminate)
                st[g] = select(g);
                if (st[g] == TFHE_OK && cnt > 0) st[g] = body(g, lo, cnt);
                if (st[g] != TFHE_OK) msg[g] = g_last_error;  // thread_local: this thread's message
            } catch (const std::exception& e) {
                st[g] = TFHE_ERR_INTERNAL, msg[g] = e.what();
            } catch (...) {
                st[g] = TFHE_ERR_INTERNAL, msg[g] = "unknown exception";
            }
        });
    }
    for (auto& t : th) t.join();
    for (size_t g = 0; g < D; ++g)
        if (st[g] != TFHE_OK) return fail(st[g], "device " + std::to_string(g) + ": " + msg[g]);
    return TFHE_OK;
}

template <typename F>
tfhe_status for_each_shard(tfhe_ctx* c, size_t B, F&& body) {
    return run_shards(
        c->devs.size(), B,
        [&](size_t g) -> tfhe_status {
            HCHECK(hipSetDevice(c->devs[g].id));
            return TFHE_OK;
        },
        [&](size_t g, size_t lo, size_t cnt) { return body(c->devs[g], lo, cnt); });
}

// Host <-> device copies through two pinned 8 MiB blocks: the host copy pool fills (or
// drains) block k+1 while the DMA engine moves block k.  Pageable hipMemcpyAsync stages
// through the runtime's buffers with one host thread; this path is ~2x faster.
tfhe_status ensure_pinned(Device& d) {
    for (int k = 0; k < 2; ++k) {
        if (!d.pin[k]) HCHECK(hipHostMalloc(&d.pin[k], kStageBytes, hipHostMallocDefault));
        if (!d.pin_ev[k]) HCHECK(hipEventCreateWithFlags(&d.pin_ev[k], hipEventDisableTiming));
    }
    return TFHE_OK;
}
// words u64 host -> device through the pinned blocks; wb < 8: the narrow wire format -- the host
// pool narrows each block into pinned memory, the DMA moves wb bytes per word into `pk` (device),
// and one kernel widens pk into dst.  wb is the caller's guess from the array's modulus; a value
// that does not fit (an unreduced input) sends the whole array again as u64.
tfhe_status h2d_staged(Device& d, uint64_t* dst, const HostIn& src, size_t words, hipStream_t s, int wb = 8,
                       void* pk = nullptr) {
    SCHECK(ensure_pinned(d));
    const size_t per = kStageBytes / wb;  // words per block
    uint64_t seen = 0;
    for (size_t off = 0, k = 0; off < words; off += per, ++k) {
        const int slot = (int)(k & 1);
        const size_t nw = std::min(per, words - off);
        HCHECK(hipEventSynchronize(d.pin_ev[slot]));  // the DMA that last read this block is done
        if (wb == 8) {
            parallel_memcpy_in((uint64_t*)d.pin[slot], src, off, nw);
            HCHECK(hipMemcpyAsync(dst + off, d.pin[slot], nw * 8, hipMemcpyHostToDevice, s));
        } else {
            seen |= parallel_narrow_in(d.pin[slot], src, off, nw, wb);
            HCHECK(hipMemcpyAsync((char*)pk + off * wb, d.pin[slot], nw * wb, hipMemcpyHostToDevice, s));
        }
        HCHECK(hipEventRecord(d.pin_ev[slot], s));
    }
    if (wb == 8) return TFHE_OK;
    if (seen >> (8 * wb)) return h2d_staged(d, dst, src, words, s);
    HCHECK(launch_widen(pk, wb, dst, words, s));
    return TFHE_OK;
}
// words u64 device -> host; wb < 8 (every value below 2^(8 wb)): one kernel narrows src into pk,
// the DMA moves wb bytes per word, the host pool widens each block into dst
tfhe_status d2h_staged(Device& d, const HostOut& dst, const uint64_t* src, size_t words, hipStream_t s, int wb = 8,
                       void* pk = nullptr) {
    SCHECK(ensure_pinned(d));
    if (wb != 8) HCHECK(launch_narrow(src, wb, pk, words, s));
    const char* from = wb == 8 ? (const char*)src : (const char*)pk;
    const size_t per = kStageBytes / wb;
    size_t prev_off = 0, prev_nw = 0;
    for (size_t off = 0, k = 0;; off += per, ++k) {
        const int slot = (int)(k & 1);
        const bool more = off < words;
        const size_t nw = more ? std::min(per, words - off) : 0;
        if (more) {
            HCHECK(hipEventSynchronize(d.pin_ev[slot]));
            HCHECK(hipMemcpyAsync(d.pin[slot], from + off * wb, nw * wb, hipMemcpyDeviceToHost, s));
            HCHECK(hipEventRecord(d.pin_ev[slot], s));
        }
        if (k > 0) {  // drain the previous block while this one is in flight
            const int ps = (int)((k - 1) & 1);
            HCHECK(hipEventSynchronize(d.pin_ev[ps]));
            if (wb == 8) parallel_memcpy_out(dst, prev_off, (const uint64_t*)d.pin[ps], prev_nw);
            else parallel_widen_out(dst, prev_off, d.pin[ps], prev_nw, wb);
        }
        if (!more) break;
        prev_off = off, prev_nw = nw;
    }
    return TFHE_OK;
}

// The host-array EvalAcc's output while its blind rotation still runs.  The launch wrote completion
// flags (BRDone: 4 words per ciphertext, one per wave, stored in pinned host memory after the wave's
// accumulator words reached HBM); workgroups are dispatched in ciphertext order, so the ciphertexts of
// block k finish before most of block k+1's.  For each 8 MiB block the host waits for its flags, the
// DMA copies it (u64, no narrowing kernel: it would have to wait for the whole launch) on the copy
// stream, and the host drains the previous block into dst.  Only the last block or two, which finish
// with the launch's last wave, are exposed after the kernel -- instead of the whole 67 MB.
// The wait never hangs: if the compute stream completes (or fails) with a flag unset, or 120 s pass,
// the call fails.
tfhe_status wait_flags(const uint32_t* flags, size_t lo, size_t hi, hipStream_t cs) {
    const volatile uint32_t* f = flags;
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = lo, polls = 0; i < hi; ++polls) {
        if (f[i] != 0) {
            ++i;
            continue;
        }
        // a miss: pause (the spinning thread shares its core with the host pool draining other blocks,
        // ADVICE r3), yield every 64 misses, check the stream every 1024
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#elif defined(__aarch64__)
        __builtin_arm_yield();
#endif
        if ((polls & 63) == 63) std::this_thread::yield();
        if ((polls & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(cs);
            if (q == hipSuccess) {
                if (f[i] == 0) return fail(TFHE_ERR_INTERNAL, "blind rotation finished without its completion flag");
            } else if (q != hipErrorNotReady) {
                return fail(TFHE_ERR_DEVICE, std::string("blind rotation: ") + hipGetErrorString(q));
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
                return fail(TFHE_ERR_DEVICE, "blind rotation: completion flags not set within 120 s");
        }
    }
    return TFHE_OK;
}

tfhe_status d2h_flagged(Device& d, const HostOut& dst, const uint64_t* src, size_t cts, size_t wpc, hipStream_t xs,
                        hipStream_t cs) {
    SCHECK(ensure_pinned(d));
    const size_t cpb = std::max<size_t>(1, (kStageBytes / 8) / wpc);  // ciphertexts per block
    if (cpb * wpc * 8 > kStageBytes) return fail(TFHE_ERR_UNSUPPORTED, "accumulator larger than a staging block");
    size_t prev_lo = 0, prev_n = 0;
    for (size_t lo = 0, k = 0;; lo += cpb, ++k) {
        const int slot = (int)(k & 1);
        const bool more = lo < cts;
        const size_t n = more ? std::min(cpb, cts - lo) : 0;
        if (more) {
            SCHECK(wait_flags(d.flags, 4 * lo, 4 * (lo + n), cs));
            HCHECK(hipEventSynchronize(d.pin_ev[slot]));
            HCHECK(hipMemcpyAsync(d.pin[slot], src + lo * wpc, n * wpc * 8, hipMemcpyDeviceToHost, xs));
            HCHECK(hipEventRecord(d.pin_ev[slot], xs));
        }
        if (k > 0) {
            const int ps = (int)((k - 1) & 1);
            HCHECK(hipEventSynchronize(d.pin_ev[ps]));
            parallel_memcpy_out(dst, prev_lo * wpc, (const uint64_t*)d.pin[ps], prev_n * wpc);
        }
        if (!more) break;
        prev_lo = lo, prev_n = n;
    }
    return TFHE_OK;
}

tfhe_status ensure_flags(Device& d, size_t words) {
    if (words <= d.flags_words) return TFHE_OK;
    if (d.flags) HCHECK(hipHostFree(d.flags));
    d.flags = nullptr, d.flags_words = 0;
    HCHECK(hipHostMalloc((void**)&d.flags, words * 4, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
    d.flags_words = words;
    return TFHE_OK;
}

// Host-array runner: in-arrays are [B][in_words] (up to 2), out [B][out_words].  Each
// device's shard is cut into sub-batches.  Kernels run in order on the device's compute
// stream (lane-0 scratch); copies run on its copy stream (stream2) into two alternating
// device I/O sets, ordered by events: the kernels of k wait for H2D(k), D2H(k) waits for the
// kernels of k, and H2D(k+2) follows D2H(k) on the copy stream (so it reuses k's I/O set only
// after k's kernels and D2H are done).  The host queues H2D(k+1) and the kernels of k+1
// before it drains D2H(k): the compute stream waits for PCIe only for the first sub-batch's
// input and the last one's output.  op(device, in1, in2, out, count, index of the first
// ciphertext) queues its kernels on d.stream.
// Sub-batches per shard: 1 unless TFHE_HOST_PARTS asks for more.  Measured (STD128 NAND,
// 8192, profiles/r02_host): one sub-batch 45.0 ms, 2: 46.2, 4: 51.5, 8: 59.7 -- the split
// blind rotations (2048 workgroups each: a launch tail apiece), the key switches (~1 ms each at
// any batch) and the runtime's blit kernels for the sub-8 MiB copies, which run beside the
// blind rotation, cost more than the 3.4 ms of PCIe they hide.
size_t host_parts(const tfhe_ctx* c, size_t cnt) {
    const size_t want = (size_t)std::max(1, c->kn.host_parts);  // knob (TFHE_HOST_PARTS)
    return std::min(want, std::max<size_t>(1, cnt / 256));
}

tfhe_status ensure_io_set(Scratch& sc, size_t words, size_t pk_bytes) {
    if (words > sc.io_words) {
        hipFree(sc.io);
        sc.io = nullptr, sc.io_words = 0;
        HCHECK(hipMalloc(&sc.io, words * sizeof(uint64_t)));
        sc.io_words = words;
    }
    if (pk_bytes > sc.pk_bytes) {
        hipFree(sc.pk);
        sc.pk = nullptr, sc.pk_bytes = 0;
        HCHECK(hipMalloc(&sc.pk, pk_bytes));
        sc.pk_bytes = pk_bytes;
    }
    return TFHE_OK;
}

// PCIe wire width of an array: the narrowest of u16 / u32 / u64 that holds every value (inputs:
// the OR of the words; outputs: the op's bound); the wire knob 0 (TFHE_WIRE=0) keeps u64.  The
// completion-flag output of the host-array EvalAcc (d2h_flagged) follows the acc_flags knob.

// Value bounds of the runner's arrays (0: unknown): an array crosses PCIe in the narrowest of u16 /
// u32 / u64 that holds its bound (h2d_staged / d2h_staged).  Inputs are checked as they are packed
// (an unreduced input goes again as u64); outputs must respect their bound (the op's modulus).
struct WireLim {
    uint64_t in1 = 0, in2 = 0, out_in = 0, out = 0;
};

// out_in: the output rows' initial contents (uploaded into the output set before the kernels of
// their sub-batch, for ops that work in place on the output, e.g. the blind rotation).
// Arrays are HostRows views (flat or row pointers); w1 / w2 / wo are their record widths.
template <typename Op>
tfhe_status run_lwe_batch_v(tfhe_ctx* c, size_t B, const HostIn& in1, const HostIn& in2, const HostOut& out, Op&& op,
                            WireLim wl, const HostIn& out_in, bool flag_out = false) {
    const size_t w1 = in1.w, w2 = in2.empty() ? 0 : in2.w, wo = out.w;
    const bool has2 = !in2.empty(), has_oi = !out_in.empty();
    return for_each_shard(c, B, [&](Device& d, size_t lo, size_t cnt) -> tfhe_status {
        const size_t parts = host_parts(c, cnt);
        const size_t sub = std::min((cnt + parts - 1) / parts, c->max_chunk);
        const size_t w_in2 = has2 ? w2 : 0, io_words = sub * (w1 + w_in2 + wo);
        const bool nar = c->kn.wire != 0;
        auto width = [nar](uint64_t lim) { return nar && lim ? wire_bytes(lim - 1) : 8; };
        const int wb1 = width(wl.in1), wb2 = has2 ? width(wl.in2) : 8, wbi = has_oi ? width(wl.out_in) : 8;
        const int wbo = width(wl.out);
        const size_t pk1 = sub * w1 * wb1, pk2 = sub * w_in2 * wb2, pko = sub * wo * std::max(wbi, wbo);
        SCHECK(ensure_scratch(c, d, sub));
        SCHECK(ensure_io_set(d.sc, io_words, pk1 + pk2 + pko));
        SCHECK(ensure_io_set(d.sc2, io_words, pk1 + pk2 + pko));
        for (hipEvent_t* e : {&d.h2d_ev[0], &d.h2d_ev[1], &d.k_ev[0], &d.k_ev[1]})
            if (!*e) HCHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        SCHECK(sc_acquire(d, d.stream));
        const hipStream_t cs = d.stream, xs = d.stream2;
        uint64_t* io[2] = {d.sc.io, d.sc2.io};
        char* pk[2] = {(char*)d.sc.pk, (char*)d.sc2.pk};
        const bool trace = c->kn.trace != 0;
        auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
        const double t0 = trace ? now() : 0;
        auto dout_of = [&](int set) { return io[set] + sub * (w1 + w_in2); };
        // D2H of sub-batch k (set k & 1): after its kernels, drained into `out` by the host
        auto d2h = [&](size_t k) -> tfhe_status {
            const size_t off = lo + k * sub, b = std::min(sub, lo + cnt - off);
            const int set = (int)(k & 1);
            HCHECK(hipStreamWaitEvent(xs, d.k_ev[set], 0));
            return d2h_staged(d, out.sub(off), dout_of(set), b * wo, xs, wbo, pk[set] + pk1 + pk2);
        };
        tfhe_status st = TFHE_OK;
        bool done_out = false;  // the flagged path drained the output already
        const size_t n_sub = (cnt + sub - 1) / sub;
        for (size_t k = 0; k < n_sub && st == TFHE_OK; ++k) {
            const size_t off = lo + k * sub, b = std::min(sub, lo + cnt - off);
            const int set = (int)(k & 1);
            uint64_t *din1 = io[set], *din2 = has2 ? io[set] + sub * w1 : nullptr, *dout = dout_of(set);
            st = h2d_staged(d, din1, in1.sub(off), b * w1, xs, wb1, pk[set]);
            if (trace) std::fprintf(stderr, "[tfhe] sub-batch %zu input 1 (%s) staged at %.2f ms\n", k,
                                    in1.flat ? "flat" : "rows", now() - t0);
            if (st == TFHE_OK && has2) st = h2d_staged(d, din2, in2.sub(off), b * w2, xs, wb2, pk[set] + pk1);
            if (st == TFHE_OK && has_oi)
                st = h2d_staged(d, dout, out_in.sub(off), b * wo, xs, wbi, pk[set] + pk1 + pk2);
            if (st != TFHE_OK) break;
            if (trace) std::fprintf(stderr, "[tfhe] sub-batch %zu inputs staged at %.2f ms (wire %d/%d/%d/%d B)\n", k,
                                    now() - t0, wb1, wb2, wbi, wbo);
            // no early return below this point: both streams are synchronised before returning
            if (hipEventRecord(d.h2d_ev[set], xs) != hipSuccess || hipStreamWaitEvent(cs, d.h2d_ev[set], 0) != hipSuccess) {
                st = fail(TFHE_ERR_DEVICE, "host batch: event ordering failed");
                break;
            }
            // flag_out (EvalAcc): one sub-batch lets its blind rotation flag finished ciphertexts
            const bool flagged = flag_out && n_sub == 1 && c->kn.acc_flags != 0;
            if (flagged) {
                st = ensure_flags(d, 4 * b);
                if (st != TFHE_OK) break;
                std::memset(d.flags, 0, 4 * b * sizeof(uint32_t));  // no kernel of an earlier call is left
                d.br_done = BRDone{};
                d.br_done.flags = d.flags;
            }
            st = op(d, din1, din2, dout, b, off);
            const bool written = flagged && d.br_done.written;
            d.br_done = BRDone{};
            if (st != TFHE_OK) break;
            if (written) {  // the blind rotation was the op's last kernel: drain while it runs
                if (trace) std::fprintf(stderr, "[tfhe] sub-batch %zu queued at %.2f ms (flagged output)\n", k, now() - t0);
                st = d2h_flagged(d, out.sub(off), dout, b, wo, xs, cs);
                if (trace) std::fprintf(stderr, "[tfhe] flagged output drained at %.2f ms\n", now() - t0);
                if (st != TFHE_OK) break;
                done_out = true;
                continue;
            }
            if (hipEventRecord(d.k_ev[set], cs) != hipSuccess) {
                st = fail(TFHE_ERR_DEVICE, "host batch: event record failed");
                break;
            }
            if (trace) std::fprintf(stderr, "[tfhe] sub-batch %zu queued at %.2f ms\n", k, now() - t0);
            if (k > 0) st = d2h(k - 1);
        }
        if (st == TFHE_OK && n_sub > 0 && !done_out) {
            if (trace) {
                HCHECK(hipStreamSynchronize(cs));
                std::fprintf(stderr, "[tfhe] last sub-batch's kernels done at %.2f ms\n", now() - t0);
            }
            st = d2h(n_sub - 1);
        }
        const hipError_t e1 = hipStreamSynchronize(cs), e2 = hipStreamSynchronize(xs);
        if (trace) std::fprintf(stderr, "[tfhe] host batch %zu in %zu sub-batches: done %.2f ms\n", cnt, n_sub, now() - t0);
        if (st == TFHE_OK && (e1 != hipSuccess || e2 != hipSuccess))
            st = fail(TFHE_ERR_DEVICE, std::string("host batch: ") + hipGetErrorString(e1 != hipSuccess ? e1 : e2));
        return st;
    });
}

// flat [B][w] arrays
template <typename Op>
tfhe_status run_lwe_batch(tfhe_ctx* c, size_t B, const uint64_t* in1, size_t w1, const uint64_t* in2, size_t w2,
                          uint64_t* out, size_t wo, Op&& op, WireLim wl, const uint64_t* out_in = nullptr,
                          bool flag_out = false) {
    return run_lwe_batch_v(c, B, flat_rows(in1, w1), in2 ? flat_rows(in2, w2) : HostIn{}, flat_rows(out, wo),
                           std::forward<Op>(op), wl, out_in ? flat_rows(out_in, wo) : HostIn{}, flag_out);
}

tfhe_status check_ctx(tfhe_ctx* c) {
    if (!c || c->devs.empty()) return fail(TFHE_ERR_NOT_SET_UP, "context not set up (call tfhe_setup)");
    return TFHE_OK;
}

tfhe_status create_ctx(const tfhe_params* p, int num_gpus, std::unique_ptr<tfhe_ctx>& out) {
    if (!p) return fail(TFHE_ERR_INVALID_ARGUMENT, "null params");
    auto c = std::make_unique<tfhe_ctx>();
    c->p = *p;
    std::string err;
    if (params_finish(&c->p, &err) != TFHE_OK) return fail(TFHE_ERR_INVALID_ARGUMENT, err);
    SCHECK(init_derived(c.get()));
    int count = 0;
    HCHECK(hipGetDeviceCount(&count));
    if (count < 1) return fail(TFHE_ERR_DEVICE, "no HIP device visible");
    // Test hook: TFHE_LOGICAL_DEVICES=k presents k logical devices, all on physical device 0, each
    // with its own arena, streams, scratch and host thread -- the multi-device setup, replication
    // (peer copies: one RCCL communicator cannot hold a device twice), sharding and error paths
    // run on a one-GPU box (tests/test_gpu_multidevice.py).  Read per setup.
    if (const char* rl = std::getenv("TFHE_RCCL_LIB")) c->rccl_lib = rl;
    const char* lg = std::getenv("TFHE_LOGICAL_DEVICES");
    const int logical = lg ? std::atoi(lg) : 0;
    if (logical > 1) count = logical;
    // GPUSetup(numGPUs): numGPUs <= 0 or more than visible uses every visible device
    // (bootstrapping.cu:736-739)
    if (num_gpus < 1 || num_gpus > count) num_gpus = count;
    c->devs.resize(num_gpus);
    for (int g = 0; g < num_gpus; ++g) c->devs[g].id = logical > 1 ? 0 : g;
    out = std::move(c);
    return TFHE_OK;
}

}  // namespace

tfhe_ctx::~tfhe_ctx() {
    for (auto& d : devs) free_device(d);
}

namespace {
// Every extern "C" body runs under this: no C++ exception crosses the C-ABI.
template <typename F>
tfhe_status guarded(F&& body) {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return fail(TFHE_ERR_OUT_OF_MEMORY, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(TFHE_ERR_INTERNAL, std::string("internal error: ") + e.what());
    } catch (...) {
        return fail(TFHE_ERR_INTERNAL, "internal error");
    }
}
}  // namespace

// ===========================================================================
// extern "C" entry points
// ===========================================================================
extern "C" {

int tfhe_abi_version(void) { return TFHE_HIP_ABI_VERSION; }

tfhe_status tfhe_set_kernel_variant(int variant) {
    if (!set_fast_variant(variant)) return fail(TFHE_ERR_INVALID_ARGUMENT, "unknown kernel variant");
    return TFHE_OK;
}
int tfhe_get_kernel_variant(void) { return get_fast_variant(); }

const char* tfhe_last_error(void) { return g_last_error.c_str(); }

const char* tfhe_status_string(tfhe_status s) {
    switch (s) {
        case TFHE_OK: return "ok";
        case TFHE_ERR_INVALID_ARGUMENT: return "invalid argument";
        case TFHE_ERR_UNSUPPORTED: return "unsupported";
        case TFHE_ERR_NOT_SET_UP: return "not set up";
        case TFHE_ERR_DEVICE: return "device error";
        case TFHE_ERR_OUT_OF_MEMORY: return "out of memory";
        default: return "internal error";
    }
}

tfhe_status tfhe_params_from_set(int paramset, tfhe_params* out) {
    return guarded([&]() -> tfhe_status {
        if (!out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null output");
        tfhe_status s = params_from_set(paramset, out);
        if (s != TFHE_OK) return fail(s, "unknown parameter set");
        return TFHE_OK;
    });
}

tfhe_status tfhe_params_from_logq(int paramset, int arb_func, uint32_t logQ, int64_t N, uint32_t baseG,
                                  uint32_t num_digits_to_throw, tfhe_params* out) {
    return guarded([&]() -> tfhe_status {
        if (!out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null output");
        tfhe_status s = params_from_logq(paramset, arb_func, logQ, N, baseG, num_digits_to_throw, out);
        if (s != TFHE_OK) return fail(s, "unsupported logQ parameter request (STD128/TOY, 11 <= logQ <= 29)");
        return TFHE_OK;
    });
}

tfhe_status tfhe_params_finish(tfhe_params* p) {
    return guarded([&]() -> tfhe_status {
        if (!p) return fail(TFHE_ERR_INVALID_ARGUMENT, "null params");
        std::string err;
        tfhe_status s = params_finish(p, &err);
        return s == TFHE_OK ? s : fail(s, err);
    });
}

extern "C++" {  // (a C++ return type: no C linkage inside the extern "C" block)
namespace {
// RCCL, loaded when a context spans several devices (no link-time dependency for one-GPU use)
struct RcclApi {
    bool ok = false;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclBroadcast) bcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    decltype(&ncclGetVersion) version = nullptr;  // optional (reported by tfhe_rccl_selftest)
};
// path: "" = the system RCCL (librccl.so.1); otherwise TFHE_RCCL_LIB, read at setup -- a test build of the
// same six entry points (tests/stub_rccl: broadcasts by device copies, so the group / sync / destroy
// sequence below runs on a one-GPU box with logical devices).  Loaded once per path.
const RcclApi& rccl(const std::string& path) {
    static std::mutex mu;
    static std::vector<std::pair<std::string, std::unique_ptr<RcclApi>>> loaded;
    std::lock_guard<std::mutex> lock(mu);
    for (auto& e : loaded)
        if (e.first == path) return *e.second;
    loaded.emplace_back(path, std::make_unique<RcclApi>([&] {
        RcclApi a;
        void* h = path.empty() ? dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL) : dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h && path.empty()) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return a;
        a.init_all = (decltype(a.init_all))dlsym(h, "ncclCommInitAll");
        a.bcast = (decltype(a.bcast))dlsym(h, "ncclBroadcast");
        a.group_start = (decltype(a.group_start))dlsym(h, "ncclGroupStart");
        a.group_end = (decltype(a.group_end))dlsym(h, "ncclGroupEnd");
        a.destroy = (decltype(a.destroy))dlsym(h, "ncclCommDestroy");
        a.err = (decltype(a.err))dlsym(h, "ncclGetErrorString");
        a.version = (decltype(a.version))dlsym(h, "ncclGetVersion");
        a.ok = a.init_all && a.bcast && a.group_start && a.group_end && a.destroy && a.err;
        return a;
    }()));
    return *loaded.back().second;
}

// Sum of the checksum partials of `bytes` at p on device `dev` (stream synchronised)
tfhe_status buffer_checksum(int dev, const void* p, size_t bytes, hipStream_t stream, uint64_t& out) {
    DevBuf part;
    HCHECK(hipSetDevice(dev));
    HCHECK(hipMalloc(&part.p, kChecksumBlocks * sizeof(uint64_t)));
    HCHECK(launch_checksum(p, bytes, part.as<uint64_t>(), stream));
    std::vector<uint64_t> h(kChecksumBlocks);
    HCHECK(hipMemcpyAsync(h.data(), part.p, h.size() * 8, hipMemcpyDeviceToHost, stream));
    HCHECK(hipStreamSynchronize(stream));
    out = 0;
    for (uint64_t v : h) out += v;
    return TFHE_OK;
}
tfhe_status arena_checksum(Device& d, size_t bytes, uint64_t& out) {
    return buffer_checksum(d.id, d.arena, bytes, d.stream, out);
}

// One RCCL broadcast of `bytes` at src (on t[0]'s device) into every target buffer: a communicator over the
// targets' devices (ncclCommInitAll), one ncclBroadcast per rank inside a group, every stream synchronised,
// the communicators destroyed.  True when every call succeeded.  The sequence of replicate_arena, and the
// one tfhe_rccl_selftest runs against the real librccl on a one-GPU box (a one-rank communicator).
struct RcclTarget {
    int device;
    void* dst;
    hipStream_t stream;
};
bool rccl_broadcast(const RcclApi& R, const void* src, size_t bytes, const std::vector<RcclTarget>& t) {
    const size_t D = t.size();
    std::vector<ncclComm_t> comms(D);
    std::vector<int> ids(D);
    for (size_t g = 0; g < D; ++g) ids[g] = t[g].device;
    if (R.init_all(comms.data(), (int)D, ids.data()) != ncclSuccess) return false;
    ncclResult_t r = R.group_start();
    for (size_t g = 0; g < D && r == ncclSuccess; ++g)  // no early return inside the group
        r = hipSetDevice(t[g].device) == hipSuccess ? R.bcast(src, t[g].dst, bytes, ncclUint8, 0, comms[g], t[g].stream)
                                                    : ncclUnhandledCudaError;
    const ncclResult_t r2 = R.group_end();
    bool synced = r == ncclSuccess && r2 == ncclSuccess;
    for (size_t g = 0; g < D; ++g) {
        hipSetDevice(t[g].device);
        synced = hipStreamSynchronize(t[g].stream) == hipSuccess && synced;
    }
    for (auto& cm : comms) R.destroy(cm);
    return synced;
}

// Device 0's image -> devices 1..D-1.  GPUSetup(numGPUs) in the reference copies every key from the
// host to each GPU in turn (bootstrapping.cu:1005-1069); here the image crosses PCIe once and is
// broadcast by RCCL over xGMI (one communicator over the context's devices, one ncclBroadcast per
// device in a group), or -- without librccl, or with TFHE_REPLICATE=peer -- copied from device 0 by
// concurrent peer DMAs.  Every device's copy is complete when this returns.
tfhe_status replicate_arena(tfhe_ctx* c, size_t bytes) {
    const size_t D = c->devs.size();
    if (D < 2) return TFHE_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const char* env = std::getenv("TFHE_REPLICATE");
    bool want_rccl = !(env && std::strcmp(env, "peer") == 0);
    // logical devices sharing one GPU (TFHE_LOGICAL_DEVICES): a real communicator cannot hold a device
    // twice; a TFHE_RCCL_LIB test build can (tests/test_gpu_rccl_stub.py)
    for (size_t g = 1; g < D; ++g)
        if (c->devs[g].id == c->devs[0].id && c->rccl_lib.empty()) want_rccl = false;
    bool done = false;
    if (want_rccl && rccl(c->rccl_lib).ok) {
        std::vector<RcclTarget> t(D);
        for (size_t g = 0; g < D; ++g) t[g] = RcclTarget{c->devs[g].id, c->devs[g].arena, c->devs[g].stream};
        done = rccl_broadcast(rccl(c->rccl_lib), c->devs[0].arena, bytes, t);
    }
    if (!done) {
        for (size_t g = 1; g < D; ++g) {
            Device& d = c->devs[g];
            HCHECK(hipSetDevice(d.id));
            HCHECK(hipMemcpyPeerAsync(d.arena, d.id, c->devs[0].arena, c->devs[0].id, bytes, d.stream));
        }
        for (size_t g = 1; g < D; ++g) {
            HCHECK(hipSetDevice(c->devs[g].id));
            HCHECK(hipStreamSynchronize(c->devs[g].stream));
        }
    }
    c->replicate_method = done ? TFHE_REPLICATE_RCCL : TFHE_REPLICATE_PEER;
    c->replicate_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    // every replica must equal device 0's image: a bad broadcast fails setup, not a later call
    uint64_t want = 0, got = 0;
    SCHECK(arena_checksum(c->devs[0], bytes, want));
    for (size_t g = 1; g < D; ++g) {
        SCHECK(arena_checksum(c->devs[g], bytes, got));
        if (got != want)
            return fail(TFHE_ERR_DEVICE, "key arena replica on device " + std::to_string(g) + " differs from device 0's (" +
                                             (done ? "RCCL broadcast" : "peer copy") + ")");
    }
    return TFHE_OK;
}

tfhe_status setup_common(tfhe_ctx** out, const tfhe_params* p, const uint64_t* bsk_coeff, bool bsk_eval,
                         const uint64_t* ksk, int num_gpus) {
    if (!out || !bsk_coeff || !ksk) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    std::unique_ptr<tfhe_ctx> c;
    SCHECK(create_ctx(p, num_gpus, c));
    std::vector<unsigned char> img;
    SCHECK(build_host_image(c.get(), bsk_coeff, bsk_eval, ksk, img));
    const size_t bytes = c->layout.total;
    for (size_t g = 0; g < c->devs.size(); ++g) {
        Device& d = c->devs[g];
        HCHECK(hipSetDevice(d.id));
        SCHECK(create_streams(d));
        HCHECK(hipMalloc(&d.arena, bytes));
    }
    HCHECK(hipSetDevice(c->devs[0].id));
    HCHECK(hipMemcpy(c->devs[0].arena, img.data(), bytes, hipMemcpyHostToDevice));
    img = std::vector<unsigned char>();
    SCHECK(replicate_arena(c.get(), bytes));
    // derived key forms, every device at once (each derives its own from its arena)
    SCHECK(run_shards(
        c->devs.size(), 2 * c->devs.size(),
        [&](size_t g) -> tfhe_status {
            HCHECK(hipSetDevice(c->devs[g].id));
            return TFHE_OK;
        },
        [&](size_t g, size_t, size_t) { return finish_device(c.get(), c->devs[g]); }));
    *out = c.release();
    return TFHE_OK;
}
}  // namespace
}  // extern "C++"

/* One-device run of replicate_arena's RCCL sequence against a real librccl (verdict r5 item 4): the stub
 * of tests/stub_rccl restates the API as declared here, so only the real library checks the dlsym table's
 * prototypes, enums and the communicator / group / broadcast / destroy order against the shipped ABI. */
tfhe_status tfhe_rccl_selftest(int device, size_t bytes, const char* lib, int* version) {
    return guarded([&]() -> tfhe_status {
        if (bytes == 0 || bytes % 8) return fail(TFHE_ERR_INVALID_ARGUMENT, "bytes must be a positive multiple of 8");
        if (version) *version = 0;
        const RcclApi& R = rccl(lib ? lib : "");
        if (!R.ok) return fail(TFHE_ERR_UNSUPPORTED, "librccl did not load (or lacks an entry point)");
        if (version && R.version && R.version(version) != ncclSuccess)
            return fail(TFHE_ERR_DEVICE, "ncclGetVersion failed");
        HCHECK(hipSetDevice(device));
        hipStream_t st = nullptr;
        HCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        struct StreamGuard {
            hipStream_t s;
            ~StreamGuard() { hipStreamDestroy(s); }
        } sg{st};
        DevBuf src, dst;
        HCHECK(hipMalloc(&src.p, bytes));
        HCHECK(hipMalloc(&dst.p, bytes));
        std::vector<uint64_t> h(bytes / 8);
        uint64_t x = 0x9E3779B97F4A7C15ull;  // splitmix64 stream
        for (auto& v : h) {
            uint64_t z = (x += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            v = z ^ (z >> 31);
        }
        HCHECK(hipMemcpy(src.p, h.data(), bytes, hipMemcpyHostToDevice));
        HCHECK(hipMemset(dst.p, 0, bytes));
        // one rank, root 0, out of place: the receive buffer gets the send buffer
        if (!rccl_broadcast(R, src.p, bytes, {RcclTarget{device, dst.p, st}}))
            return fail(TFHE_ERR_DEVICE, "RCCL communicator / broadcast failed");
        uint64_t want = 0, got = 0;
        SCHECK(buffer_checksum(device, src.p, bytes, st, want));
        SCHECK(buffer_checksum(device, dst.p, bytes, st, got));
        if (want != got) return fail(TFHE_ERR_DEVICE, "RCCL broadcast delivered a different buffer");
        return TFHE_OK;
    });
}

tfhe_status tfhe_setup(tfhe_ctx** out, const tfhe_params* p, const uint64_t* bsk_coeff, const uint64_t* ksk,
                       int num_gpus) {
    return guarded([&]() -> tfhe_status {
        return setup_common(out, p, bsk_coeff, false, ksk, num_gpus);
    });
}

tfhe_status tfhe_setup_eval(tfhe_ctx** out, const tfhe_params* p, const uint64_t* bsk_eval, const uint64_t* ksk,
                            int num_gpus) {
    return guarded([&]() -> tfhe_status {
        return setup_common(out, p, bsk_eval, true, ksk, num_gpus);
    });
}

tfhe_status tfhe_setup_from_key_image(tfhe_ctx** out, const tfhe_params* p, const void* d_src, size_t bytes,
                                      int device) {
    return guarded([&]() -> tfhe_status {
        if (!out || !d_src) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        *out = nullptr;
        std::unique_ptr<tfhe_ctx> c;
        SCHECK(create_ctx(p, 1, c));
        if (bytes != c->layout.total) return fail(TFHE_ERR_INVALID_ARGUMENT, "key image size mismatch");
        Device& d = c->devs[0];
        d.id = device;
        HCHECK(hipSetDevice(device));
        SCHECK(create_streams(d));
        HCHECK(hipMalloc(&d.arena, bytes));
        HCHECK(hipMemcpy(d.arena, d_src, bytes, hipMemcpyDeviceToDevice));
        SCHECK(finish_device(c.get(), d));
        *out = c.release();
        return TFHE_OK;
    });
}

namespace {
struct KeyFileHeader {
    char magic[8];  // "TFHEKIMG"
    uint32_t abi;
    uint32_t reserved;
    tfhe_params params;
    uint64_t bytes;
    uint64_t fnv;
};
uint64_t fnv1a64(const unsigned char* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}
}  // namespace

tfhe_status tfhe_save_key_image(tfhe_ctx* c, const char* path) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (!path) return fail(TFHE_ERR_INVALID_ARGUMENT, "null path");
        std::vector<unsigned char> img(c->layout.total);
        HCHECK(hipSetDevice(c->devs[0].id));
        HCHECK(hipStreamSynchronize(c->devs[0].stream));
        HCHECK(hipMemcpy(img.data(), c->devs[0].arena, img.size(), hipMemcpyDeviceToHost));
        KeyFileHeader hdr{};
        std::memcpy(hdr.magic, "TFHEKIMG", 8);
        hdr.abi = (uint32_t)tfhe_abi_version();
        hdr.params = c->p;
        hdr.bytes = img.size();
        hdr.fnv = fnv1a64(img.data(), img.size());
        FILE* f = std::fopen(path, "wb");
        if (!f) return fail(TFHE_ERR_INVALID_ARGUMENT, std::string("cannot open ") + path);
        const bool ok = std::fwrite(&hdr, sizeof(hdr), 1, f) == 1 && std::fwrite(img.data(), 1, img.size(), f) == img.size();
        if (std::fclose(f) != 0 || !ok) return fail(TFHE_ERR_INVALID_ARGUMENT, std::string("write failed: ") + path);
        return TFHE_OK;
    });
}

tfhe_status tfhe_setup_from_key_file(tfhe_ctx** out, const tfhe_params* p, const char* path, int device) {
    return guarded([&]() -> tfhe_status {
        if (!out || !p || !path) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        *out = nullptr;
        tfhe_params want = *p;
        std::string err;
        if (params_finish(&want, &err) != TFHE_OK) return fail(TFHE_ERR_INVALID_ARGUMENT, err);
        FILE* f = std::fopen(path, "rb");
        if (!f) return fail(TFHE_ERR_INVALID_ARGUMENT, std::string("cannot open ") + path);
        KeyFileHeader hdr{};
        std::vector<unsigned char> img;
        tfhe_status st = TFHE_OK;
        if (std::fread(&hdr, sizeof(hdr), 1, f) != 1 || std::memcmp(hdr.magic, "TFHEKIMG", 8) != 0)
            st = fail(TFHE_ERR_INVALID_ARGUMENT, "not a key image file");
        else if (hdr.abi != (uint32_t)tfhe_abi_version())
            st = fail(TFHE_ERR_INVALID_ARGUMENT, "key image written by another ABI version");
        else if (std::memcmp(&hdr.params, &want, sizeof(want)) != 0)
            st = fail(TFHE_ERR_INVALID_ARGUMENT, "key image parameters differ from the requested ones");
        else if (hdr.bytes != arena_layout(want, word_bits_for(want)).total)  // before any allocation
            st = fail(TFHE_ERR_INVALID_ARGUMENT, "key image size field does not match the parameters");
        else {
            img.resize(hdr.bytes);
            if (std::fread(img.data(), 1, img.size(), f) != img.size())
                st = fail(TFHE_ERR_INVALID_ARGUMENT, "truncated key image file");
            else if (fnv1a64(img.data(), img.size()) != hdr.fnv)
                st = fail(TFHE_ERR_INVALID_ARGUMENT, "key image checksum mismatch");
        }
        std::fclose(f);
        if (st != TFHE_OK) return st;
        std::unique_ptr<tfhe_ctx> c;
        SCHECK(create_ctx(&want, 1, c));
        if (img.size() != c->layout.total) return fail(TFHE_ERR_INVALID_ARGUMENT, "key image size mismatch");
        Device& d = c->devs[0];
        d.id = device;
        HCHECK(hipSetDevice(device));
        SCHECK(create_streams(d));
        HCHECK(hipMalloc(&d.arena, img.size()));
        HCHECK(hipMemcpy(d.arena, img.data(), img.size(), hipMemcpyHostToDevice));
        SCHECK(finish_device(c.get(), d));
        *out = c.release();
        return TFHE_OK;
    });
}

tfhe_status tfhe_export_key_image(tfhe_ctx* c, void* d_dst, size_t bytes, void* stream) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (bytes != c->layout.total) return fail(TFHE_ERR_INVALID_ARGUMENT, "key image size mismatch");
        HCHECK(hipSetDevice(c->devs[0].id));
        hipStream_t s = stream ? (hipStream_t)stream : c->devs[0].stream;
        HCHECK(hipMemcpyAsync(d_dst, c->devs[0].arena, bytes, hipMemcpyDeviceToDevice, s));
        HCHECK(hipStreamSynchronize(s));
        return TFHE_OK;
    });
}

tfhe_status tfhe_clean(tfhe_ctx* c) {
    delete c;  // ~tfhe_ctx frees every device
    return TFHE_OK;
}

tfhe_status tfhe_get_info(tfhe_ctx* c, tfhe_info* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (!out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null output");
        out->num_devices = (int)c->devs.size();
        out->word_bits = c->word_bits;
        out->bsk_device_bytes = c->layout.ksk - c->layout.bsk + (c->use_fast ? bsk_fast_bytes(c->br) : 0) +
                                (c->use_f64 ? bsk_f64_bytes(c->br) : 0) +
                                (c->use_sf ? sf_bytes(c->br) : 0);
        out->ksk_device_bytes = c->layout.total - c->layout.ksk;
        out->bootstraps = c->bootstraps.load();
        out->key_image_bytes = c->layout.total;
        out->br_kernel = c->use_fast  ? TFHE_BR_FAST
                         : c->use_f64 ? (c->f64_fold ? TFHE_BR_F64_FOLD : TFHE_BR_F64)
                         : c->use_sf  ? TFHE_BR_SF
                                      : TFHE_BR_GENERIC;
        out->replicate_method = c->replicate_method;
        out->replicate_ms = c->replicate_ms;
        out->duo_timeouts = 0;
        for (Device& d : c->devs) {
            if (!d.duo.base) continue;
            uint32_t e = 0;
            HCHECK(hipSetDevice(d.id));
            HCHECK(hipStreamSynchronize(d.stream));
            HCHECK(hipMemcpy(&e, (const uint32_t*)d.duo.base + duo_err_offset_words(), 4, hipMemcpyDeviceToHost));
            out->duo_timeouts += e;
        }
        return TFHE_OK;
    });
}

static_assert(sizeof(tfhe_knobs) == sizeof(Knobs), "tfhe_knobs mirrors tfhe::Knobs field by field");

tfhe_status tfhe_get_knobs(tfhe_ctx* c, tfhe_knobs* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (!out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null output");
        std::memcpy(out, &c->kn, sizeof(Knobs));
        return TFHE_OK;
    });
}

tfhe_status tfhe_set_knobs(tfhe_ctx* c, const tfhe_knobs* in) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (!in) return fail(TFHE_ERR_INVALID_ARGUMENT, "null knobs");
        Knobs k;
        std::memcpy(&k, in, sizeof(Knobs));
        if (const char* why = knob_out_of_range(k)) return fail(TFHE_ERR_INVALID_ARGUMENT, std::string("knob out of range: ") + why);
        if (k.probe != 0 && !f64_test_probes_compiled())
            return fail(TFHE_ERR_UNSUPPORTED, "probe builds exist only in the test library (libtfhe_hip_test.so)");
        c->kn = k;
        return TFHE_OK;
    });
}

tfhe_status tfhe_shard_range(size_t total, int world, int rank, size_t* lo, size_t* hi) {
    if (world < 1 || rank < 0 || rank >= world || !lo || !hi) return fail(TFHE_ERR_INVALID_ARGUMENT, "bad world/rank");
    size_t l, cnt;
    shard_span(total, (size_t)world, (size_t)rank, &l, &cnt);
    *lo = l, *hi = l + cnt;
    return TFHE_OK;
}

tfhe_status tfhe_host_shard_selftest(size_t B, int devices, int fail_device, size_t* spans) {
    return guarded([&]() -> tfhe_status {
        if (devices < 1 || !spans) return fail(TFHE_ERR_INVALID_ARGUMENT, "bad arguments");
        for (int g = 0; g < devices; ++g) spans[2 * g] = spans[2 * g + 1] = 0;
        return run_shards(
            (size_t)devices, B, [](size_t) { return TFHE_OK; },
            [&](size_t g, size_t lo, size_t cnt) -> tfhe_status {
                spans[2 * g] = lo, spans[2 * g + 1] = cnt;
                if ((int)g == fail_device) return fail(TFHE_ERR_DEVICE, "injected fault on shard [" + std::to_string(lo) +
                                                                            ", " + std::to_string(lo + cnt) + ")");
                return TFHE_OK;
            });
    });
}

tfhe_status tfhe_eval_acc(tfhe_ctx* c, size_t B, const uint64_t* a, uint64_t a_mod, uint64_t* acc) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!a || !acc) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const tfhe_params& p = c->p;
        const size_t wacc = 2 * (size_t)p.N;
        // the accumulators go straight into the output set and are rotated there
        return run_lwe_batch(
            c, B, a, p.n, nullptr, 0, acc, wacc,
            [&](Device& d, const uint64_t* i1, const uint64_t*, uint64_t* o, size_t b, size_t) {
                return dev_blind_rotate(c, d, i1, a_mod, o, b);
            },
            WireLim{a_mod, 0, p.Q, p.Q}, acc, true);
    });
}

tfhe_status tfhe_eval_acc_tv(tfhe_ctx* c, size_t B, const uint64_t* a, uint64_t a_mod, const uint64_t* tv,
                             uint32_t tv_len, uint64_t* acc) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!a || !tv || !acc) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const tfhe_params& p = c->p;
        if (tv_len == 0 || tv_len > p.N || p.N % tv_len != 0)
            return fail(TFHE_ERR_INVALID_ARGUMENT, "test-vector length must divide N");
        return run_lwe_batch(c, B, a, p.n, tv, tv_len, acc, 2 * (size_t)p.N,
                             [&](Device& d, const uint64_t* i1, const uint64_t* i2, uint64_t* o, size_t b, size_t) {
                                 HCHECK(launch_expand_tv(p.N, tv_len, i2, o, b, d.stream));
                                 return dev_blind_rotate(c, d, i1, a_mod, o, b);
                             },
                             WireLim{a_mod, p.Q, 0, p.Q}, nullptr, true);
    });
}

tfhe_status tfhe_eval_acc_tv_rows(tfhe_ctx* c, size_t B, const uint64_t* const* a_rows, uint64_t a_mod,
                                  const uint64_t* tv, uint32_t tv_len, uint64_t* const* acc_rows) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!a_rows || !tv || !acc_rows) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const tfhe_params& p = c->p;
        if (tv_len == 0 || tv_len > p.N || p.N % tv_len != 0)
            return fail(TFHE_ERR_INVALID_ARGUMENT, "test-vector length must divide N");
        for (size_t s = 0; s < B; ++s)
            if (!a_rows[s] || !acc_rows[2 * s] || !acc_rows[2 * s + 1])
                return fail(TFHE_ERR_INVALID_ARGUMENT, "null row pointer");
        return run_lwe_batch_v(c, B, ptr_rows(a_rows, 1, p.n, (const uint64_t*)nullptr), flat_rows(tv, tv_len),
                               ptr_rows(acc_rows, 2, p.N, (uint64_t*)nullptr),
                               [&](Device& d, const uint64_t* i1, const uint64_t* i2, uint64_t* o, size_t b, size_t) {
                                   HCHECK(launch_expand_tv(p.N, tv_len, i2, o, b, d.stream));
                                   return dev_blind_rotate(c, d, i1, a_mod, o, b);
                               },
                               WireLim{a_mod, p.Q, 0, p.Q}, HostIn{}, true);
    });
}

tfhe_status tfhe_eval_acc_device(tfhe_ctx* c, size_t B, const uint64_t* d_a, uint64_t a_mod, uint64_t* d_acc,
                                 void* stream) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!d_a || !d_acc) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        Device* dp = nullptr;
        SCHECK(device_for(c, d_acc, dp));
        Device& d = *dp;
        HCHECK(hipSetDevice(d.id));
        hipStream_t saved = d.stream;
        if (stream) d.stream = (hipStream_t)stream;
        tfhe_status st = dev_blind_rotate(c, d, d_a, a_mod, d_acc, B);
        d.stream = saved;
        return st;
    });
}

tfhe_status tfhe_mkm_switch(tfhe_ctx* c, size_t B, const uint64_t* ct_ext, uint64_t fmod, uint64_t* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!ct_ext || !out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const tfhe_params& p = c->p;
        return run_lwe_batch(c, B, ct_ext, p.N + 1, nullptr, 0, out, p.n + 1,
                             [&](Device& d, const uint64_t* i1, const uint64_t*, uint64_t* o, size_t b, size_t) {
                                 return dev_mkm(c, d, i1, fmod, o, b);
                             },
                             WireLim{p.Q, 0, 0, fmod});
    });
}

tfhe_status tfhe_mkm_switch_rows(tfhe_ctx* c, size_t B, const uint64_t* const* ext_a_rows, const uint64_t* ext_b,
                                 uint64_t fmod, uint64_t* const* out_a_rows, uint64_t* out_b) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!ext_a_rows || !ext_b || !out_a_rows || !out_b) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        for (size_t s = 0; s < B; ++s)
            if (!ext_a_rows[s] || !out_a_rows[s]) return fail(TFHE_ERR_INVALID_ARGUMENT, "null row pointer");
        const tfhe_params& p = c->p;
        return run_lwe_batch_v(c, B, ptr_rows(ext_a_rows, 1, p.N, ext_b), HostIn{},
                               ptr_rows(out_a_rows, 1, p.n, out_b),
                               [&](Device& d, const uint64_t* i1, const uint64_t*, uint64_t* o, size_t b, size_t) {
                                   return dev_mkm(c, d, i1, fmod, o, b);
                               },
                               WireLim{p.Q, 0, 0, fmod}, HostIn{});
    });
}

tfhe_status tfhe_mkm_switch_device(tfhe_ctx* c, size_t B, const uint64_t* d_ct_ext, uint64_t fmod, uint64_t* d_out,
                                   void* stream) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!d_ct_ext || !d_out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        Device* dp = nullptr;
        SCHECK(device_for(c, d_out, dp));
        Device& d = *dp;
        HCHECK(hipSetDevice(d.id));
        SCHECK(ensure_ks_scratch(c, d, B));
        hipStream_t saved = d.stream;
        if (stream) d.stream = (hipStream_t)stream;
        tfhe_status st = sc_acquire(d, d.stream);
        if (st == TFHE_OK) st = dev_mkm(c, d, d_ct_ext, fmod, d_out, B);
        const tfhe_status rel = sc_release(d, d.stream);
        d.stream = saved;
        return st != TFHE_OK ? st : rel;
    });
}

tfhe_status tfhe_eval_bin_gate(tfhe_ctx* c, int gate, size_t B, const uint64_t* ct1, const uint64_t* ct2, uint64_t q,
                               uint64_t* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "EvalBinGate: input vector is empty");
        if (!ct1 || !ct2 || !out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        if (ct1 == ct2) return fail(TFHE_ERR_INVALID_ARGUMENT, "Input ciphertexts should be independant");
        if (gate < TFHE_OR || gate > TFHE_XNOR) return fail(TFHE_ERR_INVALID_ARGUMENT, "unknown gate");
        const size_t w = c->p.n + 1;
        return run_lwe_batch(c, B, ct1, w, ct2, w, out, w,
                             [&](Device& d, const uint64_t* i1, const uint64_t* i2, uint64_t* o, size_t b, size_t) {
                                 return dev_gate(c, d, gate, i1, i2, q, o, b);
                             },
                             WireLim{q, q, 0, q});
    });
}

extern "C++" {  // (templates need C++ linkage inside the extern "C" block)
namespace {
// Frame of the device-resident fused ops: the device holding d_out, scratch for B ciphertexts, the
// caller's stream (ordered after every earlier user of the device's scratch, sc_fence).
template <typename F>
tfhe_status run_device_op(tfhe_ctx* c, size_t B, const void* d_out, void* stream, F&& body) {
    Device* dp = nullptr;
    SCHECK(device_for(c, d_out, dp));
    Device& d = *dp;
    HCHECK(hipSetDevice(d.id));
    SCHECK(ensure_scratch(c, d, B));
    hipStream_t saved = d.stream;
    if (stream) d.stream = (hipStream_t)stream;
    tfhe_status st = sc_acquire(d, d.stream);
    if (st == TFHE_OK) st = body(d);
    const tfhe_status rel = sc_release(d, d.stream);  // even after a failed launch: later users wait on it
    d.stream = saved;
    return st != TFHE_OK ? st : rel;
}
}  // namespace
}  // extern "C++"

tfhe_status tfhe_eval_bin_gate_device(tfhe_ctx* c, int gate, size_t B, const uint64_t* d_ct1, const uint64_t* d_ct2,
                                      uint64_t q, uint64_t* d_out, void* stream) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (gate < TFHE_OR || gate > TFHE_XNOR) return fail(TFHE_ERR_INVALID_ARGUMENT, "unknown gate");
        if (B == 0) return TFHE_OK;
        if (!d_ct1 || !d_ct2 || !d_out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        return run_device_op(c, B, d_out, stream,
                             [&](Device& d) { return dev_gate(c, d, gate, d_ct1, d_ct2, q, d_out, B); });
    });
}

tfhe_status tfhe_eval_func_device(tfhe_ctx* c, size_t B, const uint64_t* d_ct, uint64_t q, const uint64_t* d_lut,
                                  int per_ct_lut, uint64_t* d_out, void* stream) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!d_ct || !d_lut || !d_out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        if (q < 4 || (2ull * c->p.N) % q) return fail(TFHE_ERR_INVALID_ARGUMENT, "q must divide 2N");
        // the first LUT classifies the batch (binfhe-base-scheme.cpp:697-698): q words to the host
        std::vector<uint64_t> lut0(q);
        hipStream_t s = stream ? (hipStream_t)stream : nullptr;
        {
            Device* dp = nullptr;
            SCHECK(device_for(c, d_out, dp));
            HCHECK(hipSetDevice(dp->id));
            if (!s) s = dp->stream;
            HCHECK(hipMemcpyAsync(lut0.data(), d_lut, q * 8, hipMemcpyDeviceToHost, s));
            HCHECK(hipStreamSynchronize(s));
        }
        const int prop = check_input_function(lut0.data(), q, q);
        return run_device_op(c, B, d_out, stream, [&](Device& d) {
            return dev_func(c, d, prop, d_ct, q, d_lut, per_ct_lut ? q : 0, d_out, B);
        });
    });
}

tfhe_status tfhe_eval_floor_device(tfhe_ctx* c, size_t B, const uint64_t* d_ct, uint64_t mod, uint32_t roundbits,
                                   uint64_t* d_out, void* stream) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!d_ct || !d_out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        return run_device_op(c, B, d_out, stream,
                             [&](Device& d) { return dev_floor(c, d, d_ct, mod, roundbits, d_out, B); });
    });
}

tfhe_status tfhe_eval_sign_device(tfhe_ctx* c, size_t B, const uint64_t* d_ct, uint64_t mod, uint64_t* d_out,
                                  void* stream) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return TFHE_OK;
        if (!d_ct || !d_out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        return run_device_op(c, B, d_out, stream, [&](Device& d) { return dev_sign(c, d, d_ct, mod, d_out, B); });
    });
}

tfhe_status tfhe_eval_func(tfhe_ctx* c, size_t B, const uint64_t* ct, uint64_t q, const uint64_t* lut, int per_ct_lut,
                           uint64_t* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "EvalFunc: input vector is empty");
        if (!ct || !lut || !out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        if (q < 4 || (2ull * c->p.N) % q) return fail(TFHE_ERR_INVALID_ARGUMENT, "q must divide 2N");
        // LUT classification uses the first LUT, as the reference (binfhe-base-scheme.cpp:697-698, 815-816)
        const int prop = check_input_function(lut, q, q);
        const size_t w = c->p.n + 1;
        const uint64_t stride = per_ct_lut ? q : 0;
        // LUTs go to every device once (all of them when per ciphertext), then the batch runs
        // through the pipelined host-array runner
        const size_t D = c->devs.size();
        std::vector<uint64_t*> d_lut(D, nullptr);
        const size_t lut_words = per_ct_lut ? B * q : q;
        tfhe_status st = TFHE_OK;
        for (size_t g = 0; g < D && st == TFHE_OK; ++g) {
            if (hipSetDevice(c->devs[g].id) != hipSuccess || hipMalloc(&d_lut[g], lut_words * 8) != hipSuccess ||
                hipMemcpy(d_lut[g], lut, lut_words * 8, hipMemcpyHostToDevice) != hipSuccess)
                st = fail(TFHE_ERR_OUT_OF_MEMORY, "LUT upload failed");
        }
        if (st == TFHE_OK)
            st = run_lwe_batch(c, B, ct, w, nullptr, 0, out, w,
                               [&](Device& d, const uint64_t* i1, const uint64_t*, uint64_t* o, size_t b, size_t off) {
                                   const size_t g = (size_t)(&d - c->devs.data());  // the device's index (logical devices share an id)
                                   return dev_func(c, d, prop, i1, q, d_lut[g] + (per_ct_lut ? off * q : 0), stride, o, b);
                               },
                               WireLim{q, 0, 0, 0});
        for (size_t g = 0; g < D; ++g)
            if (d_lut[g]) hipSetDevice(c->devs[g].id), hipFree(d_lut[g]);
        return st;
    });
}

tfhe_status tfhe_eval_floor(tfhe_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint32_t roundbits,
                            uint64_t* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "EvalFloor: input vector is empty");
        if (!ct || !out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const size_t w = c->p.n + 1;
        return run_lwe_batch(c, B, ct, w, nullptr, 0, out, w,
                             [&](Device& d, const uint64_t* i1, const uint64_t*, uint64_t* o, size_t b, size_t) {
                                 return dev_floor(c, d, i1, mod, roundbits, o, b);
                             },
                             WireLim{mod, 0, 0, 0});
    });
}

tfhe_status tfhe_eval_sign(tfhe_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint64_t* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "EvalSign: input vector is empty");
        if (!ct || !out) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const size_t w = c->p.n + 1;
        return run_lwe_batch(c, B, ct, w, nullptr, 0, out, w,
                             [&](Device& d, const uint64_t* i1, const uint64_t*, uint64_t* o, size_t b, size_t) {
                                 return dev_sign(c, d, i1, mod, o, b);
                             },
                             WireLim{mod, 0, 0, 0});
    });
}

tfhe_status tfhe_eval_decomp(tfhe_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint32_t max_digits,
                             uint64_t* out, uint64_t* moduli, uint32_t* num_digits) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (B == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "EvalDecomp: input vector is empty");
        if (!ct || !out || !moduli || !num_digits) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const uint64_t q = c->p.q, beta = 128;
        if (mod <= q) return fail(TFHE_ERR_UNSUPPORTED, "EvalDecomp is only for large precision");
        // digit count and moduli are data independent (binfhe-base-scheme.cpp:1066-1080)
        std::vector<uint64_t> mods;
        for (uint64_t m = mod; m > q; m = m / q * 2 * beta) mods.push_back(q);
        {
            uint64_t m = mod;
            while (m > q) m = m / q * 2 * beta;
            mods.push_back(m);
        }
        if (mods.size() > max_digits) return fail(TFHE_ERR_INVALID_ARGUMENT, "max_digits too small");
        for (size_t i = 0; i < mods.size(); ++i) moduli[i] = mods[i];
        *num_digits = (uint32_t)mods.size();
        const uint32_t n = c->p.n;
        const size_t w = n + 1;
        return for_each_shard(c, B, [&](Device& d, size_t lo, size_t cnt) -> tfhe_status {
            const size_t chunk = std::min(cnt, c->max_chunk);
            SCHECK(ensure_scratch(c, d, chunk));
            SCHECK(sc_acquire(d, d.stream));
            DevBuf tmp_b, fl_b, dig_b;
            HCHECK(hipMalloc(&tmp_b.p, chunk * w * 8));
            HCHECK(hipMalloc(&fl_b.p, chunk * w * 8));
            HCHECK(hipMalloc(&dig_b.p, chunk * w * 8));
            uint64_t *tmp = tmp_b.as<uint64_t>(), *fl = fl_b.as<uint64_t>(), *dig = dig_b.as<uint64_t>();
            std::vector<uint64_t> host_digit(chunk * w);
            tfhe_status st = TFHE_OK;
            // every exit below leaves the stream drained before the DevBufs free their memory
            struct Drain {
                hipStream_t s;
                ~Drain() { hipStreamSynchronize(s); }
            } drain{d.stream};
            for (size_t off = lo; off < lo + cnt && st == TFHE_OK; off += chunk) {
                const size_t b = std::min(chunk, lo + cnt - off);
                HCHECK(hipMemcpyAsync(tmp, ct + off * w, b * w * 8, hipMemcpyHostToDevice, d.stream));
                uint64_t m = mod;
                for (size_t k = 0; k < mods.size() && st == TFHE_OK; ++k) {
                    if (k + 1 < mods.size()) HCHECK(launch_lwe_op(LWE_SET_MOD, n, q, 0, tmp, nullptr, dig, b, d.stream));
                    else HCHECK(hipMemcpyAsync(dig, tmp, b * w * 8, hipMemcpyDeviceToDevice, d.stream));
                    HCHECK(hipMemcpyAsync(host_digit.data(), dig, b * w * 8, hipMemcpyDeviceToHost, d.stream));
                    HCHECK(hipStreamSynchronize(d.stream));
                    for (size_t s = 0; s < b; ++s)
                        std::memcpy(out + ((off + s) * max_digits + k) * w, host_digit.data() + s * w, w * 8);
                    if (k + 1 < mods.size()) {
                        st = dev_floor(c, d, tmp, m, 0, fl, b);
                        if (st != TFHE_OK) break;
                        const uint64_t nm = m / q * 2 * beta;
                        HCHECK(launch_lwe_op(LWE_MODSWITCH, n, nm, m, fl, nullptr, tmp, b, d.stream));
                        m = nm;
                    }
                }
            }
            return st;
        });
    });
}

tfhe_status tfhe_ciphertext_mul_matrix(tfhe_ctx* c, size_t K, const uint64_t* ct, size_t cols, const int64_t* matrix,
                                       uint64_t modulus, uint64_t* out) {
    return guarded([&]() -> tfhe_status {
        SCHECK(check_ctx(c));
        if (K == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "Input ciphertexts are empty.");
        if (cols == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "Input matrix is empty.");
        if (!ct || !matrix || !out || modulus == 0) return fail(TFHE_ERR_INVALID_ARGUMENT, "null argument");
        const uint32_t w = c->p.n + 1;
        Device& d = c->devs[0];
        HCHECK(hipSetDevice(d.id));
        DevBuf dct, dm, dout;
        HCHECK(hipMalloc(&dct.p, K * w * 8));
        HCHECK(hipMalloc(&dm.p, K * cols * 8));
        HCHECK(hipMalloc(&dout.p, cols * w * 8));
        struct Drain {
            hipStream_t s;
            ~Drain() { hipStreamSynchronize(s); }
        } drain{d.stream};
        HCHECK(hipMemcpyAsync(dct.p, ct, K * w * 8, hipMemcpyHostToDevice, d.stream));
        HCHECK(hipMemcpyAsync(dm.p, matrix, K * cols * 8, hipMemcpyHostToDevice, d.stream));
        HCHECK(launch_ct_mul_matrix(w, K, dct.as<uint64_t>(), cols, dm.as<int64_t>(), modulus, dout.as<uint64_t>(),
                                    d.stream));
        HCHECK(hipMemcpyAsync(out, dout.p, cols * w * 8, hipMemcpyDeviceToHost, d.stream));
        HCHECK(hipStreamSynchronize(d.stream));
        return TFHE_OK;
    });
}

// GPULWEOperation::GPUSetup(numGPUs) (lwe-operation.cu:143-146) ignores numGPUs and works on device 0;
// so does this (CiphertextMulMatrix runs on device 0): any count is accepted, as long as a device exists
// (round 4 refused numGPUs above the visible count -- found by the multi-device drop-in test)
tfhe_status tfhe_lwe_gpu_setup(int num_gpus) {
    (void)num_gpus;
    return guarded([&]() -> tfhe_status {
        int count = 0;
        HCHECK(hipGetDeviceCount(&count));
        if (count < 1) return fail(TFHE_ERR_DEVICE, "no HIP device visible");
        return TFHE_OK;
    });
}

tfhe_status tfhe_lwe_gpu_clean(void) { return TFHE_OK; }

tfhe_status tfhe_host_selftest(const tfhe_params* pin) {
    return guarded([&]() -> tfhe_status {
        if (!pin) return fail(TFHE_ERR_INVALID_ARGUMENT, "null params");
        tfhe_params p = *pin;
        std::string err;
        if (params_finish(&p, &err) != TFHE_OK) return fail(TFHE_ERR_INVALID_ARGUMENT, err);
        NttTables t = make_ntt_tables(p.Q, p.N);
        // (1) forward/inverse round trip and (2) product vs schoolbook on a pseudo-random pair
        std::vector<uint64_t> a(p.N), b(p.N), ref(p.N, 0);
        uint64_t s = 0x1234567;
        for (uint32_t i = 0; i < p.N; ++i) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            a[i] = (s >> 7) % p.Q;
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            b[i] = (s >> 7) % p.Q;
        }
        for (uint32_t i = 0; i < p.N; ++i)
            for (uint32_t j = 0; j < p.N; ++j) {
                uint64_t v = mulmod(a[i], b[j], p.Q);
                if (i + j < p.N) ref[i + j] = addmod(ref[i + j], v, p.Q);
                else ref[i + j - p.N] = submod(ref[i + j - p.N], v, p.Q);
            }
        std::vector<uint64_t> A = a, Bv = b;
        host_ntt_fwd(t, A.data());
        host_ntt_fwd(t, Bv.data());
        for (uint32_t i = 0; i < p.N; ++i) A[i] = mulmod(A[i], Bv[i], p.Q);
        host_ntt_inv(t, A.data(), true);
        if (A != ref) return fail(TFHE_ERR_INTERNAL, "host NTT product mismatch");
        // (3) monomial table: NTT(X^m)[x] = psi^(e_x * m)
        for (uint32_t m : {1u, 3u, p.N - 1, p.N + 5, 2 * p.N - 1}) {
            std::vector<uint64_t> mon(p.N, 0);
            if (m < p.N) mon[m] = 1;
            else mon[m - p.N] = p.Q - 1;
            host_ntt_fwd(t, mon.data());
            for (uint32_t x = 0; x < p.N; ++x) {
                uint32_t idx = (uint32_t)(((uint64_t)t.eidx[x] * m) % (2ull * p.N));
                if (mon[x] != addmod(t.mono[idx], 1, p.Q)) return fail(TFHE_ERR_INTERNAL, "monomial table mismatch");
            }
        }
        // (3b) the slot exponents are 2 bitrev(x) + 1 (the fast kernel relies on it)
        for (uint32_t x = 0; x < p.N; ++x)
            if (t.eidx[x] != 2 * bitrev(x, t.logN) + 1) return fail(TFHE_ERR_INTERNAL, "eidx is not 2 bitrev(x) + 1");
        // (4) Shoup companions at the chosen word width
        const int wb = word_bits_for(p);
        const u128 R = (u128)1 << wb;
        for (uint32_t x = 0; x < p.N; ++x) {
            const uint64_t w = t.psi_br[x], wp = shoup_companion(w, p.Q, wb);
            const uint64_t aa = a[x] | (wb == 32 ? 0x80000000ull : 0x8000000000000000ull);
            const uint64_t mask = wb == 32 ? 0xFFFFFFFFull : ~0ull;
            const uint64_t qt = (uint64_t)(((u128)aa * wp) >> wb);
            const uint64_t r = (uint64_t)(((u128)aa * w - (u128)qt * p.Q) % R) & mask;
            if (r >= 2 * p.Q || r % p.Q != mulmod(aa % p.Q, w, p.Q)) return fail(TFHE_ERR_INTERNAL, "Shoup bound");
        }
        // (5) the narrow PCIe wire format's host side (pool jobs above and below the 1 MiB cut)
        for (size_t n : {(size_t)1000, (size_t)3 << 17}) {
            std::vector<uint64_t> src(n), back(n, ~0ull);
            for (size_t i = 0; i < n; ++i) src[i] = (i * 2654435761u) & 0xFFFFFFFFu;
            if (parallel_or(src.data(), n) >> 32 || wire_bytes(parallel_or(src.data(), n)) != 4)
                return fail(TFHE_ERR_INTERNAL, "wire width");
            for (int wb : {2, 4}) {
                std::vector<uint8_t> packed(n * wb);
                parallel_narrow(packed.data(), src.data(), n, wb);
                parallel_widen(back.data(), packed.data(), n, wb);
                const uint64_t mask = wb == 2 ? 0xFFFFu : 0xFFFFFFFFu;
                for (size_t i = 0; i < n; ++i)
                    if (back[i] != (src[i] & mask)) return fail(TFHE_ERR_INTERNAL, "wire narrow/widen");
            }
        }
        return TFHE_OK;
    });
}

}  // extern "C"
