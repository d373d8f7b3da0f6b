// kernels.hpp -- launch wrappers for the HIP kernels (definitions in *.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <cstdint>

namespace tfhe {

// Scalar parameters every blind-rotation kernel needs (the reference's
// params_CUDA[10], bootstrapping.cu:917-929, plus derived constants).
struct BRParams {
    uint32_t N, logN, n, dG2, digits, thr, logG;
    uint64_t Q;
    uint64_t r1;  // floor(2^b / Q), b = word bits, for lazy-sum reduction
};

// Launch choices of one context: read from the environment once, at setup (engine.hip
// knobs_from_env), changed afterwards only through tfhe_set_knobs (tests, A/B runs).  The C-ABI
// mirror is tfhe_knobs (include/tfhe_hip.h); the launchers below take them by reference.
struct Knobs {
    int32_t ks_tiled_min = -1;  // smallest batch on the tiled key switch; -1: default (1), 0: never
    int32_t ks_cts = 0;         // ciphertexts per thread of the tiled key switch; 0: by key width / batch
    int32_t ks_split = 32;      // most block groups the key-switch steps split over at small batches (u16 / u32 keys: 16 at most); 1: none
    int32_t ks_pk = 1;          // 0: no packed u16 column sums
    int32_t host_parts = 1;     // sub-batches per device of the host-array runner
    int32_t wire = 1;           // 0: u64 PCIe words (no narrow wire format)
    int32_t acc_flags = 1;      // 0: no completion-flagged EvalAcc output
    int32_t f64w = 1;           // retired (round 5: the slot-layout FP64 kernel it selected is gone); must be 1
    int32_t sf2 = 1;            // 0: gen3sf instead of the wave-local sf2
    int32_t generic = 0;        // 0: gen3 / v2 by N; 1: v1 (all digits in LDS); 2: v2 also at N = 2048
    int32_t trace = 0;          // host-array runner timeline on stderr
    int32_t probe = 0;          // test library only (TFHE_TEST_PROBES): f64w fault probe / timing builds
    int32_t duo = 128;          // most ciphertexts per launch on the two-workgroup forms (sf2duo: two digits;
                                // f64wduo: STD128Q class; <= 256); 0: never
    int32_t sf2p = 1;           // 0: sf2 with one ciphertext per workgroup instead of two (sf2p) above the duo batches
    int32_t split4 = 384;       // STD128 class: batches up to this size run fast4's two-group form (SPLIT); 0: never
    int32_t ks40 = 1;           // 8-byte keys with qKS = 2^(33..37): the tiled key switch on split-word records; 0: u64
};

// Device tables for one (Q, N), word type W (uint32_t or uint64_t storage).
struct DevTables {
    const void* psi;     // [N]  forward twiddles, bit-reversed order
    const void* psi_sh;  // [N]  Shoup companions
    const void* ipsi;    // [N]  inverse twiddles
    const void* ipsi_sh; // [N]
    const void* mono;    // [2N] psi^k - 1
    const void* mono_sh; // [2N]
    const uint32_t* eidx;// [N]  NTT(X)[x] = psi^eidx[x]
};

// Completion flags of a blind rotation (host-array EvalAcc: engine.hip d2h_flagged).  A launcher
// whose kernel stores flags[ct] = gen in host memory once ciphertext ct's accumulator is in HBM
// sets written; the others leave it false and the caller waits for the whole launch instead.
struct BRDone {
    uint32_t* flags = nullptr;  // pinned host memory, one word per ciphertext
    uint32_t gen = 0;
    bool written = false;
};

// Generic LDS-resident blind rotation: one workgroup per ciphertext.
//   a[B][n] mod amod, acc[B][2][N] (u64, coefficient) in/out, acc0 transposed on exit.
//   bsk/bsk_sh: [n][2][dG2][2][N] in W, NTT domain, scaled by N^-1.
hipError_t launch_blind_rotate_generic(int word_bits, const BRParams& P, const DevTables& T, const void* bsk,
                                       const void* bsk_sh, const uint64_t* a, uint64_t amod, uint64_t* acc, size_t B,
                                       hipStream_t s, const Knobs& kn);

// Fast STD128-class blind rotation (W = u32, N = 1024, dG2 = 8): register-resident
// transforms, one wavefront per ciphertext.  Returns hipErrorNotSupported when the
// parameters do not match its specialisation.
// split_max: batches up to this size run the two-group form (k_blind_rotate_fast4 SPLIT; tfhe_knobs.split4)
hipError_t launch_blind_rotate_fast(const BRParams& P, const DevTables& T, const void* bsk_fast, const uint64_t* a,
                                    uint64_t amod, uint64_t* acc, size_t B, hipStream_t s, BRDone* dn = nullptr,
                                    int split_max = 0);
bool fast_path_supported(const BRParams& P, int word_bits);
// Converts the generic device BSK and tables into the fast kernel's Montgomery form.
hipError_t launch_pack_bsk_fast(const BRParams& P, const DevTables& T, const void* bsk, void* bsk_fast,
                                hipStream_t s);
size_t bsk_fast_bytes(const BRParams& P);
// build of the specialised kernel (see blind_rotate_fast.hip); 0 = default; false if unknown
bool set_fast_variant(int v);
int get_fast_variant();
// 4-wavefront variant (blind_rotate_fast4.hip): its table block, packed behind the fast tables,
// and its launch (K: the fast kernel's FastConst).  Digit shape: dig digits per polynomial
// (dG2 = 2 dig), baseG = 2^logg, thr thrown digits, fold = top digit eliminated.
struct Fast4Shape {
    int dig, logg, thr;
    bool fold;
};
bool fast4_shape_supported(const Fast4Shape& sh);
size_t fast4_table_words();
hipError_t launch_pack_tables_fast4(uint32_t Q, const DevTables& T, void* out, hipStream_t s);
hipError_t launch_blind_rotate_fast4(int variant, const Fast4Shape& sh, const void* K, uint32_t n, uint32_t loga,
                                     const int32_t* tabs4, const int32_t* bsk, const uint64_t* a, uint64_t* acc,
                                     size_t B, hipStream_t s, BRDone* dn = nullptr, int split_max = 0);

// Exact-FP64 blind rotation for 2^32 <= Q < 2^50, N = 2048 (STD192 / STD192Q / STD128Q classes):
// keys/tables as centred doubles derived on device from the generic (u64) arena.
bool f64_path_supported(const BRParams& P, int word_bits);
// an instance exists for this context's (Q width, top-digit fold) combination (f64w or slot layout)
bool f64_instance_available(const BRParams& P, bool fold);
size_t bsk_f64_bytes(const BRParams& P);
// fold: eliminate the top digit's transforms (keys packed accordingly); only when
// f64_fold_enabled(P) (thr = 0; WRAP correction where the top digit is not always exact;
// TFHE_F64_FOLD=1 folds only exact sets, 0 turns it off).
bool f64_fold_enabled(const BRParams& P);
// true only in the test library (blind_rotate_f64.hip built with -DTFHE_TEST_PROBES)
bool f64_test_probes_compiled();
hipError_t launch_pack_bsk_f64(const BRParams& P, const DevTables& T, const void* bsk, bool fold, void* out,
                               hipStream_t s);
struct DuoDev;
// duo: the device's duo state (STD128Q-class batches up to kn.duo and the device's co-resident pairs run
// k_blind_rotate_f64wduo)
hipError_t launch_blind_rotate_f64(const BRParams& P, const DevTables& T, const void* keys, bool fold, const uint64_t* a,
                                   uint64_t amod, uint64_t* acc, size_t B, hipStream_t s, const Knobs& kn,
                                   DuoDev* duo = nullptr);
// true when the context's FP64 blind rotation has the two-workgroup form (STD128Q class)
bool f64_duo_form(const BRParams& P, bool fold);

// Special-form u64 blind rotation (gen3sf, blind_rotate_generic.hip) for N = 2048 and
// Q = 2^54 - c, c < 2^20 (the logQ / arbFunc contexts): constants as (w, w 2^31 mod Q), five
// multiplies per product.  sf: the W1 arrays (psi, ipsi, mono, bsk) derived on device.
bool sf_path_supported(const BRParams& P, int word_bits);
size_t sf_bytes(const BRParams& P);
hipError_t launch_pack_sf(const BRParams& P, const DevTables& T, const void* bsk, void* out, hipStream_t s);
hipError_t launch_blind_rotate_sf(const BRParams& P, const DevTables& T, const void* bsk, const void* sf,
                                  const uint64_t* a, uint64_t amod, uint64_t* acc, size_t B, hipStream_t s,
                                  const Knobs& kn, DuoDev* duo);

// Two-workgroup ("duo") blind rotations for batches too small to fill the chip (k_blind_rotate_sf2duo,
// blind_rotate_generic.hip; k_blind_rotate_f64wduo, blind_rotate_f64.hip): one per-device buffer,
// allocated at setup for the contexts that have a duo form.
//   xbuf  [pairs][2 members][2 round parities][2048] u64   the per-round hand-off (16 KiB per member)
//   flags [pairs][2 members][32] u32                        word 0: the member's round flag; word 1 of
//                                                           member 0's line: the pair's failed word
//   err   one 128-B line                                    timed-out workgroups since setup
//   save  [pairs][2][2048] u64                              the input accumulators (the rescue's input)
constexpr uint32_t kDuoMaxPairs = 256;
constexpr uint32_t kDuoN = 2048;
// Per device (engine.hip, finish_device): the buffer above; the partner-wait deadline in wall-clock ticks
// (s_memrealtime counts at hipDeviceAttributeWallClockRate: kDuoWaitMs of it); the pairs the device holds
// co-resident (the duo forms take 116-135 KiB of LDS, one workgroup per CU: half the CU count) -- a larger
// batch runs the one-workgroup kernel, so a pair's partner is never queued behind its own launch's pairs;
// and the fence that orders duo launches from different streams on the one buffer (event + host mutex).
constexpr uint32_t kDuoWaitMs = 10;
struct DuoDev {
    void* base = nullptr;
    uint64_t wait_ticks = 0;
    uint32_t resident_pairs = 0;
    hipEvent_t fence = nullptr;
    std::mutex* mu = nullptr;
};
struct DuoBuf {
    uint64_t* xbuf;
    uint32_t* flags;
    uint32_t* err;
    uint64_t* save;
    uint64_t wait_ticks;  // a member waits at most this long for its partner's flag in any round
};
inline DuoBuf duo_layout(const DuoDev& D) {
    DuoBuf X;
    X.xbuf = (uint64_t*)D.base;
    X.flags = (uint32_t*)(X.xbuf + (size_t)kDuoMaxPairs * 4 * kDuoN);
    X.err = X.flags + kDuoMaxPairs * 2 * 32;
    X.save = (uint64_t*)(X.err + 32);
    X.wait_ticks = D.wait_ticks;
    return X;
}
// Runs `launch` (the duo kernel and its rescue, on stream s) after every earlier duo launch on this device's
// buffer, whatever stream it was queued on.
template <class F>
hipError_t duo_serialised(DuoDev& D, hipStream_t s, F&& launch) {
    std::lock_guard<std::mutex> lock(*D.mu);
    if (hipError_t e = hipStreamWaitEvent(s, D.fence, 0); e != hipSuccess) return e;
    if (hipError_t e = launch(); e != hipSuccess) return e;
    return hipEventRecord(D.fence, s);
}
inline size_t duo_bytes() { return (size_t)kDuoMaxPairs * (4 * kDuoN * 8 + 2 * 128) + 128 + (size_t)kDuoMaxPairs * 2 * kDuoN * 8; }
inline uint32_t duo_err_offset_words() { return (uint32_t)((size_t)kDuoMaxPairs * 4 * kDuoN * 2 + kDuoMaxPairs * 2 * 32); }

// MKM: ModSwitch(Q->qKS), KeySwitch, ModSwitch(qKS->fmod).
//   ext[B][N+1] mod Q -> out[B][n+1] mod fmod.
//   kska: [N][baseKS][dKS][n_pad] (A part, rows padded to 16 bytes), kskb: [N][baseKS][dKS] (B),
//   both in ksk_bits words.
struct KSParams {
    uint32_t N, n, baseKS, dKS, n_pad;
    uint64_t Q, qKS;
};
hipError_t launch_mkm(const KSParams& P, int ksk_bits, const void* kska, const void* kskb, const uint64_t* ext,
                      uint64_t fmod, uint64_t* out, size_t B, hipStream_t s);
// Batch-tiled form of the same (ks_tiled.hip): the KSK is staged in LDS once per tile of
// up to 1024 ciphertexts instead of gathered per ciphertext.  scratch: ks_tiled_scratch_bytes
// (transposed digit planes).  hipErrorNotSupported when dKS > 16 or baseKS too large.
size_t ks_tiled_scratch_bytes(const KSParams& P, size_t B);
bool ks_tiled_supported(const KSParams& P);
// ksk40: the split-word records of 8-byte keys (ks40_bytes > 0: qKS = 2^(32+b), 1 <= b <= 5, the logQ contexts;
// derived at setup by launch_pack_ks40 from the arena's u64 KSK); nullptr: the u64 form
hipError_t launch_ks_tiled(const KSParams& P, int ksk_bits, const void* kska, const void* kskb, const uint64_t* ext,
                           uint64_t fmod, uint64_t* out, size_t B, void* scratch, hipStream_t s, const Knobs& kn,
                           const void* ksk40 = nullptr);
size_t ks40_bytes(const KSParams& P);
hipError_t launch_pack_ks40(const KSParams& P, const void* kska, void* out, hipStream_t s);

// ---- test vectors, extraction and LWE glue (binfhe-base-scheme.cpp) ----
enum TvMode : uint32_t {
    TV_GATE = 0,    // BootstrapGateCore: +-(Q/8+1) by range [q1,q2)
    TV_HALF = 1,    // f0/f1: x<q/2 ? fmod-q/4 : q/4
    TV_FLOOR2 = 2,  // f2 of EvalFloor
    TV_SIGN3 = 3,   // f3 of EvalSign
    TV_LUT = 4,     // LUT[x]
    TV_LUT1 = 5,    // x<q/2 ? LUT[x] : fmod - LUT[x-q/2]
    TV_LUT2 = 6,    // LUT2 = LUT++LUT, arbitrary-function second bootstrap
};
struct TvParams {
    uint32_t mode, N, n;
    uint64_t Q, ctmod, fmod;
    uint64_t q1, q2;        // gate range
    uint64_t Q8;            // Q/8 + 1
    const uint64_t* lut;    // TV_LUT*: [q] or [B][q]
    uint64_t lut_stride;    // 0: shared LUT
    uint64_t lut_len;       // original LUT length (q)
};
// ct[B][n+1] -> acc[B][2][N] (acc0 = 0, acc1 = test vector), a_out[B][n] = a part
hipError_t launch_build_testvector(const TvParams& P, const uint64_t* ct, uint64_t* acc, uint64_t* a_out, size_t B,
                                   hipStream_t s);
// tv[B][tvlen] -> acc[B][2][N]: acc0 = 0, acc1[j * (N / tvlen)] = tv[j], other coefficients 0
hipError_t launch_expand_tv(uint32_t N, uint32_t tvlen, const uint64_t* tv, uint64_t* acc, size_t B, hipStream_t s);
// u16 / u32 (wb = 2 / 4 bytes) <-> u64 words: the narrow PCIe wire format of the host-array runner
hipError_t launch_widen(const void* src, int wb, uint64_t* dst, size_t n, hipStream_t s);
hipError_t launch_narrow(const uint64_t* src, int wb, void* dst, size_t n, hipStream_t s);
// acc[B][2][N] (acc0 transposed) -> ext[B][N+1]: a = acc0, b = acc1[0] + b_add mod Q
hipError_t launch_extract(uint32_t N, uint64_t Q, uint64_t b_add, const uint64_t* acc, uint64_t* ext, size_t B,
                          hipStream_t s);

enum LweOp : uint32_t {
    LWE_ADD = 0,        // out = x + y mod m
    LWE_SUB = 1,        // out = x - y mod m
    LWE_DOUBLE_SUB = 2, // out = 2(x - y) mod m   (XOR_FAST prep)
    LWE_NOT = 3,        // out = NOT x (EvalNOT, binfhe-base-scheme.cpp:147-159)
    LWE_ADD_CONST = 4,  // b += c mod m
    LWE_SUB_CONST = 5,  // b -= c mod m
    LWE_SET_MOD = 6,    // every word mod m (LWECiphertextImpl::SetModulus)
    LWE_MODSWITCH = 7,  // RoundqQ(x, m, c)  (lwe-pke.cpp:204-215), c = old modulus
    LWE_COPY = 8,
};
// element-wise over B ciphertexts of n+1 words; y may be null for unary ops
hipError_t launch_lwe_op(uint32_t op, uint32_t n, uint64_t m, uint64_t c, const uint64_t* x, const uint64_t* y,
                         uint64_t* out, size_t B, hipStream_t s);

// Position-mixed checksum of `bytes` (a multiple of 8) of device memory: kChecksumBlocks u64 partials,
// whose sum (mod 2^64) the host forms.  engine.hip compares every key-arena replica with device 0's.
constexpr unsigned kChecksumBlocks = 1024;
hipError_t launch_checksum(const void* p, size_t bytes, uint64_t* partial, hipStream_t s);

// CiphertextMulMatrix: out[c][w] = sum_k matrix[k][c] * ct[k][w] mod modulus.
// ct and matrix are device copies the launch reduces in place into [0, modulus).
hipError_t launch_ct_mul_matrix(uint32_t width, size_t K, uint64_t* ct, size_t cols, int64_t* matrix,
                                uint64_t modulus, uint64_t* out, hipStream_t s);

}  // namespace tfhe
