/*
 * tfhe_hip.h -- C-ABI of the MI355X-native batched CGGI/GINX bootstrapping engine.
 *
 * This is the drop-in boundary.  The reference (eric070021/TFHE-GPU) exposes its
 * GPU path as seven C++ static members that OpenFHE's unchanged BinFHE code calls
 * (SURVEY.md 8(b)).  Each of those maps onto one entry point here; the OpenFHE
 * side binding (the shim that defines those seven C++ symbols over this ABI, translating
 * NativeVector / NativePoly <-> u64 rows) is tfhe-gpu_amd/shim/bootstrapping_hip.cpp;
 * INTEGRATION.md describes how a maintainer links it into src/binfhe.
 *
 *   reference symbol                                        entry point
 *   GPUFFTBootstrap::GPUSetup       bootstrapping.cuh:111   tfhe_setup_eval (OpenFHE EVALUATION-format BSK) or tfhe_setup
 *   GPUFFTBootstrap::GPUClean       bootstrapping.cuh:116   tfhe_clean
 *   GPUFFTBootstrap::EvalAcc_CUDA   bootstrapping.cuh:126   tfhe_eval_acc
 *   GPUFFTBootstrap::MKMSwitch_CUDA bootstrapping.cuh:135   tfhe_mkm_switch
 *   GPULWEOperation::CiphertextMulMatrix_CUDA lwe-operation.cuh:49  tfhe_ciphertext_mul_matrix
 *   GPULWEOperation::GPUSetup       lwe-operation.cuh:57    tfhe_lwe_gpu_setup
 *   GPULWEOperation::GPUClean       lwe-operation.cuh:62    tfhe_lwe_gpu_clean
 *
 * Above those, the vector BinFHEContext surface (binfhecontext.cpp:316-347 ->
 * binfhe-base-scheme.cpp:598-1085) is offered as fused entry points that keep
 * every chained bootstrap on the device: tfhe_eval_bin_gate, tfhe_eval_func,
 * tfhe_eval_floor, tfhe_eval_sign, tfhe_eval_decomp.
 *
 * Conventions
 *  - All integers are u64, little-endian, flat row-major arrays in HOST memory
 *    unless the name ends in _device (then device pointers, ordered on the given
 *    hipStream_t passed as void*; the call runs on the context's device that
 *    holds the output buffer, found with hipPointerGetAttributes).
 *  - LWE ciphertext: [n+1] words, a[0..n-1] then b.
 *  - RLWE accumulator: [2][N] words, coefficient form.
 *  - BSK (coefficient form): [n][2][dG2][2][N]: LWE index i, ternary key
 *    (0: s_i=+1, 1: s_i=-1; rgsw-acc-cggi.cpp:53-77), gadget row (poly + 2*digit,
 *    rgsw-acc-cggi.cpp:229-238), RLWE poly, coefficient.  The reference keeps the
 *    RingGSWACCKey in EVALUATION form for OpenFHE's own NTT; the shim converts
 *    it with SetFormat(COEFFICIENT) exactly as the reference's KeyCopy_FFT does
 *    (bootstrapping.cu:1112-1137).
 *  - KSK: [N][baseKS][dKS][n+1], B stored at index n (the reference's device
 *    layout, bootstrapping.cu:961-975).
 *  - Errors: every call returns tfhe_status; tfhe_last_error() gives a message.
 *    The reference exit()s on device faults (bootstrapping.cu:28-37); here the
 *    caller decides (the shim converts to OPENFHE_THROW).
 *  - Not re-entrant per context (like the reference's static state); separate
 *    contexts are independent.
 */
#ifndef TFHE_HIP_H
#define TFHE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFHE_HIP_ABI_VERSION 8  /* 2: tfhe_info.br_kernel; 3: tfhe_info.replicate_*, tfhe_eval_acc_tv, sharding;
                                   4: row-pointer host arrays (tfhe_eval_acc_tv_rows, tfhe_mkm_switch_rows);
                                   5: device-resident EvalFunc / EvalFloor / EvalSign; tfhe_knobs;
                                   6: tfhe_knobs.duo / .sf2p, tfhe_info.duo_timeouts (two-workgroup and
                                      two-ciphertext sf2 forms);
                                   7: tfhe_knobs.split4 (two-group STD128 form); the duo forms cover
                                      STD128Q (f64wduo) and timed-out pairs are recomputed;
                                   8: tfhe_knobs.ks40 (split-word key-switch records for 8-byte keys);
                                      tfhe_rccl_selftest; the duo form covers the STD192 classes */

typedef enum tfhe_status {
    TFHE_OK = 0,
    TFHE_ERR_INVALID_ARGUMENT = 1,
    TFHE_ERR_UNSUPPORTED = 2,
    TFHE_ERR_NOT_SET_UP = 3,
    TFHE_ERR_DEVICE = 4,
    TFHE_ERR_OUT_OF_MEMORY = 5,
    TFHE_ERR_INTERNAL = 6
} tfhe_status;

/* BINFHE_PARAMSET (binfhe-constants.h:46-90) */
typedef enum tfhe_paramset {
    TFHE_TOY = 0, TFHE_MEDIUM, TFHE_STD128_AP, TFHE_STD128_APOPT, TFHE_STD128, TFHE_STD128_OPT, TFHE_STD192,
    TFHE_STD192_OPT, TFHE_STD256, TFHE_STD256_OPT, TFHE_STD128Q, TFHE_STD128Q_OPT, TFHE_STD192Q,
    TFHE_STD192Q_OPT, TFHE_STD256Q, TFHE_STD256Q_OPT, TFHE_SIGNED_MOD_TEST
} tfhe_paramset;

/* BINGATE (binfhe-constants.h:101) */
typedef enum tfhe_gate {
    TFHE_OR = 0, TFHE_AND, TFHE_NOR, TFHE_NAND, TFHE_XOR_FAST, TFHE_XNOR_FAST, TFHE_XOR, TFHE_XNOR
} tfhe_gate;

/* Flat parameter record (the reference's params_CUDA[10], bootstrapping.cu:917-929,
 * plus the gadget base).  digitsG, dKS and dG2 are derived by tfhe_params_finish. */
typedef struct tfhe_params {
    uint32_t n;                /* LWE dimension */
    uint32_t N;                /* ring dimension (power of two) */
    uint64_t q;                /* LWE modulus */
    uint64_t Q;                /* RLWE modulus, prime, Q = 1 mod 2N */
    uint64_t qKS;              /* key-switching modulus */
    uint32_t baseKS;           /* key-switching base */
    uint32_t baseG;            /* gadget base, power of two */
    uint32_t numDigitsToThrow; /* approximate gadget decomposition */
    uint32_t digitsG;          /* ceil(log Q / log baseG)           (derived) */
    uint32_t dKS;              /* ceil(log qKS / log baseKS)        (derived) */
    uint32_t dG2;              /* 2*(digitsG - numDigitsToThrow)    (derived) */
} tfhe_params;

typedef struct tfhe_info {
    int num_devices;           /* devices the context shards over */
    int word_bits;             /* 32: Q fits the u32 Shoup path; 64 otherwise */
    uint64_t bsk_device_bytes; /* per device */
    uint64_t ksk_device_bytes; /* per device */
    uint64_t bootstraps;       /* blind rotations executed since setup */
    uint64_t key_image_bytes;  /* size of the exportable device key image */
    int br_kernel;             /* blind rotation for power-of-two a-moduli: TFHE_BR_* */
    int replicate_method;      /* how setup replicated the key image to devices 1..: TFHE_REPLICATE_* */
    double replicate_ms;       /* wall time of that replication (0 for one device) */
    uint32_t duo_timeouts;     /* workgroups of the two-workgroup forms (sfduo: one- and two-digit special-form
                                  contexts; f64wduo: STD128Q and STD192 classes) that timed out waiting for their partner
                                  (10 ms of wall clock in one round) since setup, summed over devices
                                  (synchronises them); the ciphertexts of such a pair are recomputed from
                                  their saved inputs by the one-workgroup kernel (sf2 / f64w) queued behind
                                  the same launch, so outputs stay exact */
} tfhe_info;

/* tfhe_info.replicate_method */
#define TFHE_REPLICATE_NONE 0  /* one device */
#define TFHE_REPLICATE_RCCL 1  /* one RCCL broadcast from device 0 over xGMI (librccl, loaded at setup) */
#define TFHE_REPLICATE_PEER 2  /* concurrent peer copies from device 0 (no RCCL, or TFHE_REPLICATE=peer) */

/* tfhe_info.br_kernel */
#define TFHE_BR_GENERIC 0      /* generic v2 (or v1) Shoup kernel, blind_rotate_generic.hip */
#define TFHE_BR_FAST 1         /* specialised STD128 kernel, blind_rotate_fast4.hip */
#define TFHE_BR_F64 2          /* exact-FP64 kernel, blind_rotate_f64.hip */
#define TFHE_BR_F64_FOLD 3     /* exact-FP64 kernel, top digit's transforms eliminated */
#define TFHE_BR_RNS 4          /* (retired in round 3: the four-prime RNS kernel; never returned) */
#define TFHE_BR_SF 5           /* special-form u64 kernel (Q = 2^54 - c), blind_rotate_generic.hip sf2 / gen3sf */

typedef struct tfhe_ctx tfhe_ctx;

/* ---- parameters (binfhecontext.cpp:42-181) ---- */
tfhe_status tfhe_params_from_set(int paramset, tfhe_params* out);
tfhe_status tfhe_params_from_logq(int paramset, int arb_func, uint32_t logQ, int64_t N, uint32_t baseG,
                                  uint32_t num_digits_to_throw, tfhe_params* out);
tfhe_status tfhe_params_finish(tfhe_params* p);

/* ---- reference boundary ----
 * num_gpus as GPUSetup(numGPUs) (bootstrapping.cu:736-739): <= 0 or more than visible = every visible
 * device; batches are cut into one contiguous shard per device. */
tfhe_status tfhe_setup(tfhe_ctx** out, const tfhe_params* p, const uint64_t* bsk_coeff, const uint64_t* ksk,
                       int num_gpus);
/* Same, with the BSK exactly as OpenFHE holds it after KeyGen / BTKeyLoad: EVALUATION
 * format, (*BSkey)[0][key][i][l][m].GetValues() in [n][2][dG2][2][N] order (rgsw-acc-cggi.cpp:231-236).
 * Replaces the host INTT the reference runs in GPUSetup_core (bootstrapping.cu:874-1083)
 * and the shim's SetFormat(COEFFICIENT): the library's NTT uses OpenFHE's root
 * (RootOfUnity(2N, Q), rgsw-cryptoparameters.h:80, nbtheory.cpp:284-343) and transform
 * (transformnat-impl.h:196-236, 684-706), so the values are taken as they are.  Entries
 * must be < Q (TFHE_ERR_INVALID_ARGUMENT otherwise). */
tfhe_status tfhe_setup_eval(tfhe_ctx** out, const tfhe_params* p, const uint64_t* bsk_eval, const uint64_t* ksk,
                            int num_gpus);
tfhe_status tfhe_clean(tfhe_ctx* ctx);
/* a[B][n] mod a_mod; acc[B][2][N] coefficient in/out; acc0 returned transposed
 * (the callers rely on it: binfhe-base-scheme.cpp:665-671, 1203-1204). */
tfhe_status tfhe_eval_acc(tfhe_ctx* ctx, size_t B, const uint64_t* a, uint64_t a_mod, uint64_t* acc);
/* EvalAcc_CUDA for the accumulators the vector callers build (BootstrapGateCore / BootstrapFuncCore,
 * binfhe-base-scheme.cpp:1110-1138, 1163-1185): acc0 = 0 and acc1 zero except at multiples of
 * N / tv_len, whose values are tv[B][tv_len] (tv_len = a_mod / 2 there).  Same output as tfhe_eval_acc
 * on the expanded accumulators, with tv_len instead of 2N words per ciphertext sent to the device
 * (the drop-in shim detects the shape, tfhe-gpu_amd/shim/bootstrapping_hip.cpp). */
tfhe_status tfhe_eval_acc_tv(tfhe_ctx* ctx, size_t B, const uint64_t* a, uint64_t a_mod, const uint64_t* tv,
                             uint32_t tv_len, uint64_t* acc);
/* ct_ext[B][N+1] mod Q -> out[B][n+1] mod fmod: ModSwitch(qKS), KeySwitch, ModSwitch(fmod) */
tfhe_status tfhe_mkm_switch(tfhe_ctx* ctx, size_t B, const uint64_t* ct_ext, uint64_t fmod, uint64_t* out);
/* Row-pointer forms of the two calls above, for callers whose ciphertexts live in separate
 * allocations (OpenFHE: one NativeVector per polynomial and per LWE "a", which the drop-in shim
 * passes as pointers to their u64 storage): the pinned PCIe staging reads and writes the rows where
 * they are, so no flat copy of the arrays exists on either side.  Same results as the flat calls.
 *   tfhe_eval_acc_tv_rows: a_rows[s] -> n words; tv[B][tv_len] flat; acc_rows[2s + j] -> polynomial
 *                          j (N words) of accumulator s (written, acc0 transposed)
 *   tfhe_mkm_switch_rows:  ext_a_rows[s] -> N words, ext_b[s]; out_a_rows[s] -> n words, out_b[s] */
tfhe_status tfhe_eval_acc_tv_rows(tfhe_ctx* ctx, size_t B, const uint64_t* const* a_rows, uint64_t a_mod,
                                  const uint64_t* tv, uint32_t tv_len, uint64_t* const* acc_rows);
tfhe_status tfhe_mkm_switch_rows(tfhe_ctx* ctx, size_t B, const uint64_t* const* ext_a_rows, const uint64_t* ext_b,
                                 uint64_t fmod, uint64_t* const* out_a_rows, uint64_t* out_b);
/* out[c] = sum_k matrix[k][c] * ct[k] mod modulus, c < cols: ct[K][n+1], matrix[K][cols], out[cols][n+1] */
tfhe_status tfhe_ciphertext_mul_matrix(tfhe_ctx* ctx, size_t K, const uint64_t* ct, size_t cols, const int64_t* matrix,
                                       uint64_t modulus, uint64_t* out);
tfhe_status tfhe_lwe_gpu_setup(int num_gpus);
tfhe_status tfhe_lwe_gpu_clean(void);

/* ---- vector BinFHEContext surface, bootstraps chained on device ---- */
tfhe_status tfhe_eval_bin_gate(tfhe_ctx* ctx, int gate, size_t B, const uint64_t* ct1, const uint64_t* ct2, uint64_t q,
                               uint64_t* out);
/* lut: [q] shared (per_ct_lut = 0) or [B][q] (per_ct_lut = 1); out mod q */
tfhe_status tfhe_eval_func(tfhe_ctx* ctx, size_t B, const uint64_t* ct, uint64_t q, const uint64_t* lut, int per_ct_lut,
                           uint64_t* out);
tfhe_status tfhe_eval_floor(tfhe_ctx* ctx, size_t B, const uint64_t* ct, uint64_t mod, uint32_t roundbits,
                            uint64_t* out);
/* ct mod `mod`; out mod q (the LWE modulus) */
tfhe_status tfhe_eval_sign(tfhe_ctx* ctx, size_t B, const uint64_t* ct, uint64_t mod, uint64_t* out);
/* out[B][max_digits][n+1]; moduli[max_digits]; *num_digits set */
tfhe_status tfhe_eval_decomp(tfhe_ctx* ctx, size_t B, const uint64_t* ct, uint64_t mod, uint32_t max_digits,
                             uint64_t* out, uint64_t* moduli, uint32_t* num_digits);

/* ---- device-resident variants (inputs/outputs already in HBM) ----
 * The device is the one holding d_out / d_acc (a multi-device context runs the
 * call on that device's key arena; the stream must belong to it).  A buffer on
 * a device the context does not use is TFHE_ERR_INVALID_ARGUMENT. */
tfhe_status tfhe_eval_bin_gate_device(tfhe_ctx* ctx, int gate, size_t B, const uint64_t* d_ct1,
                                      const uint64_t* d_ct2, uint64_t q, uint64_t* d_out, void* stream);
tfhe_status tfhe_eval_acc_device(tfhe_ctx* ctx, size_t B, const uint64_t* d_a, uint64_t a_mod, uint64_t* d_acc,
                                 void* stream);
tfhe_status tfhe_mkm_switch_device(tfhe_ctx* ctx, size_t B, const uint64_t* d_ct_ext, uint64_t fmod, uint64_t* d_out,
                                   void* stream);
/* The chained vector ops of binfhe-base-scheme.cpp:679-1037 with every intermediate in HBM (the
 * same pipelines as tfhe_eval_func / _floor / _sign).  d_lut: [q] or [B][q] in device memory; its
 * first q words are read back once per call to classify the batch (binfhe-base-scheme.cpp:697-698). */
tfhe_status tfhe_eval_func_device(tfhe_ctx* ctx, size_t B, const uint64_t* d_ct, uint64_t q, const uint64_t* d_lut,
                                  int per_ct_lut, uint64_t* d_out, void* stream);
tfhe_status tfhe_eval_floor_device(tfhe_ctx* ctx, size_t B, const uint64_t* d_ct, uint64_t mod, uint32_t roundbits,
                                   uint64_t* d_out, void* stream);
tfhe_status tfhe_eval_sign_device(tfhe_ctx* ctx, size_t B, const uint64_t* d_ct, uint64_t mod, uint64_t* d_out,
                                  void* stream);

/* ---- key replication for one-process-per-GPU deployments ----
 * The packed device key image (NTT-domain BSK with Shoup companions, packed
 * KSK, tables) can be copied device-to-device (e.g. broadcast over RCCL/xGMI by
 * torch.distributed) and adopted by another process without host conversion. */
tfhe_status tfhe_export_key_image(tfhe_ctx* ctx, void* d_dst, size_t bytes, void* stream);
tfhe_status tfhe_setup_from_key_image(tfhe_ctx** out, const tfhe_params* p, const void* d_src, size_t bytes,
                                      int device);
/* The same image as a file (cache the packed layout on disk; replaces
 * BTKeyLoad + GPUSetup's host conversion, binfhecontext.h:208-220, bootstrapping.cu:874-1083):
 * header {magic "TFHEKIMG", ABI version, tfhe_params, image bytes, FNV-1a 64 of the image}
 * followed by the image.  Loading checks magic, version, parameters, size and checksum
 * before touching the device. */
tfhe_status tfhe_save_key_image(tfhe_ctx* ctx, const char* path);
tfhe_status tfhe_setup_from_key_file(tfhe_ctx** out, const tfhe_params* p, const char* path, int device);

/* ---- introspection ---- */
tfhe_status tfhe_get_info(tfhe_ctx* ctx, tfhe_info* out);
const char* tfhe_status_string(tfhe_status s);
const char* tfhe_last_error(void);
int tfhe_abi_version(void);
/* host-only self test of the NTT tables and packing (no GPU needed); 0 = pass */
tfhe_status tfhe_host_selftest(const tfhe_params* p);

/* ---- sharding (no reference counterpart; the reference deals SM_count-sized chunks round-robin,
 * bootstrapping.cu:1617): contiguous shard `rank` of `world` over `total` units, sizes differing by at
 * most one -- the split tfhe_setup(num_gpus) contexts use across their devices and bench.py uses across
 * ranks.  tfhe_host_shard_selftest runs the multi-device runner (one host thread per device) on
 * `devices` fake devices with no GPU: spans[2g], spans[2g+1] = the (lo, count) device g was given;
 * fail_device >= 0 makes that device's body fail, and the call returns its status with
 * tfhe_last_error() = "device <g>: ...". ---- */
tfhe_status tfhe_shard_range(size_t total, int world, int rank, size_t* lo, size_t* hi);
tfhe_status tfhe_host_shard_selftest(size_t B, int devices, int fail_device, size_t* spans);
/* The RCCL sequence of tfhe_setup(num_gpus)'s key replication (communicator over the devices, one
 * ncclBroadcast per rank in a group, streams synchronised, communicators destroyed) run on ONE device with
 * a one-rank communicator: `bytes` (a multiple of 8) of a seeded buffer broadcast out of place and the two
 * copies' checksums compared.  lib NULL or "" = the system librccl (what tfhe_setup loads); *version =
 * ncclGetVersion's (0 if the library lacks it).  TFHE_ERR_UNSUPPORTED when the library does not load;
 * TFHE_ERR_DEVICE when a call fails or the copy differs.  Checks the engine's RCCL binding against the
 * real library on a one-GPU box (the reference's GPUSetup(numGPUs) copies per GPU from the host,
 * bootstrapping.cu:1005-1069). */
tfhe_status tfhe_rccl_selftest(int device, size_t bytes, const char* lib, int* version);

/* ---- launch knobs (no reference counterpart): the kernel-form choices earlier rounds measured A/B.
 * Read from the environment once, when a context is set up (TFHE_KS_TILED_MIN, TFHE_KS_CTS,
 * TFHE_KS_SPLIT, TFHE_KS_PK, TFHE_HOST_PARTS, TFHE_WIRE, TFHE_ACC_FLAGS, TFHE_F64W, TFHE_SF2,
 * TFHE_GENERIC, TFHE_DUO, TFHE_SF2P, TFHE_SPLIT4, TFHE_KS40, TFHE_TRACE); afterwards only tfhe_set_knobs changes them -- no
 * launch reads the environment.  Every setting computes the same outputs (each is a parity-tested
 * cross-check).  A variable that is not a whole number, or a value out of the field's range, fails
 * the setup with TFHE_ERR_INVALID_ARGUMENT (tfhe_set_knobs checks the same ranges).  tfhe_set_knobs
 * must not run while another call on the same context is in flight (the calls read the knobs
 * without a lock, as OpenFHE's BinFHEContext is not safe to reconfigure mid-call either). ---- */
typedef struct tfhe_knobs {
    int32_t ks_tiled_min; /* smallest batch on the batch-tiled key switch; -1: the default (1); 0: never */
    int32_t ks_cts;       /* ciphertexts per thread in the tiled key switch: 0 (by key width / batch), 1, 2, 4 (4: the packed
                             u16 form only -- STD128's keys, its default from 2048 ciphertexts; other widths take 2) */
    int32_t ks_split;     /* most block groups the key-switch steps split over at small batches (1: none) */
    int32_t ks_pk;        /* 0: 32-bit column sums for u16 keys instead of packed u16 pairs */
    int32_t host_parts;   /* sub-batches per device in the host-array runner (>= 1) */
    int32_t wire;         /* 0: u64 words over PCIe (no narrow wire format) */
    int32_t acc_flags;    /* 0: host-array EvalAcc waits for the whole launch (no completion flags) */
    int32_t f64w;         /* retired: must be 1 (round 5 removed the slot-layout FP64 kernel 0 selected) */
    int32_t sf2;          /* 0: gen3sf special-form blind rotation instead of the wave-local sf2 */
    int32_t generic;      /* generic kernel form: 0 by N; 1 v1 (digits in LDS); 2 v2 also at N = 2048 */
    int32_t trace;        /* host-array runner timeline on stderr */
    int32_t probe;        /* test library only (lib/libtfhe_hip_test.so): fault-probe / timing builds */
    int32_t duo;          /* one- and two-digit special-form contexts (sfduo) and STD128Q- / STD192-class FP64 contexts (f64wduo):
                             batches up to this size (default 128, at most 256) run each ciphertext on two
                             workgroups, and only while the device holds every pair co-resident (a duo workgroup
                             takes one CU: at most half the CU count, 128 on MI355X); 0: never */
    int32_t sf2p;         /* two-digit special-form contexts, batches of 512 or more: 1 (default) runs two
                             ciphertexts per workgroup (sf2p, whose shared LDS holds the whole monomial factor
                             table); 0: one per workgroup (sf2) */
    int32_t split4;       /* STD128-class contexts: batches up to this size (default 384) run each ciphertext's two
                             polynomials on two groups of four wavefronts (fast4 SPLIT); 0: never */
    int32_t ks40;         /* contexts whose key-switching keys need 8-byte words with qKS = 2^33 .. 2^37 (the logQ
                             contexts: 2^35): 1 (default) runs the tiled key switch on split-word records derived
                             at setup (u32 low word + u8 high part per key, 80 B per 16-column row segment instead
                             of 128 B); 0: on the u64 words */
} tfhe_knobs;
tfhe_status tfhe_get_knobs(tfhe_ctx* ctx, tfhe_knobs* out);
tfhe_status tfhe_set_knobs(tfhe_ctx* ctx, const tfhe_knobs* in);

/* ---- extension (no reference counterpart): build of the specialised STD128-class blind
 * rotation used by later calls, for A/B runs and tests; 0 restores the default.  Process-wide;
 * initial value from TFHE_FAST_VARIANT.  Every build computes the same output. ---- */
tfhe_status tfhe_set_kernel_variant(int variant);
int tfhe_get_kernel_variant(void);

#ifdef __cplusplus
}
#endif
#endif /* TFHE_HIP_H */
