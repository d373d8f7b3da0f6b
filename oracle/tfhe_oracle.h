/*
 * tfhe_oracle.h -- CPU restatement of OpenFHE's CGGI/GINX bootstrapping path.
 *
 * TEST INFRASTRUCTURE ONLY.  This code is the parity oracle for the HIP engine
 * in tfhe-gpu_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product library never links it.
 *
 * It restates, in plain C with exact u64/u128 arithmetic, the reference path
 * that north_star pins bit-exactness to (the CPU NTT path of OpenFHE inside
 * /root/reference, NOT the reference's FP64 cuFFTDx GPU kernel):
 *   - parameter selection      src/binfhe/lib/binfhecontext.cpp:42-181
 *   - signed gadget decompose   src/binfhe/lib/rgsw-acc.cpp:57-111
 *   - CGGI accumulator          src/binfhe/lib/rgsw-acc-cggi.cpp:143-155, 246-307
 *   - (X^m - 1) monomials       src/binfhe/include/rgsw-cryptoparameters.h:141-159
 *   - RoundqQ / ModSwitch       src/binfhe/lib/lwe-pke.cpp:41-46, 204-215
 *   - KeySwitch                 src/binfhe/lib/lwe-pke.cpp:299-321
 *   - vector scheme glue        src/binfhe/lib/binfhe-base-scheme.cpp:598-1277
 *
 * Parity pin: the KAT digests in tests/golden/kat_openfhe.json were produced
 * by the reference itself (OpenFHE CPU path) in the survey container
 * (SURVEY.md Appendix B); tests/test_oracle_kat.py checks this oracle
 * against every one of them.
 *
 * Data layout (all flat, little-endian u64, row-major):
 *   LWE ciphertext      [n+1]            a[0..n-1], b at index n
 *   RLWE accumulator    [2][N]           coefficient form
 *   BSK (coefficients)  [n][2][dG2][2][N]   i, key(+1/-1), gadget row, poly, coeff
 *   KSK                 [N][baseKS][dKS][n+1]  B stored at index n
 */
#ifndef TFHE_ORACLE_H
#define TFHE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint32_t n;                 /* LWE dimension */
    uint32_t N;                 /* ring dimension */
    uint64_t q;                 /* LWE modulus */
    uint64_t Q;                 /* RLWE (NTT-friendly) modulus */
    uint64_t qKS;               /* key-switching modulus */
    uint32_t baseKS;            /* key-switching base */
    uint32_t baseG;             /* gadget base (power of two) */
    uint32_t numDigitsToThrow;  /* approximate-decomposition digits dropped */
    uint32_t digitsG;           /* ceil(log Q / log baseG) */
    uint32_t dKS;               /* ceil(log qKS / log baseKS) */
    uint32_t dG2;               /* 2 * (digitsG - numDigitsToThrow) */
    uint32_t logG;              /* log2(baseG) */
} or_params;

/* BINFHE_PARAMSET numbering of src/binfhe/include/binfhe-constants.h:46-90 */
enum { OR_TOY = 0, OR_MEDIUM, OR_STD128_AP, OR_STD128_APOPT, OR_STD128, OR_STD128_OPT, OR_STD192,
       OR_STD192_OPT, OR_STD256, OR_STD256_OPT, OR_STD128Q, OR_STD128Q_OPT, OR_STD192Q,
       OR_STD192Q_OPT, OR_STD256Q, OR_STD256Q_OPT, OR_SIGNED_MOD_TEST };
/* BINGATE numbering of binfhe-constants.h:101 */
enum { OR_OR = 0, OR_AND, OR_NOR, OR_NAND, OR_XOR_FAST, OR_XNOR_FAST, OR_XOR, OR_XNOR };

/* binfhecontext.cpp:115-181 */
int or_params_from_set(int set, or_params* p);
/* binfhecontext.cpp:51-113 (arbFunc / logQ variant) */
int or_params_from_logq(int set, int arbFunc, uint32_t logQ, int64_t N, uint32_t baseG, uint32_t numDigitsToThrow,
                        or_params* p);

/* exact helpers exposed for unit tests */
uint64_t or_roundqQ(uint64_t v, uint64_t q, uint64_t Q);                    /* lwe-pke.cpp:41-46 */
int or_is_prime(uint64_t x);
/* c = a*b in Z_Q[X]/(X^N+1), schoolbook O(N^2) (slow reference for NTT tests) */
void or_polymul_schoolbook(const or_params* p, const uint64_t* a, const uint64_t* b, uint64_t* c);
/* same product through the oracle's own NTT */
void or_polymul_ntt(const or_params* p, const uint64_t* a, const uint64_t* b, uint64_t* c);
/* OpenFHE EVALUATION format: minimal primitive 2N-th root (nbtheory.cpp:284-343) and the
 * bit-reversed Cooley-Tukey transform (transformnat-impl.h:196-236, 684-706); `polys`
 * polynomials of N words, inverse includes the N^-1 scaling. */
uint64_t or_root_of_unity(uint64_t Q, uint32_t N);
void or_openfhe_ntt(uint64_t Q, uint32_t N, size_t polys, const uint64_t* in, uint64_t* out, int inverse);
/* rgsw-acc.cpp:57-111: in [2][N] -> out [dG2][N], row = poly + 2*digit, values mod Q */
void or_signed_digit_decompose(const or_params* p, const uint64_t* in, uint64_t* out);

/* ---- keys / context ---- */
typedef struct or_ctx or_ctx;
/* bsk_coeff [n][2][dG2][2][N], ksk [N][baseKS][dKS][n+1]; both copied */
or_ctx* or_create(const or_params* p, const uint64_t* bsk_coeff, const uint64_t* ksk);
void or_destroy(or_ctx* c);
void or_set_threads(int nthreads);

/* KAT synthetic keys (SURVEY.md Appendix B recipe; splitmix64 stream) */
typedef struct { uint64_t s; } or_rng;
uint64_t or_splitmix64(or_rng* r);
/* out[i] = splitmix64() % mod, i < count (the same stream as count calls of or_splitmix64) */
void or_splitmix_fill(or_rng* r, size_t count, uint64_t mod, uint64_t* out);
/* FNV-1a-64 over the little-endian bytes of w[0..count-1] (the golden-vector digest) */
uint64_t or_fnv1a64(const uint64_t* w, size_t count);
void or_kat_keys(const or_params* p, or_rng* r, uint64_t* bsk_coeff, uint64_t* ksk);

/* Valid keys (for decrypt-correctness): ternary LWE key sk[n] (mod qKS, as the
 * reference KeyGen, binfhecontext.cpp:224-227), RGSW BSK (rgsw-acc-cggi.cpp:43-77,213-240)
 * and KSK (lwe-pke.cpp:218-295). Deterministic from rng. */
void or_keygen(const or_params* p, or_rng* r, uint64_t* sk, uint64_t* bsk_coeff, uint64_t* ksk);
/* lwe-pke.cpp:56-88 ; ct [n+1] */
void or_encrypt(const or_params* p, or_rng* r, const uint64_t* sk, int64_t m, uint64_t ptxt_mod, uint64_t mod,
                uint64_t* ct);
/* lwe-pke.cpp:92-130 */
int64_t or_decrypt(const or_params* p, const uint64_t* sk, const uint64_t* ct, uint64_t ptxt_mod, uint64_t mod);

/* ---- the hot path ---- */
/* EvalAcc_CUDA contract (bootstrapping.cu:1139-1702): a[B][n] mod amod, acc[B][2][N]
 * coefficient in/out, output acc0 already transposed. */
void or_eval_acc(const or_ctx* c, size_t B, const uint64_t* a, uint64_t amod, uint64_t* acc);
/* MKMSwitch_CUDA contract (bootstrapping.cu:1855-1935): ct_ext[B][N+1] mod Q -> out[B][n+1] mod fmod */
void or_mkm_switch(const or_ctx* c, size_t B, const uint64_t* ct_ext, uint64_t fmod, uint64_t* out);

/* ---- vector BinFHEScheme surface (binfhe-base-scheme.cpp:598-1085) ---- */
/* ct* [B][n+1], all mod q; out [B][n+1] mod q. Returns 0 or an error code. */
int or_eval_bin_gate(const or_ctx* c, int gate, size_t B, const uint64_t* ct1, const uint64_t* ct2, uint64_t q,
                     uint64_t* out);
/* LUT of length q (one LUT for the whole batch); out mod q */
int or_eval_func(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t q, const uint64_t* lut, uint64_t* out);
/* per-ciphertext LUTs lut[B][q] */
int or_eval_func_vec(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t q, const uint64_t* luts, uint64_t* out);
/* ct mod `mod`; out mod `mod` */
int or_eval_floor(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint32_t roundbits, uint64_t* out);
/* ct mod `mod` (> q); out mod q */
int or_eval_sign(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint64_t* out);
/* ct mod `mod`; out [B][max_digits][n+1]; moduli[max_digits]; returns digit count (<0 on error) */
int or_eval_decomp(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint32_t max_digits, uint64_t* out,
                   uint64_t* moduli);

/* bootstraps performed since or_create (for throughput accounting) */
uint64_t or_bootstrap_count(const or_ctx* c);

#ifdef __cplusplus
}
#endif
#endif
