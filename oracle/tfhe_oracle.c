/*
 * tfhe_oracle.c -- CPU restatement of OpenFHE's CGGI/GINX bootstrap (TEST INFRASTRUCTURE).
 *
 * See tfhe_oracle.h for scope and the reference lines each function follows.
 * Arithmetic is exact: every modular product goes through unsigned __int128 and
 * `%`.  Speed is secondary; correctness must be evident on reading.  Batches run
 * one ciphertext per OpenMP thread, the same loop structure the reference uses
 * on the CPU (independent single-ciphertext evaluations).
 */
#include "tfhe_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

static int g_threads = 0;
void or_set_threads(int nthreads) { g_threads = nthreads; }
static int nthreads_for(size_t B) {
#ifdef _OPENMP
    int t = g_threads > 0 ? g_threads : omp_get_max_threads();
    if ((size_t)t > B) t = (int)B;
    return t < 1 ? 1 : t;
#else
    (void)B;
    return 1;
#endif
}

/* ------------------------------------------------------------------ */
/* modular helpers                                                     */
/* ------------------------------------------------------------------ */
static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)(((u128)a * b) % m); }
static inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t m) {
    uint64_t r = a + b; /* operands < m < 2^63 */
    return r >= m ? r - m : r;
}
/* NativeInteger::ModSubFast, ubintnat.h:1072-1084 (operands < m) */
static inline uint64_t submod(uint64_t a, uint64_t b, uint64_t m) { return a >= b ? a - b : a + (m - b); }
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t m) {
    uint64_t r = 1 % m;
    b %= m;
    while (e) {
        if (e & 1) r = mulmod(r, b, m);
        b = mulmod(b, b, m);
        e >>= 1;
    }
    return r;
}

/* deterministic Miller-Rabin for 64-bit integers */
int or_is_prime(uint64_t x) {
    static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (x < 2) return 0;
    for (int i = 0; i < 12; ++i) {
        if (x == bases[i]) return 1;
        if (x % bases[i] == 0) return 0;
    }
    uint64_t d = x - 1;
    int s = 0;
    while (!(d & 1)) { d >>= 1; ++s; }
    for (int i = 0; i < 12; ++i) {
        uint64_t y = powmod(bases[i], d, x);
        if (y == 1 || y == x - 1) continue;
        int comp = 1;
        for (int r = 1; r < s; ++r) {
            y = mulmod(y, y, x);
            if (y == x - 1) { comp = 0; break; }
        }
        if (comp) return 0;
    }
    return 1;
}

/* nbtheory.cpp:481-516 FirstPrime */
static uint64_t first_prime(uint32_t nBits, uint64_t m) {
    uint64_t r = powmod(2, nBits, m);
    uint64_t q = (1ull << nBits);
    q = r > 0 ? q + (m - r) + 1 : q + 1;
    while (!or_is_prime(q)) q += m;
    return q;
}
/* nbtheory.cpp:565-579 PreviousPrime */
static uint64_t previous_prime(uint64_t q, uint64_t m) {
    uint64_t x = q - m;
    while (!or_is_prime(x)) x -= m;
    return x;
}

static uint32_t ilog2u(uint64_t x) {
    uint32_t r = 0;
    while (x > 1) { x >>= 1; ++r; }
    return r;
}

static void finish_params(or_params* p) {
    /* rgsw-cryptoparameters.h:87 and lwe-pke.cpp:305 use natural-log ratios */
    p->digitsG = (uint32_t)ceil(log((double)p->Q) / log((double)p->baseG));
    p->dKS = (uint32_t)ceil(log((double)p->qKS) / log((double)p->baseKS));
    p->dG2 = 2 * (p->digitsG - p->numDigitsToThrow);
    p->logG = ilog2u(p->baseG);
}

int or_params_from_set(int set, or_params* p) {
    /* binfhecontext.cpp:137-155: numberBits, cyclOrder, n, q, qKS (0 = Q), baseKS, baseG */
    static const struct { int set; uint32_t bits, cycl, n, q; uint64_t qks; uint32_t bks, g; } T[] = {
        {OR_TOY, 27, 1024, 64, 512, 0, 25, 1u << 9},
        {OR_MEDIUM, 28, 2048, 422, 1024, 1u << 14, 1u << 7, 1u << 10},
        {OR_STD128_AP, 27, 2048, 512, 1024, 1u << 14, 1u << 7, 1u << 9},
        {OR_STD128_APOPT, 27, 2048, 502, 1024, 1u << 14, 1u << 7, 1u << 9},
        {OR_STD128, 27, 2048, 512, 1024, 1u << 14, 1u << 7, 1u << 7},
        {OR_STD128_OPT, 27, 2048, 502, 1024, 1u << 14, 1u << 7, 1u << 7},
        {OR_STD192, 37, 4096, 1024, 1024, 1u << 19, 28, 1u << 14},
        {OR_STD192_OPT, 37, 4096, 805, 1024, 1u << 15, 32, 1u << 13},
        {OR_STD256, 29, 4096, 1024, 2048, 1u << 14, 1u << 7, 1u << 8},
        {OR_STD256_OPT, 29, 4096, 990, 2048, 1u << 14, 1u << 7, 1u << 8},
        {OR_STD128Q, 50, 4096, 1024, 1024, 1u << 25, 32, 1u << 25},
        {OR_STD128Q_OPT, 50, 4096, 585, 1024, 1u << 15, 32, 1u << 25},
        {OR_STD192Q, 35, 4096, 1024, 1024, 1u << 17, 64, 1u << 14},
        {OR_STD192Q_OPT, 35, 4096, 875, 1024, 1u << 15, 32, 1u << 12},
        {OR_STD256Q, 27, 4096, 2048, 2048, 1u << 16, 16, 1u << 7},
        {OR_STD256Q_OPT, 27, 4096, 1225, 1024, 1u << 16, 16, 1u << 7},
        {OR_SIGNED_MOD_TEST, 28, 2048, 512, 1024, 0, 25, 1u << 7},
    };
    for (size_t i = 0; i < sizeof(T) / sizeof(T[0]); ++i) {
        if (T[i].set != set) continue;
        memset(p, 0, sizeof(*p));
        p->Q = previous_prime(first_prime(T[i].bits, T[i].cycl), T[i].cycl);
        p->N = T[i].cycl / 2;
        p->n = T[i].n;
        p->q = T[i].q;
        p->qKS = T[i].qks ? T[i].qks : p->Q;
        p->baseKS = T[i].bks;
        p->baseG = T[i].g;
        p->numDigitsToThrow = 0;
        finish_params(p);
        return 0;
    }
    return -1;
}

/* StdLatticeParm::FindRingDim for HEStd_ternary / HEStd_128_classic (stdlatticeparms.cpp:110-130) */
static uint32_t find_ring_dim_ternary128(uint32_t logQ) {
    static const uint32_t dims[] = {1024, 2048, 4096, 8192, 16384, 32768, 65536};
    static const uint32_t maxq[] = {27, 54, 109, 218, 438, 881, 1772};
    uint32_t prev = 0;
    for (int i = 0; i < 7; ++i) {
        if (logQ <= maxq[i] && logQ > prev) return dims[i];
        prev = maxq[i];
    }
    return 2 * 65536;
}

int or_params_from_logq(int set, int arbFunc, uint32_t logQ, int64_t N, uint32_t baseG, uint32_t numDigitsToThrow,
                        or_params* p) {
    if (set != OR_STD128 && set != OR_TOY) return -1;
    if (logQ > 29 || logQ < 11) return -2;
    uint32_t logQprime = 54;
    if (baseG == 0) {
        if (logQ > 25) baseG = 1u << 14;
        else if (logQ > 16) baseG = 1u << 18;
        else if (logQ > 11) baseG = 1u << 27;
        else { baseG = 1u << 5; logQprime = 27; }
    }
    uint32_t ringDim = find_ring_dim_ternary128(logQprime);
    if (N >= (int64_t)ringDim) ringDim = (uint32_t)N;
    memset(p, 0, sizeof(*p));
    p->Q = previous_prime(first_prime(logQprime, 2ull * ringDim), 2ull * ringDim);
    p->N = ringDim;
    p->q = arbFunc ? ringDim : 2ull * ringDim;
    p->qKS = 1ull << 35;
    p->n = set == OR_TOY ? 32 : 1305;
    p->baseKS = 32;
    p->baseG = baseG;
    p->numDigitsToThrow = numDigitsToThrow;
    finish_params(p);
    if (p->digitsG <= p->numDigitsToThrow) return -3;
    return 0;
}

/* lwe-pke.cpp:41-46 -- literally the reference's double formula, evaluated left to right */
uint64_t or_roundqQ(uint64_t v, uint64_t q, uint64_t Q) {
    volatile double t = (double)v * (double)q; /* volatile: forbid FMA contraction */
    double u = t / (double)Q;
    return (uint64_t)floor(0.5 + u) % q;
}

/* ------------------------------------------------------------------ */
/* negacyclic NTT mod Q (Longa-Naehrig CT forward / GS inverse)         */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t N, logN;
    uint64_t Q, Ninv;
    uint64_t* psi_br;   /* psi^brv(k)      k < N */
    uint64_t* ipsi_br;  /* psi^-brv(k)     k < N */
} ntt_tab;

static uint32_t bitrev(uint32_t x, uint32_t bits) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}

static uint64_t find_psi(uint64_t Q, uint32_t N) {
    /* primitive 2N-th root of unity: psi^N == -1 */
    for (uint64_t g = 2;; ++g) {
        uint64_t x = powmod(g, (Q - 1) / (2ull * N), Q);
        if (powmod(x, N, Q) == Q - 1) return x;
    }
}

static void ntt_init(ntt_tab* t, uint64_t Q, uint32_t N) {
    t->N = N;
    t->logN = ilog2u(N);
    t->Q = Q;
    t->Ninv = powmod(N, Q - 2, Q);
    t->psi_br = (uint64_t*)malloc(sizeof(uint64_t) * N);
    t->ipsi_br = (uint64_t*)malloc(sizeof(uint64_t) * N);
    uint64_t psi = find_psi(Q, N), ipsi = powmod(psi, Q - 2, Q);
    for (uint32_t k = 0; k < N; ++k) {
        uint32_t e = bitrev(k, t->logN);
        t->psi_br[k] = powmod(psi, e, Q);
        t->ipsi_br[k] = powmod(ipsi, e, Q);
    }
}
static void ntt_free(ntt_tab* t) {
    free(t->psi_br);
    free(t->ipsi_br);
}

static void ntt_fwd(const ntt_tab* t, uint64_t* a) {
    const uint64_t Q = t->Q;
    uint32_t len = t->N;
    for (uint32_t m = 1; m < t->N; m <<= 1) {
        len >>= 1;
        for (uint32_t i = 0; i < m; ++i) {
            uint64_t S = t->psi_br[m + i];
            uint32_t j1 = 2 * i * len;
            for (uint32_t j = j1; j < j1 + len; ++j) {
                uint64_t U = a[j], V = mulmod(a[j + len], S, Q);
                a[j] = addmod(U, V, Q);
                a[j + len] = submod(U, V, Q);
            }
        }
    }
}
static void ntt_inv(const ntt_tab* t, uint64_t* a) {
    const uint64_t Q = t->Q;
    uint32_t len = 1;
    for (uint32_t m = t->N; m > 1; m >>= 1) {
        uint32_t h = m >> 1, j1 = 0;
        for (uint32_t i = 0; i < h; ++i) {
            uint64_t S = t->ipsi_br[h + i];
            for (uint32_t j = j1; j < j1 + len; ++j) {
                uint64_t U = a[j], V = a[j + len];
                a[j] = addmod(U, V, Q);
                a[j + len] = mulmod(submod(U, V, Q), S, Q);
            }
            j1 += 2 * len;
        }
        len <<= 1;
    }
    for (uint32_t j = 0; j < t->N; ++j) a[j] = mulmod(a[j], t->Ninv, Q);
}

/* OpenFHE's EVALUATION format (what RingGSWACCKey polynomials hold after BTKeyLoad /
 * KeyGen, rgsw-acc-cggi.cpp:231-236).
 * Root: RootOfUnity(2N, Q) (rgsw-cryptoparameters.h:80) = the smallest primitive 2N-th
 * root of unity, nbtheory.cpp:284-343 (any generator's (Q-1)/2N power, then the minimum
 * over its odd powers).  Table: Table[bitrev(i)] = root^i (transformnat-impl.h:684-706).
 * Transform: ForwardTransformToBitReverseInPlace (transformnat-impl.h:196-236), Cooley-Tukey
 * with omega = Table[m + i] -- the same loop as ntt_fwd above. */
uint64_t or_root_of_unity(uint64_t Q, uint32_t N) {
    const uint64_t r = find_psi(Q, N), r2 = mulmod(r, r, Q);
    uint64_t best = r, x = r;
    for (uint32_t k = 3; k < 2 * N; k += 2) {
        x = mulmod(x, r2, Q);
        if (x < best) best = x;
    }
    return best;
}

void or_openfhe_ntt(uint64_t Q, uint32_t N, size_t polys, const uint64_t* in, uint64_t* out, int inverse) {
    ntt_tab t;
    t.N = N;
    t.logN = ilog2u(N);
    t.Q = Q;
    t.Ninv = powmod(N, Q - 2, Q);
    t.psi_br = (uint64_t*)malloc(sizeof(uint64_t) * N);
    t.ipsi_br = (uint64_t*)malloc(sizeof(uint64_t) * N);
    const uint64_t psi = or_root_of_unity(Q, N), ipsi = powmod(psi, Q - 2, Q);
    for (uint32_t k = 0; k < N; ++k) {
        t.psi_br[bitrev(k, t.logN)] = powmod(psi, k, Q);
        t.ipsi_br[bitrev(k, t.logN)] = powmod(ipsi, k, Q);
    }
    for (size_t k = 0; k < polys; ++k) {
        uint64_t* a = out + k * N;
        for (uint32_t j = 0; j < N; ++j) a[j] = in[k * N + j] % Q;
        if (inverse) ntt_inv(&t, a); /* InverseTransformFromBitReverseInPlace, incl. N^-1 */
        else ntt_fwd(&t, a);
    }
    ntt_free(&t);
}

void or_polymul_schoolbook(const or_params* p, const uint64_t* a, const uint64_t* b, uint64_t* c) {
    const uint32_t N = p->N;
    const uint64_t Q = p->Q;
    for (uint32_t k = 0; k < N; ++k) c[k] = 0;
    for (uint32_t i = 0; i < N; ++i)
        for (uint32_t j = 0; j < N; ++j) {
            uint64_t v = mulmod(a[i], b[j], Q);
            uint32_t k = i + j;
            if (k < N) c[k] = addmod(c[k], v, Q);
            else c[k - N] = submod(c[k - N], v, Q); /* X^N = -1 */
        }
}

void or_polymul_ntt(const or_params* p, const uint64_t* a, const uint64_t* b, uint64_t* c) {
    ntt_tab t;
    ntt_init(&t, p->Q, p->N);
    uint64_t* x = (uint64_t*)malloc(sizeof(uint64_t) * p->N);
    memcpy(x, a, sizeof(uint64_t) * p->N);
    memcpy(c, b, sizeof(uint64_t) * p->N);
    ntt_fwd(&t, x);
    ntt_fwd(&t, c);
    for (uint32_t k = 0; k < p->N; ++k) c[k] = mulmod(c[k], x[k], p->Q);
    ntt_inv(&t, c);
    free(x);
    ntt_free(&t);
}

/* ------------------------------------------------------------------ */
/* rgsw-acc.cpp:57-111  SignedDigitDecompose ("variant A")              */
/* ------------------------------------------------------------------ */
void or_signed_digit_decompose(const or_params* p, const uint64_t* in, uint64_t* out) {
    const uint32_t N = p->N, logG = p->logG, thr = p->numDigitsToThrow;
    const uint32_t digits = p->digitsG - thr;
    const uint64_t Q = p->Q, QHalf = Q >> 1;
    const int64_t Qi = (int64_t)Q;
    const uint32_t sh = 64 - logG; /* gBitsMaxBits = NativeInteger::MaxBits() - gBits */
    for (uint32_t j = 0; j < 2; ++j)
        for (uint32_t k = 0; k < N; ++k) {
            uint64_t t = in[j * N + k];
            int64_t d = t < QHalf ? (int64_t)t : (int64_t)t - Qi;
            int64_t r;
            for (uint32_t i = 0; i < thr; ++i) {
                r = (int64_t)((uint64_t)d << sh) >> sh;
                d = (d - r) >> logG;
            }
            for (uint32_t l = 0; l < digits; ++l) {
                r = (int64_t)((uint64_t)d << sh) >> sh; /* sign-extended low logG bits */
                d -= r;
                d >>= logG;
                if (r < 0) r += Qi;
                out[(size_t)(j + 2 * l) * N + k] = (uint64_t)r;
            }
        }
}

/* ------------------------------------------------------------------ */
/* context                                                             */
/* ------------------------------------------------------------------ */
struct or_ctx {
    or_params p;
    ntt_tab t;
    uint64_t* bsk_ntt; /* [n][2][dG2][2][N] evaluation form (oracle's own NTT) */
    uint64_t* ksk;     /* [N][baseKS][dKS][n+1] */
    uint64_t nboot;
};

or_ctx* or_create(const or_params* p, const uint64_t* bsk_coeff, const uint64_t* ksk) {
    or_ctx* c = (or_ctx*)calloc(1, sizeof(or_ctx));
    c->p = *p;
    ntt_init(&c->t, p->Q, p->N);
    size_t nb = (size_t)p->n * 2 * p->dG2 * 2 * p->N;
    c->bsk_ntt = (uint64_t*)malloc(sizeof(uint64_t) * nb);
    memcpy(c->bsk_ntt, bsk_coeff, sizeof(uint64_t) * nb);
    size_t polys = nb / p->N;
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < polys; ++i) ntt_fwd(&c->t, c->bsk_ntt + i * p->N);
    size_t nk = (size_t)p->N * p->baseKS * p->dKS * (p->n + 1);
    c->ksk = (uint64_t*)malloc(sizeof(uint64_t) * nk);
    memcpy(c->ksk, ksk, sizeof(uint64_t) * nk);
    return c;
}

void or_destroy(or_ctx* c) {
    if (!c) return;
    ntt_free(&c->t);
    free(c->bsk_ntt);
    free(c->ksk);
    free(c);
}

uint64_t or_bootstrap_count(const or_ctx* c) { return c->nboot; }

/* acc <- acc * (X^m - 1) contribution: out += src * (X^m - 1), coefficient form.
 * Monomial table semantics of rgsw-cryptoparameters.h:141-159: m in [0,N) is X^m - 1,
 * m in [N,2N) is -X^(m-N) - 1 (= X^m - 1 since X^N = -1); m == 0 is the zero poly. */
static void add_mul_monomial_minus_one(const or_params* p, const uint64_t* src, uint32_t m, uint64_t* out) {
    const uint32_t N = p->N;
    const uint64_t Q = p->Q;
    if (m == 0) return;
    for (uint32_t k = 0; k < N; ++k) {
        uint32_t e = k + m; /* src[k] X^k * X^m */
        uint64_t v = src[k];
        e %= 2 * N;
        if (e < N) out[e] = addmod(out[e], v, Q);
        else out[e - N] = submod(out[e - N], v, Q);
        out[k] = submod(out[k], v, Q); /* - src */
    }
}

/* One ciphertext of rgsw-acc-cggi.cpp:143-155 / 246-307 with acc kept in coefficient
 * form (the reference keeps it in EVALUATION form; both are the same ring element).
 * work: (dG2 + 4) * N words. */
static void eval_acc_one(const or_ctx* c, const uint64_t* a, uint64_t amod, uint64_t* acc, uint64_t* work) {
    const or_params* p = &c->p;
    const uint32_t N = p->N, n = p->n, dG2 = p->dG2;
    const uint64_t Q = p->Q, M = 2ull * N;
    uint64_t* dct = work;                     /* [dG2][N] */
    uint64_t* s = work + (size_t)dG2 * N;     /* [2 keys][2 polys][N] */
    for (uint32_t i = 0; i < n; ++i) {
        /* rgsw-acc-cggi.cpp:153: mod.ModSub(a[i], mod) * (M / modInt) */
        uint64_t ai = ((amod - a[i] % amod) % amod) * (M / amod);
        uint32_t idxPos = (uint32_t)(ai % M);
        uint32_t idxNeg = (uint32_t)((M - ai) % M); /* M.ModSub(a, M); index M -> 0 */
        or_signed_digit_decompose(p, acc, dct);
        for (uint32_t l = 0; l < dG2; ++l) ntt_fwd(&c->t, dct + (size_t)l * N);
        const uint64_t* ek = c->bsk_ntt + (size_t)i * 2 * dG2 * 2 * N; /* [key][row][poly][N] */
        for (uint32_t key = 0; key < 2; ++key)
            for (uint32_t j = 0; j < 2; ++j) {
                uint64_t* sk = s + (size_t)(key * 2 + j) * N;
                for (uint32_t x = 0; x < N; ++x) {
                    uint64_t sum = 0;
                    for (uint32_t l = 0; l < dG2; ++l)
                        sum = addmod(sum, mulmod(dct[(size_t)l * N + x], ek[((size_t)(key * dG2 + l) * 2 + j) * N + x], Q), Q);
                    sk[x] = sum;
                }
                ntt_inv(&c->t, sk);
            }
        /* acc_j += S0j * (X^idxPos - 1) + S1j * (X^idxNeg - 1) */
        for (uint32_t j = 0; j < 2; ++j) {
            add_mul_monomial_minus_one(p, s + (size_t)(0 * 2 + j) * N, idxPos, acc + (size_t)j * N);
            add_mul_monomial_minus_one(p, s + (size_t)(1 * 2 + j) * N, idxNeg, acc + (size_t)j * N);
        }
    }
    /* extraction transpose (poly.cpp:762-770, automorphism X -> X^-1) on acc0, reduced values */
    uint64_t* t0 = work;
    memcpy(t0, acc, sizeof(uint64_t) * N);
    acc[0] = t0[0];
    for (uint32_t k = 1; k < N; ++k) acc[k] = t0[N - k] == 0 ? 0 : Q - t0[N - k];
}

void or_eval_acc(const or_ctx* c, size_t B, const uint64_t* a, uint64_t amod, uint64_t* acc) {
    const or_params* p = &c->p;
    const size_t wsz = (size_t)(p->dG2 + 4) * p->N;
#pragma omp parallel num_threads(nthreads_for(B))
    {
        uint64_t* work = (uint64_t*)malloc(sizeof(uint64_t) * wsz);
#pragma omp for schedule(dynamic, 1)
        for (size_t s = 0; s < B; ++s) eval_acc_one(c, a + s * p->n, amod, acc + s * 2 * p->N, work);
        free(work);
    }
    ((or_ctx*)c)->nboot += B;
}

/* ModSwitch(qKS) -> KeySwitch -> ModSwitch(fmod) for one extracted ciphertext
 * (lwe-pke.cpp:204-215, 299-321; bootstrapping.cu:73-118) */
static void mkm_one(const or_ctx* c, const uint64_t* ct, uint64_t fmod, uint64_t* out, uint64_t* work) {
    const or_params* p = &c->p;
    const uint32_t N = p->N, n = p->n, bks = p->baseKS, dks = p->dKS;
    const uint64_t qKS = p->qKS;
    uint64_t* x = work; /* N+1 */
    for (uint32_t k = 0; k <= N; ++k) x[k] = or_roundqQ(ct[k], qKS, p->Q);
    uint64_t* a = work + N + 1; /* n */
    for (uint32_t k = 0; k < n; ++k) a[k] = 0;
    uint64_t b = x[N];
    for (uint32_t i = 0; i < N; ++i) {
        uint64_t atmp = x[i];
        for (uint32_t j = 0; j < dks; ++j, atmp /= bks) {
            uint64_t a0 = atmp % bks;
            const uint64_t* row = c->ksk + (((size_t)i * bks + a0) * dks + j) * (n + 1);
            for (uint32_t k = 0; k < n; ++k) a[k] = submod(a[k], row[k], qKS);
            b = submod(b, row[n], qKS);
        }
    }
    for (uint32_t k = 0; k < n; ++k) out[k] = or_roundqQ(a[k], fmod, qKS);
    out[n] = or_roundqQ(b, fmod, qKS);
}

void or_mkm_switch(const or_ctx* c, size_t B, const uint64_t* ct_ext, uint64_t fmod, uint64_t* out) {
    const or_params* p = &c->p;
#pragma omp parallel num_threads(nthreads_for(B))
    {
        uint64_t* work = (uint64_t*)malloc(sizeof(uint64_t) * (p->N + 1 + p->n));
#pragma omp for schedule(dynamic, 4)
        for (size_t s = 0; s < B; ++s) mkm_one(c, ct_ext + s * (p->N + 1), fmod, out + s * (p->n + 1), work);
        free(work);
    }
}

/* ------------------------------------------------------------------ */
/* KAT and valid key generation                                        */
/* ------------------------------------------------------------------ */
uint64_t or_splitmix64(or_rng* r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void or_splitmix_fill(or_rng* r, size_t count, uint64_t mod, uint64_t* out) {
    for (size_t i = 0; i < count; ++i) out[i] = or_splitmix64(r) % mod;
}

uint64_t or_fnv1a64(const uint64_t* w, size_t count) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < count; ++i)
        for (int b = 0; b < 8; ++b) {
            h ^= (w[i] >> (8 * b)) & 0xff;
            h *= 0x100000001b3ull;
        }
    return h;
}

void or_kat_keys(const or_params* p, or_rng* r, uint64_t* bsk, uint64_t* ksk) {
    const size_t nb = (size_t)p->n * 2 * p->dG2 * 2 * p->N;
    for (size_t i = 0; i < nb; ++i) bsk[i] = or_splitmix64(r) % p->Q;
    const size_t nk = (size_t)p->N * p->baseKS * p->dKS * (p->n + 1);
    for (size_t i = 0; i < nk; ++i) ksk[i] = or_splitmix64(r) % p->qKS;
}

static uint64_t rng_uniform(or_rng* r, uint64_t m) { return or_splitmix64(r) % m; }
static int64_t rng_ternary(or_rng* r) { return (int64_t)(or_splitmix64(r) % 3) - 1; }
static int64_t rng_gauss(or_rng* r) {
    /* rounded Gaussian, sigma 3.19 (the reference's STD_DEV, binfhecontext.cpp:133) */
    double u1 = ((or_splitmix64(r) >> 11) + 1.0) * (1.0 / 9007199254740993.0);
    double u2 = (or_splitmix64(r) >> 11) * (1.0 / 9007199254740992.0);
    double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    return (int64_t)llround(3.19 * z);
}
static uint64_t to_mod(int64_t v, uint64_t m) {
    int64_t r = v % (int64_t)m;
    return (uint64_t)(r < 0 ? r + (int64_t)m : r);
}

/* Keys from ONE splitmix64 stream, in this order: s (n ternary), sN (N ternary); per KSK row (i, j, k) its
 * Gaussian (2 draws) then n uniforms; per BSK row (i, key, row) N uniforms then N Gaussians.  Every draw is
 * one or two fixed steps of the counter-based generator (state_k = state_0 + k gamma), so each row reads
 * its own stream position and the rows are filled in parallel (OpenMP) -- the same keys as a sequential
 * walk, bit for bit (round 6: tests/test_oracle_units.py pins the digest; the GPU suite's valid-key tests
 * spent most of their time here). */
static or_rng rng_at(const or_rng* r0, uint64_t draws) {
    or_rng r = {r0->s + draws * 0x9E3779B97F4A7C15ull};
    return r;
}

void or_keygen(const or_params* p, or_rng* r, uint64_t* sk, uint64_t* bsk, uint64_t* ksk) {
    const uint32_t n = p->n, N = p->N, dG2 = p->dG2, bks = p->baseKS, dks = p->dKS;
    const uint64_t Q = p->Q, qKS = p->qKS;
    int64_t* s = (int64_t*)malloc(sizeof(int64_t) * n);
    int64_t* sN = (int64_t*)malloc(sizeof(int64_t) * N);
    for (uint32_t i = 0; i < n; ++i) { s[i] = rng_ternary(r); sk[i] = to_mod(s[i], qKS); }
    for (uint32_t i = 0; i < N; ++i) sN[i] = rng_ternary(r);
    const or_rng r_ksk = *r;
    /* KSK: lwe-pke.cpp:218-295; A[i][j][k] uniform, B = e + sN[i]*j*baseKS^k + <A, s> mod qKS */
    const size_t ksk_rows = (size_t)N * bks * dks, ksk_draws = 2 + (size_t)n;
    uint64_t* smod = (uint64_t*)malloc(sizeof(uint64_t) * n);
    for (uint32_t l = 0; l < n; ++l) smod[l] = to_mod(s[l], qKS);
#pragma omp parallel for schedule(static)
    for (size_t rowi = 0; rowi < ksk_rows; ++rowi) {
        const uint32_t k = (uint32_t)(rowi % dks), j = (uint32_t)((rowi / dks) % bks), i = (uint32_t)(rowi / dks / bks);
        uint64_t pw = 1;
        for (uint32_t z = 0; z < k; ++z) pw = mulmod(pw, bks, qKS);
        or_rng rr = rng_at(&r_ksk, rowi * ksk_draws);
        uint64_t* row = ksk + rowi * (n + 1);
        uint64_t b = addmod(to_mod(rng_gauss(&rr), qKS), mulmod(to_mod(sN[i], qKS), mulmod(j, pw, qKS), qKS), qKS);
        for (uint32_t l = 0; l < n; ++l) {
            row[l] = rng_uniform(&rr, qKS);
            b = addmod(b, mulmod(row[l], smod[l], qKS), qKS);
        }
        row[n] = b;
    }
    free(smod);
    /* BSK: rgsw-acc-cggi.cpp:43-77 (ternary MUX keys) and 213-240 (KeyGenCGGI), coefficient form.
     * row i: (a_i, a_i*sN + e_i); m ? row[i][i&1][0] += G^((i>>1)+throw) */
    const or_rng r_bsk = rng_at(&r_ksk, ksk_rows * ksk_draws);
    const size_t bsk_rows = (size_t)n * 2 * dG2, bsk_draws = 3 * (size_t)N;
    ntt_tab t;
    ntt_init(&t, Q, N);
    uint64_t* sNt = (uint64_t*)malloc(sizeof(uint64_t) * N);  /* NTT(sN mod Q), once */
    for (uint32_t x = 0; x < N; ++x) sNt[x] = to_mod(sN[x], Q);
    ntt_fwd(&t, sNt);
#pragma omp parallel
    {
        uint64_t* prod = (uint64_t*)malloc(sizeof(uint64_t) * N);
#pragma omp for schedule(dynamic, 4)
        for (size_t rowi = 0; rowi < bsk_rows; ++rowi) {
            const uint32_t row = (uint32_t)(rowi % dG2), key = (uint32_t)((rowi / dG2) % 2), i = (uint32_t)(rowi / dG2 / 2);
            const int m = key == 0 ? (s[i] == 1) : (s[i] == -1);
            uint64_t* pa = bsk + (rowi * 2 + 0) * N;
            uint64_t* pb = bsk + (rowi * 2 + 1) * N;
            or_rng rr = rng_at(&r_bsk, rowi * bsk_draws);
            for (uint32_t x = 0; x < N; ++x) pa[x] = rng_uniform(&rr, Q);
            memcpy(prod, pa, sizeof(uint64_t) * N);
            ntt_fwd(&t, prod);
            for (uint32_t x = 0; x < N; ++x) prod[x] = mulmod(prod[x], sNt[x], Q);
            ntt_inv(&t, prod);
            for (uint32_t x = 0; x < N; ++x) pb[x] = addmod(prod[x], to_mod(rng_gauss(&rr), Q), Q);
            if (m) {
                uint64_t g = powmod(p->baseG, (row >> 1) + p->numDigitsToThrow, Q);
                uint64_t* tgt = (row & 1) ? pb : pa;
                tgt[0] = addmod(tgt[0], g, Q);
            }
        }
        free(prod);
    }
    *r = rng_at(&r_bsk, bsk_rows * bsk_draws);  /* the caller's stream continues after the keys */
    ntt_free(&t);
    free(sNt);
    free(s);
    free(sN);
}

/* lwe-pke.cpp:56-88 (sk stored mod qKS; SwitchModulus to `mod` keeps the centred value) */
static uint64_t sk_to_mod(uint64_t v, uint64_t qKS, uint64_t mod) {
    int64_t c = v > qKS / 2 ? (int64_t)v - (int64_t)qKS : (int64_t)v;
    return to_mod(c, mod);
}
void or_encrypt(const or_params* p, or_rng* r, const uint64_t* sk, int64_t m, uint64_t ptxt_mod, uint64_t mod,
                uint64_t* ct) {
    const uint32_t n = p->n;
    uint64_t b = addmod(mulmod(to_mod(m % (int64_t)ptxt_mod, ptxt_mod), mod / ptxt_mod, mod), to_mod(rng_gauss(r), mod), mod);
    for (uint32_t i = 0; i < n; ++i) {
        ct[i] = rng_uniform(r, mod);
        b = addmod(b, mulmod(ct[i], sk_to_mod(sk[i], p->qKS, mod), mod), mod);
    }
    ct[n] = b;
}
/* lwe-pke.cpp:92-130 */
int64_t or_decrypt(const or_params* p, const uint64_t* sk, const uint64_t* ct, uint64_t ptxt_mod, uint64_t mod) {
    uint64_t inner = 0;
    for (uint32_t i = 0; i < p->n; ++i) inner = addmod(inner, mulmod(ct[i], sk_to_mod(sk[i], p->qKS, mod), mod), mod);
    uint64_t rr = submod(ct[p->n], inner, mod);
    rr = addmod(rr, mod / (ptxt_mod * 2), mod);
    return (int64_t)(((u128)ptxt_mod * rr) / mod);
}

/* ------------------------------------------------------------------ */
/* vector scheme glue (binfhe-base-scheme.cpp:598-1277)                */
/* ------------------------------------------------------------------ */
/* gate constants, rgsw-cryptoparameters.h:130-137 */
static uint64_t gate_const(int gate, uint64_t q) {
    static const uint64_t k[] = {5, 7, 1, 3, 5, 1};
    return k[gate] * (q >> 3);
}

typedef uint64_t (*lut_fn)(uint64_t x, uint64_t q, uint64_t Q, const void* ctx, size_t idx);

/* BootstrapGateCore (vector) binfhe-base-scheme.cpp:1087-1145 + extraction :664-672 + MKM.
 * ct [B][n+1] mod q (already combined); out [B][n+1] mod q */
static void bootstrap_gate(const or_ctx* c, int gate, size_t B, const uint64_t* ct, uint64_t q, uint64_t* out) {
    const or_params* p = &c->p;
    const uint32_t N = p->N, n = p->n;
    const uint64_t Q = p->Q, Q8 = Q / 8 + 1, Q8Neg = Q - Q8;
    uint64_t* acc = (uint64_t*)calloc((size_t)B * 2 * N, sizeof(uint64_t));
    uint64_t* a = (uint64_t*)malloc(sizeof(uint64_t) * B * n);
    const uint64_t qHalf = q >> 1, q1 = gate_const(gate, q), q2 = addmod(q1, qHalf, q);
    const uint64_t factor = 2ull * N / q;
    for (size_t s = 0; s < B; ++s) {
        const uint64_t* x = ct + s * (n + 1);
        memcpy(a + s * n, x, sizeof(uint64_t) * n);
        uint64_t b = x[n];
        uint64_t* m = acc + s * 2 * N + N;
        for (uint64_t j = 0; j < qHalf; ++j) {
            uint64_t temp = submod(b, j, q);
            if (q1 < q2) m[j * factor] = (temp >= q1 && temp < q2) ? Q8Neg : Q8;
            else m[j * factor] = (temp >= q2 && temp < q1) ? Q8 : Q8Neg;
        }
    }
    or_eval_acc(c, B, a, q, acc);
    uint64_t* ext = (uint64_t*)malloc(sizeof(uint64_t) * B * (N + 1));
    for (size_t s = 0; s < B; ++s) {
        memcpy(ext + s * (N + 1), acc + s * 2 * N, sizeof(uint64_t) * N);
        ext[s * (N + 1) + N] = addmod(Q8, acc[s * 2 * N + N], Q); /* b = Q/8+1 + acc1[0] */
    }
    or_mkm_switch(c, B, ext, q, out);
    free(ext);
    free(a);
    free(acc);
}

/* BootstrapFuncCore + BootstrapFunc (vector) binfhe-base-scheme.cpp:1147-1211 */
static void bootstrap_func(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t ctmod, lut_fn f, const void* fctx,
                           uint64_t fmod, uint64_t* out) {
    const or_params* p = &c->p;
    const uint32_t N = p->N, n = p->n;
    const uint64_t Q = p->Q;
    uint64_t* acc = (uint64_t*)calloc((size_t)B * 2 * N, sizeof(uint64_t));
    uint64_t* a = (uint64_t*)malloc(sizeof(uint64_t) * B * n);
    const uint64_t factor = 2ull * N / ctmod, scale = Q / fmod;
    for (size_t s = 0; s < B; ++s) {
        const uint64_t* x = ct + s * (n + 1);
        memcpy(a + s * n, x, sizeof(uint64_t) * n);
        uint64_t b = x[n];
        uint64_t* m = acc + s * 2 * N + N;
        for (uint64_t j = 0; j < (ctmod >> 1); ++j) {
            uint64_t temp = submod(b % ctmod, j, ctmod);
            m[j * factor] = scale * f(temp, ctmod, fmod, fctx, s);
        }
    }
    or_eval_acc(c, B, a, ctmod, acc);
    uint64_t* ext = (uint64_t*)malloc(sizeof(uint64_t) * B * (N + 1));
    for (size_t s = 0; s < B; ++s) {
        memcpy(ext + s * (N + 1), acc + s * 2 * N, sizeof(uint64_t) * N);
        ext[s * (N + 1) + N] = acc[s * 2 * N + N];
    }
    or_mkm_switch(c, B, ext, fmod, out);
    free(ext);
    free(a);
    free(acc);
}

/* the lambdas of binfhe-base-scheme.cpp (x, q, Q) -> value; parameter names as there */
static uint64_t f_half(uint64_t x, uint64_t q, uint64_t Q, const void* u, size_t i) { /* f0 / f1 */
    (void)u; (void)i;
    return x < q / 2 ? Q - q / 4 : q / 4;
}
static uint64_t f_floor2(uint64_t x, uint64_t q, uint64_t Q, const void* u, size_t i) { /* f2, :973-980 */
    (void)u; (void)i;
    if (x < q / 4) return Q - q / 2 - x;
    else if (q / 4 <= x && x < 3 * q / 4) return x;
    return Q + q / 2 - x;
}
static uint64_t f_sign3(uint64_t x, uint64_t q, uint64_t Q, const void* u, size_t i) { /* f3, :1029-1031 */
    (void)u; (void)i;
    return x < q / 2 ? Q / 4 : Q - Q / 4;
}
typedef struct { const uint64_t* lut; size_t stride; } lut_ctx; /* stride 0: shared LUT */
static uint64_t f_lut(uint64_t x, uint64_t q, uint64_t Q, const void* u, size_t i) { /* fLUT */
    (void)q; (void)Q;
    const lut_ctx* L = (const lut_ctx*)u;
    return L->lut[i * L->stride + x];
}
static uint64_t f_lut1(uint64_t x, uint64_t q, uint64_t Q, const void* u, size_t i) { /* fLUT1 / fLUT2 */
    const lut_ctx* L = (const lut_ctx*)u;
    const uint64_t* lut = L->lut + i * L->stride;
    return x < q / 2 ? lut[x] : Q - lut[x - q / 2];
}
/* LUT2 = LUT ++ LUT (binfhe-base-scheme.cpp:717-718) */
typedef struct { const uint64_t* lut; size_t stride; uint64_t len; } lut2_ctx;
static uint64_t f_lut2(uint64_t x, uint64_t q, uint64_t Q, const void* u, size_t i) {
    const lut2_ctx* L = (const lut2_ctx*)u;
    const uint64_t* lut = L->lut + i * L->stride;
    uint64_t y = x < q / 2 ? x : x - q / 2;
    uint64_t v = lut[y % L->len];
    return x < q / 2 ? v : Q - v;
}

/* LWE helpers (lwe-pke.cpp:175-201, lwe-ciphertext.h:120-124); ct [n+1] */
static void lwe_add_const(uint64_t* ct, uint32_t n, uint64_t c, uint64_t mod) { ct[n] = addmod(ct[n], c, mod); }
static void lwe_sub_const(uint64_t* ct, uint32_t n, uint64_t c, uint64_t mod) { ct[n] = submod(ct[n], c, mod); }
static void lwe_set_modulus(uint64_t* ct, uint32_t n, uint64_t mod) {
    for (uint32_t i = 0; i <= n; ++i) ct[i] %= mod;
}

int or_eval_bin_gate(const or_ctx* c, int gate, size_t B, const uint64_t* ct1, const uint64_t* ct2, uint64_t q,
                     uint64_t* out) {
    const uint32_t n = c->p.n;
    if (B == 0) return -1;
    if (gate < 0 || gate > OR_XNOR) return -2;
    const size_t L = (size_t)B * (n + 1);
    if (gate == OR_XOR || gate == OR_XNOR) {
        uint64_t* n1 = (uint64_t*)malloc(sizeof(uint64_t) * L);
        uint64_t* n2 = (uint64_t*)malloc(sizeof(uint64_t) * L);
        uint64_t* t1 = (uint64_t*)malloc(sizeof(uint64_t) * L);
        uint64_t* t2 = (uint64_t*)malloc(sizeof(uint64_t) * L);
        for (size_t i = 0; i < L; ++i) {
            size_t k = i % (n + 1);
            if (k < n) { n1[i] = ct1[i] == 0 ? 0 : q - ct1[i]; n2[i] = ct2[i] == 0 ? 0 : q - ct2[i]; }
            else { n1[i] = submod(q >> 2, ct1[i], q); n2[i] = submod(q >> 2, ct2[i], q); }
        }
        or_eval_bin_gate(c, OR_AND, B, ct1, n2, q, t1);
        or_eval_bin_gate(c, OR_AND, B, n1, ct2, q, t2);
        or_eval_bin_gate(c, OR_OR, B, t1, t2, q, out);
        if (gate == OR_XNOR)
            for (size_t i = 0; i < L; ++i) {
                size_t k = i % (n + 1);
                out[i] = k < n ? (out[i] == 0 ? 0 : q - out[i]) : submod(q >> 2, out[i], q);
            }
        free(n1); free(n2); free(t1); free(t2);
        return 0;
    }
    uint64_t* prep = (uint64_t*)malloc(sizeof(uint64_t) * L);
    for (size_t i = 0; i < L; ++i) {
        if (gate == OR_XOR_FAST || gate == OR_XNOR_FAST) {
            uint64_t d = submod(ct1[i], ct2[i], q);
            prep[i] = addmod(d, d, q);
        } else {
            prep[i] = addmod(ct1[i], ct2[i], q);
        }
    }
    bootstrap_gate(c, gate, B, prep, q, out);
    free(prep);
    return 0;
}

/* binfhe-base-scheme.cpp:162-186 */
static int check_input_function(const uint64_t* lut, uint64_t len, uint64_t mod) {
    int ret = 0;
    uint64_t h = len / 2;
    if (lut[0] == mod - lut[h]) {
        for (uint64_t i = 1; i < h; ++i)
            if (lut[i] != mod - lut[h + i]) { ret = 2; break; }
    } else if (lut[0] == lut[h]) {
        ret = 1;
        for (uint64_t i = 1; i < h; ++i)
            if (lut[i] != lut[h + i]) { ret = 2; break; }
    } else {
        ret = 2;
    }
    return ret;
}

static int eval_func_impl(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t q, const uint64_t* luts,
                          size_t stride, uint64_t* out) {
    const uint32_t n = c->p.n, N = c->p.N;
    const uint64_t beta = 128;
    if (B == 0) return -1;
    const size_t L = (size_t)B * (n + 1);
    int prop = check_input_function(luts, q, q);
    uint64_t* ct1 = (uint64_t*)malloc(sizeof(uint64_t) * L);
    memcpy(ct1, ct, sizeof(uint64_t) * L);
    if (prop == 0) {
        lut_ctx Lc = {luts, stride};
        for (size_t s = 0; s < B; ++s) lwe_add_const(ct1 + s * (n + 1), n, beta, q);
        bootstrap_func(c, B, ct1, q, f_lut, &Lc, q, out);
        free(ct1);
        return 0;
    }
    if (prop == 2) {
        if (q > N) { free(ct1); return -3; }
        const uint64_t dq = q << 1;
        /* ct1 modulus raised to dq (values unchanged); ct2 = ct1 + beta mod dq */
        uint64_t* ct2 = (uint64_t*)malloc(sizeof(uint64_t) * L);
        uint64_t* ct3 = (uint64_t*)malloc(sizeof(uint64_t) * L);
        memcpy(ct2, ct1, sizeof(uint64_t) * L);
        for (size_t s = 0; s < B; ++s) lwe_add_const(ct2 + s * (n + 1), n, beta, dq);
        bootstrap_func(c, B, ct2, dq, f_half, NULL, dq, ct3);
        for (size_t s = 0; s < B; ++s) {
            uint64_t* x1 = ct1 + s * (n + 1);
            uint64_t* x3 = ct3 + s * (n + 1);
            for (uint32_t k = 0; k <= n; ++k) x3[k] = submod(x1[k], x3[k], dq); /* EvalSubEq2 */
            lwe_add_const(x3, n, beta, dq);
            lwe_sub_const(x3, n, q >> 1, dq);
        }
        lut2_ctx L2 = {luts, stride, q};
        bootstrap_func(c, B, ct3, dq, f_lut2, &L2, dq, out);
        for (size_t s = 0; s < B; ++s) lwe_set_modulus(out + s * (n + 1), n, q);
        free(ct2);
        free(ct3);
        free(ct1);
        return 0;
    }
    /* periodic */
    for (size_t s = 0; s < B; ++s) lwe_add_const(ct1 + s * (n + 1), n, beta, q);
    uint64_t* ct2 = (uint64_t*)malloc(sizeof(uint64_t) * L);
    bootstrap_func(c, B, ct1, q, f_half, NULL, q, ct2);
    for (size_t s = 0; s < B; ++s) {
        const uint64_t* x0 = ct + s * (n + 1);
        uint64_t* x2 = ct2 + s * (n + 1);
        for (uint32_t k = 0; k <= n; ++k) x2[k] = submod(x0[k], x2[k], q);
        lwe_add_const(x2, n, beta, q);
        lwe_sub_const(x2, n, q >> 2, q);
    }
    lut_ctx Lc = {luts, stride};
    bootstrap_func(c, B, ct2, q, f_lut1, &Lc, q, out);
    free(ct2);
    free(ct1);
    return 0;
}

int or_eval_func(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t q, const uint64_t* lut, uint64_t* out) {
    return eval_func_impl(c, B, ct, q, lut, 0, out);
}
int or_eval_func_vec(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t q, const uint64_t* luts, uint64_t* out) {
    return eval_func_impl(c, B, ct, q, luts, q, out);
}

/* binfhe-base-scheme.cpp:926-987 */
int or_eval_floor(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint32_t roundbits, uint64_t* out) {
    const uint32_t n = c->p.n;
    const uint64_t beta = 128;
    if (B == 0) return -1;
    const uint64_t q = roundbits == 0 ? c->p.q : beta * 2 * (1ull << roundbits);
    const size_t L = (size_t)B * (n + 1);
    uint64_t* ct1m = (uint64_t*)malloc(sizeof(uint64_t) * L);
    uint64_t* ct2 = (uint64_t*)malloc(sizeof(uint64_t) * L);
    memcpy(out, ct, sizeof(uint64_t) * L); /* out plays ct1 */
    for (size_t s = 0; s < B; ++s) lwe_add_const(out + s * (n + 1), n, beta, mod);
    memcpy(ct1m, out, sizeof(uint64_t) * L);
    for (size_t s = 0; s < B; ++s) lwe_set_modulus(ct1m + s * (n + 1), n, q);
    bootstrap_func(c, B, ct1m, q, f_half, NULL, mod, ct2);
    for (size_t i = 0; i < L; ++i) out[i] = submod(out[i], ct2[i], mod);
    memcpy(ct1m, out, sizeof(uint64_t) * L);
    for (size_t s = 0; s < B; ++s) lwe_set_modulus(ct1m + s * (n + 1), n, q);
    bootstrap_func(c, B, ct1m, q, f_floor2, NULL, mod, ct2);
    for (size_t i = 0; i < L; ++i) out[i] = submod(out[i], ct2[i], mod);
    free(ct1m);
    free(ct2);
    return 0;
}

/* ModSwitch (lwe-pke.cpp:204-215) of a whole batch, in place */
static void modswitch_batch(uint64_t* ct, size_t B, uint32_t n, uint64_t newmod, uint64_t oldmod) {
    for (size_t i = 0; i < B * (n + 1); ++i) ct[i] = or_roundqQ(ct[i], newmod, oldmod);
}

/* binfhe-base-scheme.cpp:989-1037 (vector EvalSign: no mod<=q guard, single key) */
int or_eval_sign(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint64_t* out) {
    const uint32_t n = c->p.n;
    const uint64_t beta = 128, q = c->p.q;
    if (B == 0) return -1;
    const size_t L = (size_t)B * (n + 1);
    uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * L);
    uint64_t* fl = (uint64_t*)malloc(sizeof(uint64_t) * L);
    memcpy(tmp, ct, sizeof(uint64_t) * L);
    while (mod > q) {
        or_eval_floor(c, B, tmp, mod, 0, fl);
        uint64_t newmod = mod / q * 2 * beta;
        memcpy(tmp, fl, sizeof(uint64_t) * L);
        modswitch_batch(tmp, B, n, newmod, mod);
        mod = newmod;
    }
    for (size_t s = 0; s < B; ++s) lwe_add_const(tmp + s * (n + 1), n, beta, mod);
    bootstrap_func(c, B, tmp, mod, f_sign3, NULL, q, out);
    for (size_t s = 0; s < B; ++s) lwe_sub_const(out + s * (n + 1), n, q >> 2, q);
    free(tmp);
    free(fl);
    return 0;
}

/* binfhe-base-scheme.cpp:1039-1085 */
int or_eval_decomp(const or_ctx* c, size_t B, const uint64_t* ct, uint64_t mod, uint32_t max_digits, uint64_t* out,
                   uint64_t* moduli) {
    const uint32_t n = c->p.n;
    const uint64_t beta = 128, q = c->p.q;
    if (B == 0) return -1;
    if (mod <= q) return -2;
    const size_t L = (size_t)B * (n + 1), row = (size_t)(n + 1);
    uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * L);
    uint64_t* fl = (uint64_t*)malloc(sizeof(uint64_t) * L);
    memcpy(tmp, ct, sizeof(uint64_t) * L);
    uint32_t d = 0;
    while (mod > q) {
        if (d >= max_digits) { free(tmp); free(fl); return -4; }
        for (size_t s = 0; s < B; ++s) {
            uint64_t* o = out + (s * max_digits + d) * row;
            memcpy(o, tmp + s * row, sizeof(uint64_t) * row);
            lwe_set_modulus(o, n, q);
        }
        moduli[d++] = q;
        or_eval_floor(c, B, tmp, mod, 0, fl);
        uint64_t newmod = mod / q * 2 * beta;
        memcpy(tmp, fl, sizeof(uint64_t) * L);
        modswitch_batch(tmp, B, n, newmod, mod);
        mod = newmod;
    }
    if (d >= max_digits) { free(tmp); free(fl); return -4; }
    for (size_t s = 0; s < B; ++s) memcpy(out + (s * max_digits + d) * row, tmp + s * row, sizeof(uint64_t) * row);
    moduli[d++] = mod;
    free(tmp);
    free(fl);
    return (int)d;
}
