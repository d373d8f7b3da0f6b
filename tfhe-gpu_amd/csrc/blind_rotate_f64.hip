// blind_rotate_f64.hip -- CGGI blind rotation in exact FP64 integer arithmetic for
// 2^32 <= Q < 2^50 (STD192(_OPT), STD192Q(_OPT), STD128Q(_OPT); N = 2048, top digit folded).
//
// Same math as the generic kernel (rgsw-acc-cggi.cpp:246-307, rgsw-acc.cpp:57-111), but
// every NTT-domain value is an integer held exactly in a double, so a modular product is
// six FP64 instructions instead of a ~18-instruction u64 Shoup product, and keys and
// twiddles need no Shoup companions:
//     h = a*b (rounded), l = fma(a, b, -h)          a*b = h + l exactly
//     q = rint(h / Q),   r = fma(-q, Q, h) + l      r = a*b - qQ exactly, |r| <~ Q/2
// Exactness holds while |a*b| < 2^102 and every sum stays below 2^53.  Q < 2^40 (RED =
// false): no reduction inside the transforms; Q < 2^50 (RED = true, STD128Q class): the
// reductions tools/bounds_f64.py places (x - rint(x/Q) Q, three instructions).  Keys and
// tables are centred (|x| <= Q/2); the accumulator is a centred double.
// Kernels: k_blind_rotate_f64w (one 512-thread workgroup per ciphertext, wave-local passes) and
// k_blind_rotate_f64wduo (STD128Q class, two workgroups per ciphertext for small batches).
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {
namespace {


typedef double v2d __attribute__((ext_vector_type(2)));  // one 16-byte buffer load: two doubles
struct F64Const {
    double Q, Qinv;
    int64_t Qi;
    double Ninv;  // N^-1 mod Q, centred (FOLD)
    double wfac;  // 2^(gL) N^-1 mod Q, centred (WRAP)
};

// Top-digit elimination (FOLD), as in the specialised STD128 kernel (blind_rotate_fast4.hip):
// with thr = 0 and a top digit that is always the exact remainder, c = sum_l 2^(gl) d_l, so
//   sum_l D_l W_l = sum_{l<L-1} D_l (W_l - 2^-(g(L-1-l)) W_top) + C' (N 2^-(g(L-1)) W_top)
// with C' = N^-1 NTT(acc) kept in registers (C' += S every round, S the NTT-domain increment;
// the BSK carries N^-1).  One forward transform of both polynomials fewer per round.
// WRAP: when the top digit is not always exact (STD128Q: Q = 2^50 - 2^14 + 1, g = 25, the
// centred c in [2^49 - 2^24, Q/2) leaves a residual w = 1 after the last signed digit), the
// reference's digits sum to c - 2^(gL) w, so the round uses C' - 2^(gL) N^-1 NTT(w) in place
// of C'.  w is almost always 0 (about 2^-14 of rounds have a w != 0 coefficient); a
// workgroup-uniform vote skips the correction otherwise.
struct F64Fold {
    uint64_t hc[8];  // l < L-1: 2^-(g(L-1-l)); l = L-1: N 2^-(g(L-1))  (mod Q)
    uint32_t L;
    uint32_t on;
};

__device__ __forceinline__ double fmodmul(double a, double b, const F64Const& K) {
    return fmodmul_f64(a, b, K.Q, K.Qinv);  // device_math.hpp
}

__device__ __forceinline__ double fred(double x, const F64Const& K) {
    return __fma_rn(-__builtin_rint(__dmul_rn(x, K.Qinv)), K.Q, x);
}

// ---- N = 2048: radix-8 register passes over a swizzled LDS buffer -------------------------
// One thread owns 8 elements of ONE polynomial per pass (threads 0..TH/2-1 polynomial 0), so a
// transform is four passes -- stages (0-2) (3-5) (6-8) radix-8 and (9-10) two radix-4 units --
// with four barriers instead of six, and a third fewer LDS round trips.  The buffer is stored
// at swz(x): bits 0-4 of x XOR f(bits 5-7), which makes every pass's 64-bit LDS accesses, and
// the slot-per-lane accesses of the rest of the kernel, conflict-free
// (tools/lds_layouts_f64.py checks every access pattern and the index algebra).
__device__ __forceinline__ uint32_t swz(uint32_t x) {
    const uint32_t c = (x >> 5) & 7;
    return x ^ (c << 2) ^ (c & 3);
}
__device__ __forceinline__ void ct_bf(double& a, double& b, double w, const F64Const& K) {
    const double v = fmodmul(b, w, K);
    b = __dsub_rn(a, v), a = __dadd_rn(a, v);
}
__device__ __forceinline__ void gs_bf(double& a, double& b, double w, const F64Const& K) {
    const double d = __dsub_rn(a, b);
    a = __dadd_rn(a, b), b = fmodmul(d, w, K);
}

// Element addresses of a pass: ad[k] = swz(x_k) from one swizzled base and one XOR per
// element (x_k's varying bits never mix with the swizzle's inputs in an add):
//   pass A  x = tau + 256k:          swz(tau) + 256k
//   pass B  x = 256b + o + 32k:      ((256b + o) ^ f(k)) + 32k,  f(c) = (c << 2) ^ (c & 3)
//   pass C  x = 32b + o + 4k, o < 4: swz(32b + o) ^ 4k
//   unit    x = 4u + k, k < 4:       swz(4u) ^ k
__device__ __forceinline__ uint32_t swzf(uint32_t c) { return (c << 2) ^ (c & 3); }

// forward CT stages s0, s0+1, s0+2 (m0 = 2^s0) on the 8 elements at ad[]; g = block
__device__ __forceinline__ void f64_r8_fwd_core(double (&v)[8], uint32_t m0, uint32_t g, const double* psi,
                                                const F64Const& K) {
    const double w0 = psi[m0 + g];
#pragma unroll
    for (int k = 0; k < 4; ++k) ct_bf(v[k], v[k + 4], w0, K);
    const double2 w1 = *(const double2*)(psi + 2 * m0 + 2 * g);
    ct_bf(v[0], v[2], w1.x, K), ct_bf(v[1], v[3], w1.x, K);
    ct_bf(v[4], v[6], w1.y, K), ct_bf(v[5], v[7], w1.y, K);
    const double2 w2 = *(const double2*)(psi + 4 * m0 + 4 * g);
    const double2 w3 = *(const double2*)(psi + 4 * m0 + 4 * g + 2);
    ct_bf(v[0], v[1], w2.x, K), ct_bf(v[2], v[3], w2.y, K);
    ct_bf(v[4], v[5], w3.x, K), ct_bf(v[6], v[7], w3.y, K);
}
template <bool RED>
__device__ __forceinline__ void f64_r8_fwd(double* p, const uint32_t (&ad)[8], uint32_t m0, uint32_t g,
                                           const double* psi, const F64Const& K) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p[ad[k]];
    f64_r8_fwd_core(v, m0, g, psi, K);
#pragma unroll
    for (int k = 0; k < 8; ++k) p[ad[k]] = RED ? fred(v[k], K) : v[k];
}

// inverse GS stages h0, 2h0, 4h0 on the 8 elements at ad[]; g = block (8 h0 elements), m = N/(2h0).
// f64_r8_inv (RED) reduces all 8 outputs: with only the sums (k < 4) reduced, a later pass could
// take 8 unreduced products (up to ~1.5 Q each for Q near 2^50) and sum past 2^53
// (tools/bounds_f64.py walks the schedule element by element)
__device__ __forceinline__ void f64_r8_inv_core(double (&v)[8], uint32_t m, uint32_t g, const double* ipsi,
                                                const F64Const& K) {
    const double2 w0 = *(const double2*)(ipsi + m + 4 * g);
    const double2 w1 = *(const double2*)(ipsi + m + 4 * g + 2);
    gs_bf(v[0], v[1], w0.x, K), gs_bf(v[2], v[3], w0.y, K);
    gs_bf(v[4], v[5], w1.x, K), gs_bf(v[6], v[7], w1.y, K);
    const double2 w2 = *(const double2*)(ipsi + (m >> 1) + 2 * g);
    gs_bf(v[0], v[2], w2.x, K), gs_bf(v[1], v[3], w2.x, K);
    gs_bf(v[4], v[6], w2.y, K), gs_bf(v[5], v[7], w2.y, K);
    const double w3 = ipsi[(m >> 2) + g];
#pragma unroll
    for (int k = 0; k < 4; ++k) gs_bf(v[k], v[k + 4], w3, K);
}
template <bool RED>
__device__ __forceinline__ void f64_r8_inv(double* p, const uint32_t (&ad)[8], uint32_t m, uint32_t g,
                                           const double* ipsi, const F64Const& K) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p[ad[k]];
    f64_r8_inv_core(v, m, g, ipsi, K);
#pragma unroll
    for (int k = 0; k < 8; ++k) p[ad[k]] = RED ? fred(v[k], K) : v[k];
}

__device__ __forceinline__ void ad_A(uint32_t tau, uint32_t (&ad)[8]) {
    const uint32_t a0 = swz(tau);
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) ad[k] = a0 + 256 * k;
}
__device__ __forceinline__ void ad_B(uint32_t tau, uint32_t (&ad)[8]) {
    const uint32_t b0 = ((tau >> 5) << 8) + (tau & 31);
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) ad[k] = (b0 ^ swzf(k)) + 32 * k;
}
__device__ __forceinline__ void ad_C(uint32_t tau, uint32_t (&ad)[8]) {
    const uint32_t c0 = swz(((tau >> 2) << 5) + (tau & 3));
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) ad[k] = c0 ^ (4 * k);
}

// tau, laundered so that no pass's addresses are hoisted out of the round loop (they would
// stay live across the whole kernel and spill)
__device__ __forceinline__ uint32_t f64_tau() {
    uint32_t tau = threadIdx.x & 255;
    asm volatile("" : "+v"(tau));
    return tau;
}

// ---- N = 2048, wave-local passes (f64w; the sf2 design of blind_rotate_generic.hip) ----------
// Wave w owns the 256-element block w of both polynomials after pass A: passes B, C and the
// units run in wave w without workgroup barriers, the units leave slots 4u .. 4u+3 (u = 64w + l)
// of both polynomials in registers, and the products (32-byte key rows per lane), the C' update,
// the monomial factors and the inverse units stay in registers.  One barrier per forward
// transform (plus one before each further digit's pass A), one per inverse.
__device__ __forceinline__ void f64w_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// TO_LDS: the units' outputs stay in the buffer (slots 4u .. 4u+3 of the wave's block, read back
// by the products of this wave) instead of registers
// DELAY (fault probe, see k_blind_rotate_f64w): waves 1.. sleep between passes B and C
// RED: one reduction, after pass B (stage 5): inputs |x| <= Q/2 (digits, C', the WRAP digit) stay
// below 6.7 Q < 2^53 for every Q < 2^50 and leave at most 5.1 Q, which the products take as
// fmodmul operands (tools/bounds_f64.py walks the worst case; round 2 reduced after every pass)
template <bool RED, bool TO_LDS = false, bool DELAY = false>
__device__ __forceinline__ void f64w_ntt_fwd(double* buf, double (&v)[8], double (&d)[2][4], const double* psi,
                                             const F64Const& K) {
    constexpr uint32_t N = 2048;
    const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
    {
        const uint32_t tau = f64_tau();
        double* p = buf + (t >> 8) * N;
        uint32_t ad[8];
        ad_A(tau, ad);
        f64_r8_fwd_core(v, 1, 0, psi, K);
#pragma unroll
        for (int k = 0; k < 8; ++k) p[ad[k]] = v[k];
    }
    __syncthreads();
    uint32_t tw = (w << 5) | (l & 31);
    asm volatile("" : "+v"(tw));
    double* p = buf + (l >> 5) * N;
    {
        uint32_t ad[8];
        ad_B(tw, ad);
        f64_r8_fwd<RED>(p, ad, 8, tw >> 5, psi, K);
    }
    f64w_sync();
    if constexpr (DELAY) {
        if (w != 0)
            for (int z = 0; z < 32; ++z) __builtin_amdgcn_s_sleep(127);
    }
    {
        uint32_t ad[8];
        ad_C(tw, ad);
        f64_r8_fwd<false>(p, ad, 64, tw >> 2, psi, K);
    }
    f64w_sync();
    const uint32_t u = (w << 6) | l, u0 = swz(4 * u);
    const double wa = psi[N / 4 + u];
    const double2 wb = *(const double2*)(psi + N / 2 + 2 * u);
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // stages 9 (h = 2) and 10 (h = 1) on slots 4u .. 4u+3
        const double* pq = buf + q * N;
        double v0 = pq[u0], v1 = pq[u0 ^ 1], v2 = pq[u0 ^ 2], v3 = pq[u0 ^ 3];
        ct_bf(v0, v2, wa, K), ct_bf(v1, v3, wa, K);
        ct_bf(v0, v1, wb.x, K), ct_bf(v2, v3, wb.y, K);
        if constexpr (TO_LDS) {
            double* pw = buf + q * N;
            pw[u0] = v0, pw[u0 ^ 1] = v1, pw[u0 ^ 2] = v2, pw[u0 ^ 3] = v3;
        } else {
            d[q][0] = v0, d[q][1] = v1, d[q][2] = v2, d[q][3] = v3;
        }
    }
    if constexpr (TO_LDS) f64w_sync();
}

template <bool RED>
__device__ __forceinline__ void f64w_ntt_inv(double* buf, const double (&s)[2][4], double (&v)[8],
                                             const double* ipsi, const F64Const& K) {
    constexpr uint32_t N = 2048;
    const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
    const uint32_t u = (w << 6) | l, u0 = swz(4 * u);
    const double2 wb = *(const double2*)(ipsi + N / 2 + 2 * u);
    const double wa = ipsi[N / 4 + u];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        double* pq = buf + q * N;
        double v0 = s[q][0], v1 = s[q][1], v2 = s[q][2], v3 = s[q][3];
        gs_bf(v0, v1, wb.x, K), gs_bf(v2, v3, wb.y, K);
        gs_bf(v0, v2, wa, K), gs_bf(v1, v3, wa, K);
        if constexpr (RED) v0 = fred(v0, K), v1 = fred(v1, K);
        pq[u0] = v0, pq[u0 ^ 1] = v1, pq[u0 ^ 2] = v2, pq[u0 ^ 3] = v3;
    }
    f64w_sync();
    uint32_t tw = (w << 5) | (l & 31);
    asm volatile("" : "+v"(tw));
    double* p = buf + (l >> 5) * N;
    {
        uint32_t ad[8];
        ad_C(tw, ad);
        f64_r8_inv<RED>(p, ad, 256, tw >> 2, ipsi, K);
    }
    f64w_sync();
    {
        uint32_t ad[8];
        ad_B(tw, ad);
        f64_r8_inv<RED>(p, ad, 32, tw >> 5, ipsi, K);
    }
    __syncthreads();
    const uint32_t tau = f64_tau();
    const double* pa = buf + (t >> 8) * N;
    uint32_t ad[8];
    ad_A(tau, ad);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = pa[ad[k]];
    f64_r8_inv_core(v, 4, 0, ipsi, K);
}

// FOLD (thr = 0) only; LD = transformed digits (digits - 1), WRAP as in k_blind_rotate_f64.
// Monomial factors psi^(+-e) - 1 of the lane's 4 slots: two LDS table products once per round
// (then one product per use).  Round 3 measured the alternatives and removed them (round 4): gathers
// from the 2N-entry memory table at each use (STD192 474 ms), table products at each use (385 ms),
// the 8 gathers once per round (357 ms), against 315-323 ms (profiles/r02ae, r03i).
// PROBE (test library only, TFHE_TEST_PROBES; tests/test_gpu_f64w_race.py): bit 1 delays waves 1..
// inside the prologue's C' transform (between passes B and C), bit 0 omits the barrier after it --
// together they reproduce the round-0 race of the round-2 kernel; bit 2 (timing only) drops the
// barrier before each further digit's pass A; 6 (fault injection, tests/test_bench_cli.py) flips bit 40 of
// ciphertext 0's acc1[0] (the extracted b: large enough to survive every modulus switch after it)
// RESCUE (launched behind every f64wduo launch): only the ciphertexts whose duo pair timed out (the pair's
// failed word, kernels.hpp DuoBuf) run, from their saved inputs; the others exit at once
#ifndef F64W_KPRE
#define F64W_KPRE 0
#endif
template <bool RED, bool WRAP, int LD, int PROBE = 0, bool RESCUE = false>
__global__ void __launch_bounds__(512, 4)
k_blind_rotate_f64w(BRParams P, F64Const K, const double* __restrict__ tabs, const uint32_t* __restrict__ /*eidx*/,
                    const uint64_t* __restrict__ a, uint64_t amod, uint64_t* __restrict__ acc_io,
                    const uint32_t* __restrict__ rescue_failed = nullptr, const uint64_t* __restrict__ rescue_src = nullptr) {
    extern __shared__ __align__(16) double lds_d[];
    constexpr uint32_t N = 2048, TH = 512, CN = 4;
    if constexpr (RESCUE) {
        if (__hip_atomic_load(const_cast<uint32_t*>(rescue_failed + (size_t)blockIdx.x * 64 + 1), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT) == 0)
            return;  // uniform: the pair finished
    }
    double* psi = lds_d;
    double* ipsi = lds_d + N;
    double* buf = lds_d + 2 * N;  // [2][N]
    double* mt = lds_d + 4 * N;   // monomial tables (k_blind_rotate_f64)
    __shared__ int wflag[2];
    const uint32_t t = threadIdx.x, twoN = 2 * N, logG = P.logG;
    const uint32_t u4 = 4 * (((t >> 6) << 6) | (t & 63));  // this lane's slots u4 .. u4+3
    auto lpos = [t](int p, int k) -> uint32_t { return (t >> 8) * N + (t & 255) + 256 * (p * CN + k); };
    for (uint32_t k = t; k < twoN; k += TH) lds_d[k] = tabs[k];
    const double* mono = tabs + twoN;
    for (uint32_t k = t; k < 128; k += TH) {
        const uint32_t e = k < 64 ? 64 * k : k - 64;
        const double v = __dadd_rn(mono[e], 1.0);
        mt[k] = v > 0.5 * K.Q ? __dsub_rn(v, K.Q) : v;
    }
    const double* bsk = tabs + 2 * twoN;
    const uint64_t Qhalf = P.Q >> 1;
    const int64_t Qs = (int64_t)P.Q, Bh = (int64_t)1 << (logG - 1);
    // the accumulator is held centred in doubles, c in [Qhalf - Q, Qhalf) (rgsw-acc.cpp:80-110's
    // signed representative), exact below 2^53; its digits are floors of exact power-of-two scalings
    const double Qlo = (double)(int64_t)(Qhalf - P.Q), Qhi = (double)Qhalf;
    const double Bg = (double)(1ull << logG), Bginv = 1.0 / Bg;
    uint64_t* g = acc_io + (size_t)blockIdx.x * twoN;
    const uint64_t* ap = a + (size_t)blockIdx.x * P.n;
    const size_t round_words = (size_t)4 * P.dG2 * N;
    // key words through a buffer resource: uniform round + row offset, 32-bit lane offset
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(bsk), 0, -1, 0x00020000);

    const uint64_t* gin = RESCUE ? rescue_src + (size_t)blockIdx.x * twoN : g;
    double acc[2][CN];  // centred [Qhalf - Q, Qhalf), pass A's layout
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < CN; ++k) {
            uint64_t v = gin[lpos(p, k)];
            v = v >= P.Q ? v % P.Q : v;
            acc[p][k] = (double)(v < Qhalf ? (int64_t)v : (int64_t)v - Qs);
        }
    if (WRAP && t < 2) wflag[t] = 0;
    uint32_t* ex = reinterpret_cast<uint32_t*>(mt + 128);  // rotation exponents [n]
    stage_rot_exponents<TH>(ex, ap, P.n, amod, twoN);
    __syncthreads();
    double Cn[2][4];  // N^-1 NTT(acc) at slots u4 + s, |Cn| <~ Q/2
    {
        double v[8];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int k = 0; k < CN; ++k) v[p * CN + k] = acc[p][k];
        double d[2][4];
        f64w_ntt_fwd<RED, false, PROBE < 5 && (PROBE & 2) != 0>(buf, v, d, psi, K);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int s = 0; s < 4; ++s) Cn[p][s] = fmodmul(d[p][s], K.Ninv, K);
    }
    // passes C and the units of that transform read the wave's own block of the buffer, and
    // round 0's first pass A (no barrier of its own) writes every block: without this barrier a
    // wave that gets here first overwrites blocks other waves are still reading (the wrong
    // STD128Q / STD192 ciphertexts of round 2)
    if constexpr (!(PROBE < 5 && (PROBE & 1))) __syncthreads();
    // digit l of c: low logG bits (signed) of (c + Kd_l) >> (l logG), Kd_l = sum_{z<l} Bh 2^(z logG)
    // (the closed form of the reference's carries); WRAP: residual (c + KdL) >> (L logG)
    double sl[LD + 1], kl[LD + 1];  // 2^-(l logG), Kd_l 2^-(l logG): exact
    {
        int64_t Kd = 0;
        for (uint32_t l = 0; l <= (uint32_t)LD; ++l) {
            const uint32_t shift = (l == (uint32_t)LD ? P.digits : l) * logG;
            int64_t Kx = Kd;
            if (l == (uint32_t)LD)
                for (uint32_t z = l; z < P.digits; ++z) Kx = (Kx << logG) + Bh;
            sl[l] = __builtin_ldexp(1.0, -(int)shift);
            kl[l] = __dmul_rn((double)Kx, sl[l]);
            Kd = (Kd << logG) + Bh;
        }
    }

    for (uint32_t i = 0; i < P.n; ++i) {
        // rotation exponent staged in LDS (no 64-bit remainder in the round loop)
        const uint32_t ai = ex[i];
        const uint32_t round_off = i * (uint32_t)round_words * 8;  // bytes (< 2^32: launcher)
        // products: group g = (column j, key kk, row r), rows 0 .. 2LD-1 the digits', 2LD, 2LD+1
        // the C' rows; 4 slots of key words each, the next group's loaded first
        constexpr int RW = 2 * LD + 2, NG = 4 * RW;
        auto kload = [&](int gi, double (&kv)[4]) {
            const uint32_t j = gi / (2 * RW), kk = (gi / RW) & 1, r = gi % RW;
            const uint32_t o = round_off + ((kk * P.dG2 + r) * 2 + j) * N * 8;
            const v2d lo = __builtin_bit_cast(v2d, __builtin_amdgcn_raw_buffer_load_b128(rk, (int)(u4 * 8), (int)o, 0));
            const v2d hi = __builtin_bit_cast(v2d, __builtin_amdgcn_raw_buffer_load_b128(rk, (int)(u4 * 8 + 16), (int)o, 0));
            kv[0] = lo.x, kv[1] = lo.y, kv[2] = hi.x, kv[3] = hi.y;
        };
        // F64W_KPRE = d > 0: the first d key groups requested at the top of the round (a ring of d + 1)
        constexpr int KD = F64W_KPRE > 0 ? F64W_KPRE : 1, KR = KD + 1;
        double kv[KR][4];
#pragma unroll
        for (int g = 0; g < (F64W_KPRE > 0 ? KD : 0); ++g) kload(g, kv[g]);
        double D[LD][2][4];  // digits before the last; the last digit's outputs stay in LDS
        // digit l (CORR: the WRAP correction -2^(gL) N^-1 w): extraction, forward transform
        auto digit = [&](uint32_t l, auto corr_c, double (&d)[2][4], bool sync) {
            constexpr bool CORR = decltype(corr_c)::value;
            double v[8];
            bool wv = false;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int k = 0; k < CN; ++k) {
                    const double c = acc[p][k];
                    // residual after all digits (WRAP): floor((c + KdL) 2^-(L logG))
                    const double res = WRAP ? __builtin_floor(__fma_rn(c, sl[LD], kl[LD])) : 0.0;
                    if constexpr (CORR) {
                        v[p * CN + k] = __dmul_rn(res, -K.wfac);
                    } else {
                        const double f = l == 0 ? c : __builtin_floor(__fma_rn(c, sl[l], kl[l]));
                        // signed low logG bits: f - B floor(f / B + 1/2), in [-B/2, B/2)
                        v[p * CN + k] = __fma_rn(-Bg, __builtin_floor(__fma_rn(f, Bginv, 0.5)), f);
                    }
                    if (WRAP && !CORR) wv |= res != 0.0;
                }
            if (WRAP && !CORR && l == 0) {
                // round i - 1 read wflag[(i + 1) & 1] before its inverse barrier; round i + 1
                // writes it after this round's barriers; the forward barrier publishes the vote
                if (t == 0) wflag[(i + 1) & 1] = 0;
                if (wv) wflag[i & 1] = 1;
            }
            // other waves may still read their blocks (PROBE bit 2: timing experiment without it)
            if (sync && !(PROBE < 5 && (PROBE & 4))) __syncthreads();
            if (!CORR && l + 1 == LD) f64w_ntt_fwd<RED, true>(buf, v, d, psi, K);
            else f64w_ntt_fwd<RED>(buf, v, d, psi, K);
        };
        using F_ = std::false_type;
        using T_ = std::true_type;
#pragma unroll
        for (int l = 0; l < LD; ++l) digit(l, F_{}, D[l], l > 0);
        double Cx[2][4];  // C' (+ the WRAP correction)
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int s = 0; s < 4; ++s) Cx[p][s] = Cn[p][s];
        if constexpr (WRAP) {
            if (wflag[i & 1]) {
                // the correction's transform overwrites the buffer that holds the last digit's
                // outputs: transform the last digit again afterwards (rare rounds only)
                double dc[2][4];
                digit(LD, T_{}, dc, true);
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int s = 0; s < 4; ++s) Cx[p][s] = fred(__dadd_rn(Cx[p][s], dc[p][s]), K);
                digit(LD - 1, F_{}, D[LD - 1], true);
            }
        }
        uint32_t ip[4];  // slot x evaluates at psi^(2 bitrev(x) + 1) (recomputed each round, the
        uint32_t uo = u4;  // opaque copy keeps the compiler from hoisting four live values)
        asm volatile("" : "+v"(uo));
#pragma unroll
        for (int q = 0; q < 4; ++q) ip[q] = ((2 * (__builtin_bitreverse32(uo + q) >> 21) + 1) * ai) & (twoN - 1);
        double S[2][4], A[2][4];
        double Wp[4], Wm[4];  // psi^e - 1, psi^-e - 1 at the 4 slots (built at j = 0)
        if constexpr (F64W_KPRE == 0) kload(0, kv[0]);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            if (gi + KD < NG) kload(gi + KD, kv[(gi + KD) % KR]);
            __builtin_amdgcn_sched_barrier(0);
            const int j = gi / (2 * RW), kk = (gi / RW) & 1, r = gi % RW;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double dv = r < 2 * LD - 2 ? D[r >> 1][r & 1][q]
                                  : r < 2 * LD   ? buf[(r & 1) * N + (swz(u4) ^ q)]
                                                 : Cx[r & 1][q];
                const double pr = fmodmul(dv, kv[gi % KR][q], K);
                A[kk][q] = r == 0 ? pr : __dadd_rn(A[kk][q], pr);
            }
            if (kk == 1 && r == RW - 1) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t in = (twoN - ip[q]) & (twoN - 1);
                    if (j == 0) {
                        Wp[q] = __dsub_rn(fmodmul(mt[ip[q] >> 6], mt[64 + (ip[q] & 63)], K), 1.0);
                        Wm[q] = __dsub_rn(fmodmul(mt[in >> 6], mt[64 + (in & 63)], K), 1.0);
                    }
                    const double sv = fred(__dadd_rn(fmodmul(A[0][q], Wp[q], K), fmodmul(A[1][q], Wm[q], K)), K);
                    S[j][q] = sv;
                    Cn[j][q] = fred(__dadd_rn(Cn[j][q], sv), K);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        double v[8];
        f64w_ntt_inv<RED>(buf, S, v, ipsi, K);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int k = 0; k < CN; ++k) {
                // |r| < 2^52: c + r is exact; the reduction lands within 1 of [-Q/2, Q/2], and
                // the two selects make it the centred representative exactly
                double x = fred(__dadd_rn(acc[p][k], v[p * CN + k]), K);
                x = x >= Qhi ? __dsub_rn(x, K.Q) : x;
                acc[p][k] = x < Qlo ? __dadd_rn(x, K.Q) : x;
            }
    }
    __syncthreads();  // every last inverse pass has read its entries
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < CN; ++k) {
            const int64_t c = (int64_t)acc[p][k];
            buf[lpos(p, k)] = __builtin_bit_cast(double, (uint64_t)(c < 0 ? c + Qs : c));
        }
    __syncthreads();
    for (uint32_t k = t; k < N; k += TH) {  // acc0 transposed (poly.cpp:762-770)
        const uint64_t v = __builtin_bit_cast(uint64_t, buf[k == 0 ? 0 : N - k]);
        g[k] = k == 0 ? v : (v == 0 ? 0 : P.Q - v);
        g[N + k] = __builtin_bit_cast(uint64_t, buf[N + k]);
    }
    if constexpr (PROBE == 6) {  // fault injection (test library): ciphertext 0's acc1[0] off by 2^40
        if (blockIdx.x == 0 && t == 0) g[N] ^= 1ull << 40;
    }
}

// ---- f64wduo: f64w's STD128Q round on TWO workgroups per ciphertext ------------------------------
// For batches too small to fill the chip (BASELINE C5 on an 8-GPU node: 1024 EvalSign = 128 per GPU;
// f64w runs one 512-thread workgroup per ciphertext, so 128 ciphertexts occupy half the CUs and run at
// 0.39 of the 1024 rate).  The split is by NTT half, not by polynomial: the negacyclic
// transform's first stage pairs x and x + N/2, and after it the two halves of the slots are independent
// rings until the inverse's last stage.  Member h of a pair (blocks b and b + 8, one XCD under
// round-robin dispatch, as sf2duo) holds the whole accumulator (both polynomials, f64w's pass-A layout)
// and per round:
//   * extracts the digit (and the WRAP residual vote) of every coefficient, as f64w;
//   * forward: stage 0 for its half's outputs only (one product per pair, as a full stage), stages 1-2
//     on its 4 of the thread's 8 coefficients (one barrier), then stages 3-10 wave-local -- wave w owns
//     256-block w & 3 of half h of polynomial w >> 2, 4 elements per lane, radix-4 passes (3,4) (5,6)
//     (7,8) (9,10) -- so the lane ends with 4 slots of one polynomial;
//   * products for column w >> 2 of its half's slots: the lane's own polynomial's digit and C' from
//     registers, the other polynomial's from LDS (one barrier), 2 keys x 4 rows;
//   * monomial factors, C' update, inverse stages 10-3 wave-local, stages 2-1 across waves (one barrier);
//   * hands its 4 stage-1 values per thread (16 KiB) to the partner and takes the partner's (the
//     sf2duo hand-off: sc1 stores, vmcnt(0), barrier, one flag; bounded poll; sc1 loads), and both
//     finish inverse stage 0 and the accumulator update for all coefficients (4 products per thread).
// Per lane and round: 96 FP64 modular products against f64w's 176 (forward 24 / 44, products 32 / 64,
// monomials 16 / 24, inverse 24 / 44).  The reductions sit after the same stages as f64w's (forward after
// stage 5, inverse after stages 9 (sums), 6 and 3), so every value obeys f64w's bounds
// (tools/bounds_f64.py).  A member that times out sets the pair's failed word and the rescue launch
// (k_blind_rotate_f64w<..., RESCUE>) recomputes that ciphertext from its saved input.
// Buffer index of element x of a half polynomial: dswz (device_math.hpp, shared with sfduo).

// forward: v = coefficients tau + 256k of polynomial t >> 8 (all N) -> d = the NTT values of half h at this
// lane's slots 4u .. 4u+3, u = 64 (w & 3) + l of half h, polynomial w >> 2 (also left in the buffer)
template <bool RED>
__device__ __forceinline__ void f64d_fwd(double* bf, const double (&v)[8], double (&d)[4], uint32_t h,
                                         const double* psi, const F64Const& K) {
    constexpr uint32_t H = 1024;
    const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
    {
        const uint32_t tau = f64_tau();
        double* p = bf + (t >> 8) * H + dswz(tau);
        const double w0 = psi[1];
        double o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // stage 0, this half's outputs
            const double x = fmodmul(v[k + 4], w0, K);
            o[k] = h ? __dsub_rn(v[k], x) : __dadd_rn(v[k], x);
        }
        const double w1 = psi[2 + h];
        ct_bf(o[0], o[2], w1, K), ct_bf(o[1], o[3], w1, K);
        ct_bf(o[0], o[1], psi[4 + 2 * h], K), ct_bf(o[2], o[3], psi[5 + 2 * h], K);
#pragma unroll
        for (int k = 0; k < 4; ++k) p[256 * k] = o[k];
    }
    __syncthreads();
    const uint32_t B = 4 * h + (w & 3);  // 256-block of the whole polynomial
    double* q = bf + (w >> 2) * H + 256 * (w & 3);
    double x[4];
    {  // stages 3, 4
        uint32_t y = l;
        asm volatile("" : "+v"(y));
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = q[dswz(y + 64 * k)];
        const double w3 = psi[8 + B];
        ct_bf(x[0], x[2], w3, K), ct_bf(x[1], x[3], w3, K);
        ct_bf(x[0], x[1], psi[16 + 2 * B], K), ct_bf(x[2], x[3], psi[17 + 2 * B], K);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[dswz(y + 64 * k)] = x[k];
    }
    f64w_sync();
    {  // stages 5, 6 (RED: the one reduction, after stage 5, as f64w)
        const uint32_t c = l >> 4, y = 64 * c + (l & 15);
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = q[dswz(y + 16 * k)];
        const double w5 = psi[32 + 4 * B + c];
        ct_bf(x[0], x[2], w5, K), ct_bf(x[1], x[3], w5, K);
        if constexpr (RED) {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = fred(x[k], K);
        }
        ct_bf(x[0], x[1], psi[64 + 8 * B + 2 * c], K), ct_bf(x[2], x[3], psi[65 + 8 * B + 2 * c], K);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[dswz(y + 16 * k)] = x[k];
    }
    f64w_sync();
    {  // stages 7, 8
        const uint32_t c = l >> 2, y = 16 * c + (l & 3);
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = q[dswz(y + 4 * k)];
        const double w7 = psi[128 + 16 * B + c];
        ct_bf(x[0], x[2], w7, K), ct_bf(x[1], x[3], w7, K);
        ct_bf(x[0], x[1], psi[256 + 32 * B + 2 * c], K), ct_bf(x[2], x[3], psi[257 + 32 * B + 2 * c], K);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[dswz(y + 4 * k)] = x[k];
    }
    f64w_sync();
    {  // stages 9, 10: slots 4u .. 4u+3 (f64w's units with u = 64 B + l)
        const uint32_t y = 4 * l;
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = q[dswz(y + k)];
        const double w9 = psi[512 + 64 * B + l];
        ct_bf(x[0], x[2], w9, K), ct_bf(x[1], x[3], w9, K);
        const double2 w10 = *(const double2*)(psi + 1024 + 128 * B + 2 * l);
        ct_bf(x[0], x[1], w10.x, K), ct_bf(x[2], x[3], w10.y, K);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = x[k];
    }
}

// inverse: s = column w >> 2's NTT-domain increment at the lane's slots -> after stages 10..1 (wave-local,
// then one barrier and stages 2-1 across waves) o = elements tau + 256k' (k' < 4) of half h of column t >> 8
template <bool RED>
__device__ __forceinline__ void f64d_inv(double* bi, const double (&s)[4], double (&o)[4], uint32_t h,
                                         const double* ipsi, const F64Const& K) {
    constexpr uint32_t H = 1024;
    const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
    const uint32_t B = 4 * h + (w & 3);
    double* q = bi + (w >> 2) * H + 256 * (w & 3);
    double x[4] = {s[0], s[1], s[2], s[3]};
    {  // stages 10, 9 (RED: the sums, as f64w's units)
        const uint32_t y = 4 * l;
        const double2 w10 = *(const double2*)(ipsi + 1024 + 128 * B + 2 * l);
        gs_bf(x[0], x[1], w10.x, K), gs_bf(x[2], x[3], w10.y, K);
        const double w9 = ipsi[512 + 64 * B + l];
        gs_bf(x[0], x[2], w9, K), gs_bf(x[1], x[3], w9, K);
        if constexpr (RED) x[0] = fred(x[0], K), x[1] = fred(x[1], K);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[dswz(y + k)] = x[k];
    }
    f64w_sync();
    {  // stages 8, 7
        const uint32_t c = l >> 2, y = 16 * c + (l & 3);
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = q[dswz(y + 4 * k)];
        gs_bf(x[0], x[1], ipsi[256 + 32 * B + 2 * c], K), gs_bf(x[2], x[3], ipsi[257 + 32 * B + 2 * c], K);
        const double w7 = ipsi[128 + 16 * B + c];
        gs_bf(x[0], x[2], w7, K), gs_bf(x[1], x[3], w7, K);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[dswz(y + 4 * k)] = x[k];
    }
    f64w_sync();
    {  // stages 6, 5 (RED: every output of stage 6, as the end of f64w's pass C)
        const uint32_t c = l >> 4, y = 64 * c + (l & 15);
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = q[dswz(y + 16 * k)];
        gs_bf(x[0], x[1], ipsi[64 + 8 * B + 2 * c], K), gs_bf(x[2], x[3], ipsi[65 + 8 * B + 2 * c], K);
        if constexpr (RED) {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = fred(x[k], K);
        }
        const double w5 = ipsi[32 + 4 * B + c];
        gs_bf(x[0], x[2], w5, K), gs_bf(x[1], x[3], w5, K);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[dswz(y + 16 * k)] = x[k];
    }
    f64w_sync();
    {  // stages 4, 3 (RED: every output, as the end of f64w's pass B)
        uint32_t y = l;
        asm volatile("" : "+v"(y));
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = q[dswz(y + 64 * k)];
        gs_bf(x[0], x[1], ipsi[16 + 2 * B], K), gs_bf(x[2], x[3], ipsi[17 + 2 * B], K);
        const double w3 = ipsi[8 + B];
        gs_bf(x[0], x[2], w3, K), gs_bf(x[1], x[3], w3, K);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[dswz(y + 64 * k)] = RED ? fred(x[k], K) : x[k];
    }
    __syncthreads();
    {  // stages 2, 1 of half h (no reduction, as f64w's pass A)
        const uint32_t tau = f64_tau();
        const double* p = bi + (t >> 8) * H + dswz(tau);
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = p[256 * k];
        gs_bf(o[0], o[1], ipsi[4 + 2 * h], K), gs_bf(o[2], o[3], ipsi[5 + 2 * h], K);
        const double w1 = ipsi[2 + h];
        gs_bf(o[0], o[2], w1, K), gs_bf(o[1], o[3], w1, K);
    }
}

__device__ __forceinline__ void duo_store_d(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double duo_load_d(const double* p) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<uint64_t*>(const_cast<double*>(p)),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
#ifndef F64D_MFULL
#define F64D_MFULL 1
#endif
#ifndef F64D_FSW
#define F64D_FSW 1
#endif
// row e of the whole factor table lives at e ^ (bits 5-9 of e): a wave's exponents (2 bitrev(slot) + 1) a'
// share their low five bits, so unswizzled every lane of a 32-lane group hit one bank pair (a 32-way
// conflict on each of the 8 lookups per lane-round; mean 29.4 distinct addresses per bank over random a');
// with the fold the mean is 2.0 (bit 5 up varies as m a' for the group's 32 values of m)
__device__ __forceinline__ uint32_t fsw(uint32_t e) { return F64D_FSW ? e ^ ((e >> 5) & 31) : e; }
#ifndef F64D_KPRE
#define F64D_KPRE 4
#endif

// STD128Q class only (RED, WRAP, one transformed digit: f64w<true, true, 1>).  Two waves per SIMD
// (116 KiB of LDS with the whole factor table: one workgroup per CU), so the round's state fits registers
// without spills (182 VGPRs with four key groups in flight).
// PROBE 1 (test library only, TFHE_TEST_PROBES): member 1 of pair 0 stops publishing at round 2, as a
// partner that never arrives would, and the wait is a 64th of the 10 ms bound.  PROBE 2 (timing only, results
// invalid): no hand-off at all -- each member takes its own stage-1 values for its partner's -- the
// bound on what the exchange costs per round
// Hardware assumptions of the hand-off (verdict r5 item 7):
//  * ordering: the data stores and the flag are RELAXED agent-scope atomics (write-through past the CU, `sc1`);
//    the data is ordered before the flag by every wave's `s_waitcnt vmcnt(0)` (each store acknowledged) and the
//    workgroup barrier, and on the reader by the poll's load returning before the barrier and the loads behind
//    it.  That is gfx9 ISA behaviour (the MI355X_MICROARCH.md hand-off table's sc1 row), not a HIP-memory-model
//    release / acquire pair -- one of those costs about 1.7 us per round, more than the hand-off itself;
//  * pairing: members b and b + 8 share an XCD only through round-robin workgroup dispatch; correctness never
//    depends on it (agent scope), the latency does (same-XCD hand-offs measured 1.1-1.3 us, cross-XCD 1.9-2.0);
//  * liveness: both members must be resident at once.  The launcher runs the duo form only for batches up to the
//    device's co-resident pairs (one 116-KiB workgroup per CU: half the CU count) and fences duo launches of one
//    device's buffer across streams; a partner still missing after 10 ms of wall clock (s_memrealtime, e.g.
//    behind another context's kernel) fails the pair, and the rescue launch recomputes it exactly.
// The hand-off is one flag per member per round (workgroup barrier, t == 0 stores / polls, barrier).  Forms
// measured against it and removed (tools/duo_probe.py, us per round at 128 ciphertexts): data-tagged granules
// (value + round tag in one 8-byte word, no flag or barriers) polling the four words one after another 8.03
// against 7.71, the same with all four loads in flight per poll 7.56-7.71 against 7.51-7.66 (a tie), one flag
// per wavefront with no workgroup barrier 8.8-9.2 against 7.5-7.6 (profiles/r05g, r05h, r05i).
// Round 6: templated on f64w's shape as well -- <RED, WRAP, LD> = <true, true, 1> for the STD128Q class (above)
// and <false, false, 2> for the STD192 class (Q < 2^40, no reductions, two transformed digits whose outputs and
// C' are exchanged between the column's waves through three LDS buffers; 132 KiB of LDS), as f64w's two instances.
template <int PROBE = 0, bool RED = true, bool WRAP = true, int LD = 1>
__global__ void __launch_bounds__(512, 2)
k_blind_rotate_f64wduo(BRParams P, F64Const K, const double* __restrict__ tabs, const uint64_t* __restrict__ a,
                       uint64_t amod, uint64_t* __restrict__ acc_io, DuoBuf X, uint32_t pairs) {
    extern __shared__ __align__(16) double lds_d[];
    constexpr uint32_t N = 2048, H = 1024, TH = 512;
    const uint32_t b = blockIdx.x, pair = (b >> 4) * 8 + (b & 7), h = (b >> 3) & 1;
    if (pair >= pairs) return;  // both members of a pair take this branch together
    double* psi = lds_d;
    double* ipsi = lds_d + N;
    double* bf = lds_d + 2 * N;  // forward buffer [2][H]
    double* bi = bf + 2 * H;     // inverse buffer [2][H]
    double* cx = bi + 2 * H;     // this round's C' (+ the WRAP correction) [2][H], slot positions
    double* dx = cx + 2 * H;     // LD = 2: digit 0's values for the other column's waves [2][H] (digit 1: bf)
    // F64D_MFULL: the whole 2N-entry factor table psi^e - 1 (32 KiB; one workgroup per CU leaves the LDS for
    // it), one lookup per factor; otherwise the two 64-entry tables, two lookups and a product per factor
    double* mt = dx + (LD > 1 ? 2 * H : 0);  // monomial tables
    uint32_t* ex = reinterpret_cast<uint32_t*>(mt + (F64D_MFULL ? 2 * N : 128));  // rotation exponents [n]
    __shared__ int wflag[2];
    __shared__ uint32_t duo_ok;
    const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6, twoN = 2 * N, logG = P.logG;
    // this wave's polynomial / column, wave-uniform: through readfirstlane the key loads' row offset is an
    // SGPR (as w >> 2 the compiler wrapped each of the 16 key loads per round in a waterfall loop)
    const uint32_t j = __builtin_amdgcn_readfirstlane(w >> 2);
    const uint32_t u4 = 4 * (256 * h + 64 * (w & 3) + l);     // this lane's slots u4 .. u4+3 (whole ring)
    const uint32_t sp = j * H + 256 * (w & 3);                // their buffer block
    for (uint32_t k = t; k < twoN; k += TH) lds_d[k] = tabs[k];
    const double* mono = tabs + twoN;
    if constexpr (F64D_MFULL) {
        for (uint32_t k = t; k < twoN; k += TH) mt[fsw(k)] = mono[k];  // centred psi^k - 1 (k_pack_f64)
    } else {
        for (uint32_t k = t; k < 128; k += TH) {
            const uint32_t e = k < 64 ? 64 * k : k - 64;
            const double v = __dadd_rn(mono[e], 1.0);
            mt[k] = v > 0.5 * K.Q ? __dsub_rn(v, K.Q) : v;
        }
    }
    const double* bsk = tabs + 2 * twoN;
    const uint64_t Qhalf = P.Q >> 1;
    const int64_t Qs = (int64_t)P.Q, Bh = (int64_t)1 << (logG - 1);
    const double Qlo = (double)(int64_t)(Qhalf - P.Q), Qhi = (double)Qhalf;
    const double Bg = (double)(1ull << logG), Bginv = 1.0 / Bg;
    uint64_t* g = acc_io + (size_t)pair * twoN;
    const uint64_t* ap = a + (size_t)pair * P.n;
    const size_t round_words = (size_t)4 * P.dG2 * N;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(bsk), 0, -1, 0x00020000);
    const uint32_t tau = t & 255, pp = t >> 8;  // pass-A role: coefficients tau + 256k of polynomial pp

    double acc[8];  // centred, all N coefficients: tau + 256k of polynomial pp (both members)
    uint64_t* sv = X.save + (size_t)pair * twoN;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint64_t v = g[pp * N + tau + 256 * k];
        if (pp == h) sv[pp * N + tau + 256 * k] = v;  // the rescue's input if the pair times out
        v = v >= P.Q ? v % P.Q : v;
        acc[k] = (double)(v < Qhalf ? (int64_t)v : (int64_t)v - Qs);
    }
    if (t < 2) wflag[t] = 0;
    stage_rot_exponents<TH>(ex, ap, P.n, amod, twoN);
    __syncthreads();
    double Cn[4];  // N^-1 NTT(acc_j) at the lane's slots
    {
        double d[4];
        f64d_fwd<RED>(bf, acc, d, h, psi, K);
#pragma unroll
        for (int s = 0; s < 4; ++s) Cn[s] = fmodmul(d[s], K.Ninv, K);
    }
    __syncthreads();  // the prologue's wave-local passes vs round 0's pass A (f64w's round-2 race)
    // digit l of c: low logG bits (signed) of (c + Kd_l) >> (l logG); WRAP: residual (c + KdL) >> (L logG) (f64w's)
    double sl[LD + 1], kl[LD + 1];
    {
        int64_t Kd = 0;
        for (uint32_t l = 0; l <= (uint32_t)LD; ++l) {
            const uint32_t shift = (l == (uint32_t)LD ? P.digits : l) * logG;
            int64_t Kx = Kd;
            if (l == (uint32_t)LD)
                for (uint32_t z = l; z < P.digits; ++z) Kx = (Kx << logG) + Bh;
            sl[l] = __builtin_ldexp(1.0, -(int)shift);
            kl[l] = __dmul_rn((double)Kx, sl[l]);
            Kd = (Kd << logG) + Bh;
        }
    }
    uint32_t* myflag = X.flags + (pair * 2 + h) * 32;
    const uint32_t* peerflag = X.flags + (pair * 2 + (1 - h)) * 32;
    for (uint32_t i = 0; i < P.n; ++i) {
        const uint32_t ai = ex[i];
        const uint32_t round_off = i * (uint32_t)round_words * 8;  // bytes (< 2^32: launcher)
        double D[LD][4], dum[4];
        // products of column j: group gi = (key kk, row rr): rr = 2l (own digit l), 2l + 1 (the other column's
        // digit l), 2LD (own C'), 2LD + 1 (the other's); key row 2l + polynomial, 2LD + polynomial
        constexpr int RW = 2 * LD + 2, NG = 2 * RW;
        auto krow = [j](uint32_t rr) -> uint32_t { return (rr & ~1u) + ((rr & 1) ? 1 - j : j); };
        auto kload = [&](int gi, double (&kv)[4]) {
            const uint32_t kk = gi / RW, r = krow(gi % RW);
            const uint32_t o = round_off + ((kk * P.dG2 + r) * 2 + j) * N * 8;
            const v2d lo = __builtin_bit_cast(v2d, __builtin_amdgcn_raw_buffer_load_b128(rk, (int)(u4 * 8), (int)o, 0));
            const v2d hi = __builtin_bit_cast(v2d, __builtin_amdgcn_raw_buffer_load_b128(rk, (int)(u4 * 8 + 16), (int)o, 0));
            kv[0] = lo.x, kv[1] = lo.y, kv[2] = hi.x, kv[3] = hi.y;
        };
        // F64D_KPRE: the round's first key group is requested before the forward transform, so its L2
        // latency overlaps the transform instead of opening the products (two waves per SIMD hide little)
        // (F64D_KPRE = d groups in flight: the first d requested here, group g + d at product group g, a ring
        // of d + 1; 0: the round-4 form, group 0 requested at the products)
        constexpr int KD = F64D_KPRE > 0 ? F64D_KPRE : 1, KR = KD + 1 < NG ? KD + 1 : NG;
        double kv[KR][4];
#pragma unroll
        for (int g = 0; g < (F64D_KPRE > 0 ? KD : 0); ++g) kload(g, kv[g]);
        auto digit = [&](uint32_t l, bool corr, double (&d)[4]) {
            double v[8];
            bool wv = false;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double c = acc[k];
                const double res = WRAP ? __builtin_floor(__fma_rn(c, sl[LD], kl[LD])) : 0.0;
                if (WRAP && corr) {
                    v[k] = __dmul_rn(res, -K.wfac);
                } else {
                    const double f = l == 0 ? c : __builtin_floor(__fma_rn(c, sl[l], kl[l]));
                    v[k] = __fma_rn(-Bg, __builtin_floor(__fma_rn(f, Bginv, 0.5)), f);
                    if (WRAP) wv |= res != 0.0;
                }
            }
            if (WRAP && !corr && l == 0) {
                if (t == 0) wflag[(i + 1) & 1] = 0;
                if (wv) wflag[i & 1] = 1;
            }
            if (l > 0 && !corr) __syncthreads();  // other waves may still read their blocks of digit l - 1
            f64d_fwd<RED>(bf, v, d, h, psi, K);
        };
#pragma unroll
        for (int l = 0; l < LD; ++l) digit(l, false, D[l]);
        double Cx[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) Cx[s] = Cn[s];
        if (WRAP && wflag[i & 1]) {  // (uniform: published by the forward's barrier; about 2^-14 of rounds)
            __syncthreads();  // other waves may still read their blocks
            digit(LD, true, dum);
#pragma unroll
            for (int s = 0; s < 4; ++s) Cx[s] = fred(__dadd_rn(Cx[s], dum[s]), K);
        }
        // this lane's digit and C' values for the other column's waves (each wave writes only its own block of
        // every buffer; bf: the last digit, dx: digit 0 when LD = 2)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            bf[sp + dswz(4 * l + s)] = D[LD - 1][s];
            if constexpr (LD > 1) dx[sp + dswz(4 * l + s)] = D[0][s];
            cx[sp + dswz(4 * l + s)] = Cx[s];
        }
        if constexpr (PROBE != 4) __syncthreads();  // (PROBE 4, timing only: no exchange barrier, results invalid)
        double Do[LD][4], Co[4];  // the other polynomial's at the same slots
        const uint32_t so = (1 - j) * H + 256 * (w & 3);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            Do[LD - 1][s] = bf[so + dswz(4 * l + s)], Co[s] = cx[so + dswz(4 * l + s)];
            if constexpr (LD > 1) Do[0][s] = dx[so + dswz(4 * l + s)];
        }
        double A[2][4];
        if constexpr (F64D_KPRE == 0) kload(0, kv[0]);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
            if (gi + KD < NG) kload(gi + KD, kv[(gi + KD) % KR]);
            __builtin_amdgcn_sched_barrier(0);
            const int kk = gi / RW, rr = gi % RW;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const double dv = rr < 2 * LD ? ((rr & 1) ? Do[rr >> 1][s] : D[rr >> 1][s]) : (rr & 1) ? Co[s] : Cx[s];
                const double pr = fmodmul(dv, kv[gi % KR][s], K);
                A[kk][s] = rr == 0 ? pr : __dadd_rn(A[kk][s], pr);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t uo = u4;
        asm volatile("" : "+v"(uo));
        double S[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            uint32_t ip = ((2 * (__builtin_bitreverse32(uo + s) >> 21) + 1) * ai) & (twoN - 1);
            if constexpr (PROBE == 3) ip = ai & (twoN - 1);  // timing only: wave-uniform table rows
            const uint32_t in = (twoN - ip) & (twoN - 1);
            const double Wp = F64D_MFULL ? mt[fsw(ip)] : __dsub_rn(fmodmul(mt[ip >> 6], mt[64 + (ip & 63)], K), 1.0);
            const double Wm = F64D_MFULL ? mt[fsw(in)] : __dsub_rn(fmodmul(mt[in >> 6], mt[64 + (in & 63)], K), 1.0);
            S[s] = fred(__dadd_rn(fmodmul(A[0][s], Wp, K), fmodmul(A[1][s], Wm, K)), K);
            Cn[s] = fred(__dadd_rn(Cn[s], S[s]), K);
        }
        double o[4];
        f64d_inv<RED>(bi, S, o, h, ipsi, K);
        // hand-off: this half's stage-1 values of both columns to the partner (thread t's 4 at k' 512 + t)
        double* mine = reinterpret_cast<double*>(X.xbuf + (((size_t)pair * 2 + h) * 2 + (i & 1)) * N);
        const double* theirs = reinterpret_cast<const double*>(X.xbuf + (((size_t)pair * 2 + (1 - h)) * 2 + (i & 1)) * N);
        double lo[4], hi[4];
        if constexpr (PROBE != 2) {
#pragma unroll
            for (int k = 0; k < 4; ++k) duo_store_d(mine + 512 * k + t, o[k]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // every wave's stores drained; every read of the inverse buffer done
        if (PROBE != 2 && t == 0) {
            // the wait is bounded by time (wall clock, s_memrealtime): kDuoWaitMs, PROBE 1 a 64th of it
            const bool gone = PROBE == 1 && pair == 0 && h == 1 && i >= 2;
            if (!gone) __hip_atomic_store(myflag, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // (the clock is read every 8th poll, the deadline set at the first read: a partner within 8 polls
            // costs no clock read)
            bool ok = !gone;
            uint64_t t_end = 0;
            uint32_t k = 0;
            while (ok && __hip_atomic_load(const_cast<uint32_t*>(peerflag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < i + 1) {
                if ((++k & 7) == 0) {
                    const uint64_t now = wall_clock64();
                    if (t_end == 0) t_end = now + (PROBE ? X.wait_ticks >> 6 : X.wait_ticks);
                    else if (now > t_end) ok = false;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            duo_ok = ok;
            if (!ok) {
                __hip_atomic_store(X.flags + pair * 2 * 32 + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(X.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if constexpr (PROBE != 2) {
            __syncthreads();
            if (!duo_ok) break;  // uniform: the partner never arrived (the rescue launch recomputes the pair)
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double pv = PROBE == 2 ? o[k] : duo_load_d(theirs + 512 * k + t);
            lo[k] = h ? pv : o[k];
            hi[k] = h ? o[k] : pv;
        }
        const double w0 = ipsi[1];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // stage 0 for all coefficients, then f64w's accumulator update
            const double r[2] = {__dadd_rn(lo[k], hi[k]), fmodmul(__dsub_rn(lo[k], hi[k]), w0, K)};
#pragma unroll
            for (int z = 0; z < 2; ++z) {
                double x = fred(__dadd_rn(acc[k + 4 * z], r[z]), K);
                x = x >= Qhi ? __dsub_rn(x, K.Q) : x;
                acc[k + 4 * z] = x < Qlo ? __dadd_rn(x, K.Q) : x;
            }
        }
    }
    __syncthreads();
    // member h writes polynomial h (acc0 transposed, poly.cpp:762-770) through the two buffers (N doubles)
    double* st = bf;
    if (pp == h) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t c = (int64_t)acc[k];
            st[tau + 256 * k] = __builtin_bit_cast(double, (uint64_t)(c < 0 ? c + Qs : c));
        }
    }
    __syncthreads();
    for (uint32_t k = t; k < N; k += TH) {
        if (h == 0) {
            const uint64_t v = __builtin_bit_cast(uint64_t, st[k == 0 ? 0 : N - k]);
            g[k] = k == 0 ? v : (v == 0 ? 0 : P.Q - v);
        } else {
            g[N + k] = __builtin_bit_cast(uint64_t, st[k]);
        }
    }
}

// canonical u64 tables / BSK (generic arena) -> centred doubles
// a * b mod Q for Q < 2^50 in 12-bit steps (one-time packing only)
__device__ uint64_t mulmod_slow(uint64_t a, uint64_t b, uint64_t Q) {
    uint64_t r = 0;
    for (int s = 48; s >= 0; s -= 12) r = ((r << 12) % Q + a * ((b >> s) & 0xfff)) % Q;
    return r;
}

// canonical u64 tables / BSK (generic arena) -> centred doubles; F.on: fold the top digit's
// rows into the others (row = 2l + p of [n][2][dG2][2][N])
__global__ void k_pack_f64(uint64_t Q, uint32_t N, uint32_t dG2, F64Fold F, const uint64_t* __restrict__ psi,
                           const uint64_t* __restrict__ ipsi, const uint64_t* __restrict__ mono,
                           const uint64_t* __restrict__ bsk, size_t words, double* __restrict__ out) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto cen = [Q](uint64_t v) { return v > Q / 2 ? (double)(int64_t)(v - Q) : (double)v; };
    if (idx < N) out[idx] = cen(psi[idx]), out[N + idx] = cen(ipsi[idx]);
    if (idx < 2 * (size_t)N) out[2 * N + idx] = cen(mono[idx]);
    if (idx < words) {
        uint64_t v = bsk[idx] % Q;
        if (F.on) {
            const uint32_t row = (uint32_t)((idx / (2 * (size_t)N)) % dG2), l = row >> 1, p = row & 1;
            const uint32_t top = 2 * (F.L - 1) + p;
            const uint64_t wt = bsk[idx + ((size_t)top - row) * 2 * N] % Q;
            v = l + 1 < F.L ? (v + Q - mulmod_slow(wt, F.hc[l], Q)) % Q : mulmod_slow(v, F.hc[l], Q);
        }
        out[4 * (size_t)N + idx] = cen(v);
    }
}

uint64_t pow_mod(uint64_t b, uint64_t e, uint64_t Q) {
    unsigned __int128 r = 1, x = b % Q;
    for (; e; e >>= 1, x = x * x % Q)
        if (e & 1) r = r * x % Q;
    return (uint64_t)r;
}

// The top digit is the exact remainder (c = sum_l 2^(gl) d_l) for every centred c: the digit
// recursion d -> (d + 2^(g-1)) >> g is monotone, so checking both extremes suffices.
bool fold_possible(const BRParams& P) { return P.thr == 0 && P.digits >= 2 && P.digits <= 8; }

bool fold_exact(const BRParams& P) {
    if (!fold_possible(P)) return false;
    const int64_t Qs = (int64_t)P.Q, half = (int64_t)(P.Q >> 1);
    const uint32_t sh = 64 - P.logG;
    for (int64_t c : {half - 1, half - Qs}) {
        int64_t d = c;
        for (uint32_t l = 0; l < P.digits; ++l) {
            const int64_t r = (int64_t)((uint64_t)d << sh) >> sh;
            d = (d - r) >> P.logG;
        }
        if (d != 0) return false;
    }
    return true;
}

F64Fold make_fold(const BRParams& P, bool on) {
    F64Fold F{};
    F.on = on;
    F.L = P.digits;
    if (!F.on) return F;
    const uint64_t inv2 = (P.Q + 1) / 2, L = P.digits;
    for (uint32_t l = 0; l + 1 < L; ++l) F.hc[l] = pow_mod(inv2, (uint64_t)P.logG * (L - 1 - l), P.Q);
    F.hc[L - 1] = (uint64_t)((unsigned __int128)P.N * pow_mod(inv2, (uint64_t)P.logG * (L - 1), P.Q) % P.Q);
    return F;
}

}  // namespace

bool f64_path_supported(const BRParams& P, int word_bits) {
    // every parameter set with 2^32 <= Q < 2^50 has N = 2048 (STD192*, STD192Q*, STD128Q*): the N = 1024
    // instances were never reachable and were removed in round 4
    return word_bits == 64 && P.Q >= (1ull << 32) && P.Q < (1ull << 50) && P.N == 2048 && P.logG <= 32 && P.n > 0;
}

size_t bsk_f64_bytes(const BRParams& P) { return ((size_t)4 * P.N + (size_t)P.n * 4 * P.dG2 * P.N) * 8; }

// TFHE_F64_FOLD (read at setup): unset/2 = fold whenever thr = 0, with the WRAP correction where the top
// digit is not always exact (STD128Q: 16.2K vs 15.2K bootstraps/s unfolded on C5a); 1 = only where it is
// always exact (STD192 classes); 0 = never
bool f64_fold_enabled(const BRParams& P) {
    const char* e = std::getenv("TFHE_F64_FOLD");
    const int mode = e && e[0] ? e[0] - '0' : 2;
    return mode == 2 ? fold_possible(P) : mode == 1 ? fold_exact(P) : false;
}

namespace {
// The instances shipped (only combinations some parameter set reaches, each in a parity test):
//   f64w  <RED, WRAP, LD>: STD128Q(_OPT) <1, 1, 1> (+ f64wduo and the rescue form); STD192(_OPT), STD192Q(_OPT)
//   <0, 0, 2>.  Round 5 retired the slot-layout kernel (k_blind_rotate_f64, the cross-check for TFHE_F64W=0
//   and the unfolded forms): an unfolded context (TFHE_F64_FOLD=0 / 1) now runs the generic u64 kernel.
bool f64w_instance(bool red, bool wrap, int ld) { return (red && wrap && ld == 1) || (!red && !wrap && ld == 2); }
}  // namespace

bool f64_test_probes_compiled() {
#ifdef TFHE_TEST_PROBES
    return true;
#else
    return false;
#endif
}

bool f64_instance_available(const BRParams& P, bool fold) {
    if (!fold || !fold_possible(P)) return false;
    const bool red = P.Q >= (1ull << 40), wrap = !fold_exact(P);
    // f64w addresses the keys with 32-bit byte offsets (buffer resource)
    const bool fits32 = (uint64_t)P.n * 4 * P.dG2 * P.N * 8 < (1ull << 32);
    return fits32 && f64w_instance(red, wrap, (int)P.digits - 1);
}

hipError_t launch_pack_bsk_f64(const BRParams& P, const DevTables& T, const void* bsk, bool fold, void* out,
                               hipStream_t s) {
    if (fold && !fold_possible(P)) return hipErrorInvalidValue;
    const size_t words = (size_t)P.n * 4 * P.dG2 * P.N;
    hipLaunchKernelGGL(k_pack_f64, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, (uint64_t)P.Q, P.N, P.dG2,
                       make_fold(P, fold), (const uint64_t*)T.psi, (const uint64_t*)T.ipsi, (const uint64_t*)T.mono, (const uint64_t*)bsk,
                       words, (double*)out);
    return hipGetLastError();
}

bool f64_duo_form(const BRParams& P, bool fold) {
    if (!f64_path_supported(P, 64) || !fold) return false;
    return (P.Q >= (1ull << 40) && !fold_exact(P) && P.digits == 2) ||  // STD128Q class: <RED, WRAP, 1>
           (P.Q < (1ull << 40) && fold_exact(P) && P.digits == 3);      // STD192 class (round 6): <-, -, 2>
}

hipError_t launch_blind_rotate_f64(const BRParams& P, const DevTables& T, const void* keys, bool fold,
                                   const uint64_t* a, uint64_t amod, uint64_t* acc, size_t B, hipStream_t s,
                                   const Knobs& kn, DuoDev* duo) {
    if (B == 0) return hipSuccess;
    if (P.N != 2048 || !f64_instance_available(P, fold)) return hipErrorInvalidValue;
    F64Const K;
    K.Q = (double)P.Q;
    K.Qinv = 1.0 / K.Q;
    K.Qi = (int64_t)P.Q;
    const uint64_t ninv = P.Q - (P.Q - 1) / P.N;  // N (Q-1)/N = -1 mod Q
    K.Ninv = -(double)((P.Q - 1) / P.N);
    const uint64_t wf = (uint64_t)((unsigned __int128)pow_mod(2, (uint64_t)P.logG * P.digits, P.Q) * ninv % P.Q);
    K.wfac = wf > P.Q / 2 ? -(double)(P.Q - wf) : (double)wf;
    const bool wrap = fold && !fold_exact(P);
    // psi, ipsi, two polynomials, monomial tables, rotation exponents
    const size_t lds = ((size_t)4 * P.N + 128) * sizeof(double) + rot_exponent_bytes(P.n);
    auto gow = [&](auto kern) {  // f64w (the last two arguments: the rescue form's)
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(P.N / 4), lds, s, P, K, (const double*)keys, T.eidx, a,
                           amod, acc, (const uint32_t*)nullptr, (const uint64_t*)nullptr);
    };
    const bool red = P.Q >= (1ull << 40);
    const int ld = (int)P.digits - 1;
    {
#ifdef TFHE_TEST_PROBES
        // test library only (lib/libtfhe_hip_test.so): the fault probe of tests/test_gpu_f64w_race.py
        // (2: waves 1.. delayed in the prologue, barrier kept; 3: the same without the barrier -- the
        // round-2 race, wrong results) and a timing-only build (4: STD192 without the barrier before
        // digit 1's pass A, results invalid; tools/f64w_barrier_probe.sh)
        if (kn.probe != 0 && (kn.probe < 5 || kn.probe == 6)) {  // (5, 7, 9: the duo probes, below)
            if (kn.probe == 4 && !red && !wrap && ld == 2) gow(k_blind_rotate_f64w<false, false, 2, 4>);
            else if (kn.probe == 2 && red && wrap && ld == 1) gow(k_blind_rotate_f64w<true, true, 1, 2>);
            else if (kn.probe == 3 && red && wrap && ld == 1) gow(k_blind_rotate_f64w<true, true, 1, 3>);
            else if (kn.probe == 6 && red && wrap && ld == 1) gow(k_blind_rotate_f64w<true, true, 1, 6>);
            else return hipErrorInvalidValue;
            return hipGetLastError();
        }
#endif
        const bool duo_shape = (red && wrap && ld == 1) || (!red && !wrap && ld == 2);
        if (duo_shape && duo && B <= (size_t)kn.duo && B <= duo->resident_pairs && B <= kDuoMaxPairs) {
            // two workgroups per ciphertext (f64wduo), then the rescue of timed-out pairs
            const DuoBuf X = duo_layout(*duo);
            const size_t ldsd = ((size_t)2 * P.N + 3 * P.N + (ld > 1 ? P.N : 0) + (F64D_MFULL ? 2 * P.N : 128)) *
                                    sizeof(double) + rot_exponent_bytes(P.n);
            auto dk = red ? k_blind_rotate_f64wduo<0, true, true, 1> : k_blind_rotate_f64wduo<0, false, false, 2>;
            auto rk = red ? k_blind_rotate_f64w<true, true, 1, 0, true> : k_blind_rotate_f64w<false, false, 2, 0, true>;
#ifdef TFHE_TEST_PROBES
            if (red) {  // (the STD128Q instance's probes)
                if (kn.probe == 5) dk = k_blind_rotate_f64wduo<1>;  // test library only: a partner that never arrives
                if (kn.probe == 7) dk = k_blind_rotate_f64wduo<2>;  // timing only: no hand-off (results invalid)
                if (kn.probe == 9) dk = k_blind_rotate_f64wduo<3>;  // timing only: broadcast factor-table reads
                if (kn.probe == 11) dk = k_blind_rotate_f64wduo<4>;  // timing only: no D / C' exchange barrier
            } else if (kn.probe == 5) {
                dk = k_blind_rotate_f64wduo<1, false, false, 2>;  // test library only: a partner that never arrives
            }
#endif
            (void)hipFuncSetAttribute((const void*)dk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsd);
            (void)hipFuncSetAttribute((const void*)rk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            return duo_serialised(*duo, s, [&]() -> hipError_t {
                if (hipError_t e = hipMemsetAsync(X.flags, 0, (size_t)B * 2 * 128, s); e != hipSuccess) return e;
                hipLaunchKernelGGL(dk, dim3((unsigned)(16 * ((B + 7) / 8))), dim3(512), ldsd, s, P, K, (const double*)keys,
                                   a, amod, acc, X, (uint32_t)B);
                if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
                hipLaunchKernelGGL(rk, dim3((unsigned)B), dim3(512), lds, s, P, K, (const double*)keys, T.eidx, a, amod,
                                   acc, (const uint32_t*)X.flags, (const uint64_t*)X.save);
                return hipGetLastError();
            });
        }
        if (red) gow(k_blind_rotate_f64w<true, true, 1>);
        else gow(k_blind_rotate_f64w<false, false, 2>);
        return hipGetLastError();
    }
}

}  // namespace tfhe
