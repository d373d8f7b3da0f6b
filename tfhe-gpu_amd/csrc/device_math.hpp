// device_math.hpp -- exact modular arithmetic for gfx950 VALU.
//
// Every modular product on the hot path has one operand that is a key or a table
// constant (BSK coefficient, twiddle, psi^k - 1), so all of them use Shoup's
// method with a precomputed companion w' = floor(w * 2^b / Q):
//     r = a*w - mulhi(a, w')*Q  in [0, 2Q)   (wrapping b-bit arithmetic)
// On gfx950 v_mul_lo_u32 / v_mul_hi_u32 / v_mad_u64_u32 issue at the same rate
// as v_add_u32 (profiles/r01_valu_rates.txt), so a u32 Shoup product is
// 3 multiplies + 1 subtract.  W = uint32_t when Q < 2^31 (STD128: Q < 2^27),
// W = uint64_t otherwise (__umul64hi lowers to v_mad_u64_u32 chains).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace tfhe {

template <typename W>
struct WordOps;

template <>
struct WordOps<uint32_t> {
    static __device__ __forceinline__ uint32_t mulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }
};
template <>
struct WordOps<uint64_t> {
    static __device__ __forceinline__ uint64_t mulhi(uint64_t a, uint64_t b) { return __umul64hi(a, b); }
};

// a*w mod Q in [0, 2Q); requires w < Q, any a < 2^b
template <typename W>
__device__ __forceinline__ W shoup_lazy(W a, W w, W wp, W Q) {
    W qt = WordOps<W>::mulhi(a, wp);
    return a * w - qt * Q;
}
template <typename W>
__device__ __forceinline__ W csub(W a, W Q) {
    return a >= Q ? a - Q : a;
}
template <typename W>
__device__ __forceinline__ W shoup(W a, W w, W wp, W Q) {
    return csub<W>(shoup_lazy<W>(a, w, wp, Q), Q);
}
template <typename W>
__device__ __forceinline__ W addm(W a, W b, W Q) {
    return csub<W>(a + b, Q);
}
template <typename W>
__device__ __forceinline__ W subm(W a, W b, W Q) {
    return a >= b ? a - b : a + (Q - b);
}
// x mod Q for any x < 2^b, with r1 = floor(2^b / Q) (Shoup with w = 1)
template <typename W>
__device__ __forceinline__ W reduce_full(W x, W r1, W Q) {
    return csub<W>(x - WordOps<W>::mulhi(x, r1) * Q, Q);
}

// Exact FP64 modular product (the arithmetic of blind_rotate_f64.hip; also timed alone by
// tools/microbench/valu_rates.hip, which includes this header, for that kernel's roofline peak).
// a, b integers held exactly in doubles with |a b| < 2^102:
//     h = a*b (rounded), l = fma(a, b, -h)          a*b = h + l exactly
//     q = rint(h / Q),   r = fma(-q, Q, h) + l      r = a*b - qQ exactly, |r| <~ Q/2
__device__ __forceinline__ double fmodmul_f64(double a, double b, double Q, double Qinv) {
    const double h = __dmul_rn(a, b);
    const double l = __fma_rn(a, b, -h);
    const double q = __builtin_rint(__dmul_rn(h, Qinv));
    return __dadd_rn(__fma_rn(-q, Q, h), l);
}

// Special-form product for Q = 2^54 - c, c < 2^20 (the sf kernels of blind_rotate_generic.hip;
// also timed alone by tools/microbench/valu_rates.hip).  The constant w is held as (W0, W1) =
// (w, w 2^32 mod Q), both < Q; for ANY a < 2^64, a0 = a mod 2^32, a1 = a >> 32 (register halves):
//     S = a0 W0 + a1 W1 < 2^87
//     P = a0 W0lo + a1 W1lo < 2^65       (one carry out of 64 bits)
//     H = a0 W0hi + a1 W1hi + P.hi + carry 2^32 = S >> 32 < 2^55
//     r = (S mod 2^55) + (S >> 55) c2 < 2^55 + 2^32 c2,   c2 = 2c (2^55 = 2c mod Q),   r = a w mod Q
// Nine VALU: five v_mad_u64_u32, the mov that zero-extends P.hi into an aligned pair, one
// v_addc_co_u32 (the carry, kept in the SGPR lane mask v_mad_u64_u32 writes), alignbit, and.
// Round 3's form (31/31 split of a < 2^61, W1 = w 2^31, fold at 2^54) took eleven: the split
// cost an and + alignbit and the P.hi addend an extra 64-bit add.  The carry mad and the
// H mads are written out so the addends stay fused; the addc reads the carry at least three
// VALU after the mad that wrote it (it depends on both H mads), which covers gfx950's
// SGPR-write -> carry-read hazard (two wait states) without an s_nop.
// tools/bounds_sf.py checks S, H and every lazily reduced input of the sf kernels.
constexpr uint32_t SF_K = 54;
__device__ __forceinline__ uint64_t sf_mul(uint64_t a, uint64_t w0, uint64_t w1, uint32_t c2) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint64_t P1 = (uint64_t)a0 * (uint32_t)w0;
    uint64_t P, H, cy, junk0, junk1, junk2;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(P), "=s"(cy) : "v"(a1), "v"((uint32_t)w1), "v"(P1));
    const uint64_t X = P >> 32;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(H), "=s"(junk0) : "v"(a0), "v"((uint32_t)(w0 >> 32)), "v"(X));
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(H), "=s"(junk1) : "v"(a1), "v"((uint32_t)(w1 >> 32)));
    uint32_t hh;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(hh), "=s"(junk2) : "v"((uint32_t)(H >> 32)), "s"(cy));
    const uint32_t hl = (uint32_t)H;
    const uint32_t hs = __builtin_amdgcn_alignbit(hh, hl, 23);  // S >> 55 < 2^32
    const uint64_t L = ((uint64_t)(hl & 0x7fffffu) << 32) | (uint32_t)P;  // S mod 2^55
    return L + (uint64_t)hs * c2;
}

// lwe-pke.cpp:41-46 RoundqQ: floor(0.5 + (double)v * (double)q / (double)Q) % q,
// with explicitly rounded IEEE operations (no contraction, no fast-math).
__device__ __forceinline__ uint64_t round_qQ(uint64_t v, uint64_t q, uint64_t Q) {
    double t = __dmul_rn((double)v, (double)q);
    double u = __ddiv_rn(t, (double)Q);
    return (uint64_t)floor(__dadd_rn(0.5, u)) % q;
}

// Rotation exponents a'_i = ((amod - a_i) mod amod) * (2N / amod) of one ciphertext
// (rgsw-acc-cggi.cpp:153, bootstrapping.cu:1623), written to LDS once at kernel start by the whole
// workgroup, so the round loops carry no 64-bit remainder.  The caller synchronises the workgroup
// before the first read.
template <int TH>
__device__ __forceinline__ void stage_rot_exponents(uint32_t* ex, const uint64_t* ap, uint32_t n, uint64_t amod,
                                                    uint32_t twoN) {
    const uint64_t scale = (uint64_t)twoN / amod;
    for (uint32_t k = threadIdx.x; k < n; k += TH) {
        const uint64_t ar = ap[k] % amod;
        ex[k] = (uint32_t)((ar == 0 ? 0 : amod - ar) * scale);
    }
}
__host__ __device__ constexpr size_t rot_exponent_bytes(uint32_t n) { return ((size_t)n * 4 + 15) & ~(size_t)15; }

// The NTT-half duo kernels (f64wduo, blind_rotate_f64.hip; sfduo, blind_rotate_generic.hip): buffer index of
// element x of a half polynomial (block x >> 8, y = x & 255).  y's low five bits are XORed with f(y[7:5]):
// bit 5 -> bits 1, 3; bit 6 -> bit 4; bit 4 -> bits 0, 2, so that every b64 read is conflict-free per 32-lane
// group (64 banks) AND every b64 write per 16-lane group (32 banks; MI355X_MICROARCH.md "LDS"), for every pass,
// the cross-wave digit exchange and the units (tools/lds_layouts_duo.py; the round-5 first form, bits 5-7 into
// bits 0-4 only, left the writes of passes (7,8), (10,9), (8,7) and the exchange 2-way).  Both kernels hold
// 8-byte words, so the analysis covers both.
__device__ __forceinline__ uint32_t dswz(uint32_t x) {
    return x ^ (((x >> 5) & 1) * 10u) ^ (((x >> 6) & 1) << 4) ^ (((x >> 4) & 1) * 5u);
}

}  // namespace tfhe
