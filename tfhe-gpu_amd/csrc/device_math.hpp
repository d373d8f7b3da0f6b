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

}  // namespace tfhe
