// blind_rotate_fast.hip -- CGGI blind rotation specialised for the STD128 class
// (N = 1024, dG2 = 8, baseG = 2^7, Q < 2^27; STD128, STD128_OPT).
//
// Same math as the generic kernel and the oracle (rgsw-acc-cggi.cpp:246-307 and
// rgsw-acc.cpp:57-111), re-organised for gfx950:
//
//  * Two wavefronts (128 lanes) per ciphertext, two ciphertexts per workgroup.
//    A lane holds 8 coefficients of each polynomial; a 1024-point negacyclic
//    transform is four in-register radix-8 passes (3+3+3+1 Cooley-Tukey stages)
//    separated by three LDS exchanges.  Layouts (index bits b9..b0, lane t < 128,
//    register r < 8):
//        L1  r=(b9 b8 b7)  t=(b6..b0)            i = 128r + t
//        L2  r=(b6 b5 b4)  t=(b9 b8 b7 b3..b0)    i = 128(t>>4) + 16r + (t&15)
//        L3  r=(b3 b2 b1)  t=(b9..b4 b0)          i = 16(t>>1) + 2r + (t&1)
//        L4  r=(b2 b1 b0)  t=(b9..b3)             i = 8t + r
//    The wavefront bit (t bit 6) is b9 in L2..L4, so only the L1<->L2 exchange
//    crosses wavefronts (workgroup barrier); the others are wave-local.
//    Forward NTT: L1 -> L4.  Pointwise external product in L4, where a lane owns
//    8 consecutive NTT slots, so every BSK read is two 16-byte loads.  INTT:
//    L4 -> L1, so the accumulator never leaves registers in coefficient order.
//
//  * Montgomery arithmetic (R = 2^32) through v_mad_u64_u32, which gfx950 issues
//    at the rate of v_mul_lo_u32 (profiles/r01_valu_rates.txt):
//        redc(T) = hi32(m*Q + T),  m = lo32(T) * (-Q^-1)        (T < 2^62)
//    A twiddle product is 3 instructions and needs no Shoup companion, so the
//    BSK is stored once (u32, Montgomery form, pre-scaled by N^-1).  The 8-row
//    external product accumulates exact 64-bit sums (one v_mad_u64_u32 per term)
//    and reduces once per output.
//
//  * Lazy ranges (Q < 2^27): forward CT butterflies grow values by < 2Q per
//    stage and never reduce (digits enter < 2Q, outputs < 22Q < 2^32); inverse GS
//    butterflies keep values < 2Q; the accumulator is reduced to [0, Q) once per
//    round, which the next decomposition needs.
#include <cstdlib>

#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {
namespace {

constexpr uint32_t FN = 1024;
constexpr uint32_t FDG2 = 8;
constexpr uint32_t FDIG = 4;
constexpr uint32_t FLOGG = 7;
constexpr int TPC = 128;  // threads per ciphertext
constexpr int CTS = 2;    // ciphertexts per workgroup
constexpr int THREADS = TPC * CTS;

// device table block (words): psiM[1024] ipsiM[1024] monoM[2048] eidx[1024]
constexpr uint32_t T_PSI = 0, T_IPSI = 1024, T_MONO = 2048, T_EIDX = 4096, T_WORDS = 5120;
constexpr uint32_t PFN = FN + FN / 8;      // padded polynomial (swz)
constexpr uint32_t BUF_WORDS = 2 * PFN;    // per ciphertext: two polynomials
constexpr size_t LDS_BYTES = (size_t)(T_WORDS + CTS * BUF_WORDS) * 4;

struct FastConst {
    uint32_t Q, qinv, twoQ, Qhalf;
};

__device__ __forceinline__ uint32_t redc(uint64_t T, uint32_t Q, uint32_t qinv) {
    const uint32_t m = (uint32_t)T * qinv;
    return (uint32_t)(((uint64_t)m * Q + T) >> 32);
}
__device__ __forceinline__ uint32_t mmul(uint32_t a, uint32_t bM, const FastConst& K) {
    return redc((uint64_t)a * bM, K.Q, K.qinv);
}
__device__ __forceinline__ uint32_t csub32(uint32_t a, uint32_t m) { return min(a, a - m); }

// LDS word index of natural index i: 2 pad words per 16.  Affine in the register
// index for all four layouts (address = base(lane) + immediate), and at most
// 2-way bank conflicts per 32-lane group (exhaustive search, tools/ notes).
__device__ __forceinline__ uint32_t swz(uint32_t i) { return i + 2 * (i >> 4); }

__device__ __forceinline__ uint32_t ix1(uint32_t t, uint32_t r) { return r * 128 + t; }
__device__ __forceinline__ uint32_t ix2(uint32_t t, uint32_t r) { return (t >> 4) * 128 + r * 16 + (t & 15); }
__device__ __forceinline__ uint32_t ix3(uint32_t t, uint32_t r) { return (t >> 1) * 16 + r * 2 + (t & 1); }
__device__ __forceinline__ uint32_t ix4(uint32_t t, uint32_t r) { return t * 8 + r; }

template <int L>
__device__ __forceinline__ uint32_t ix(uint32_t t, uint32_t r) {
    if constexpr (L == 1) return ix1(t, r);
    else if constexpr (L == 2) return ix2(t, r);
    else if constexpr (L == 3) return ix3(t, r);
    else return ix4(t, r);
}

template <int L>
__device__ __forceinline__ void lds_store(uint32_t* buf, const uint32_t (&x)[8], uint32_t t) {
#pragma unroll
    for (uint32_t r = 0; r < 8; ++r) buf[swz(ix<L>(t, r))] = x[r];
}
template <int L>
__device__ __forceinline__ void lds_load(const uint32_t* buf, uint32_t (&x)[8], uint32_t t) {
#pragma unroll
    for (uint32_t r = 0; r < 8; ++r) x[r] = buf[swz(ix<L>(t, r))];
}

// An opaque zero: adding it to a table base stops the compiler from hoisting the
// (loop-invariant) twiddle loads out of the round loop into registers, which
// would cost ~36 VGPRs for values one LDS read away.
__device__ __forceinline__ uint32_t opaque_zero() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

// ordering of LDS traffic between lanes of one wavefront
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void bfly_ct(uint32_t& a, uint32_t& b, uint32_t w, const FastConst& K) {
    const uint32_t v = mmul(b, w, K), u = a;
    a = u + v;
    b = u - v + K.twoQ;
}
__device__ __forceinline__ void bfly_gs(uint32_t& a, uint32_t& b, uint32_t w, const FastConst& K) {
    const uint32_t u = a, v = b;
    a = csub32(u + v, K.twoQ);
    b = mmul(u - v + K.twoQ, w, K);
}

// radix-8 Cooley-Tukey pass over register bits (r2, r1, r0) = three index bits,
// twiddle psi[2^s + block] with block prefix c; FULL=false runs only the r0 stage.
template <bool FULL>
__device__ __forceinline__ void fwd_pass(uint32_t (&x)[8], const uint32_t* psi, uint32_t m, uint32_t c,
                                         const FastConst& K) {
    if constexpr (FULL) {
        const uint32_t w = psi[m + c];
#pragma unroll
        for (int r = 0; r < 4; ++r) bfly_ct(x[r], x[r + 4], w, K);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t w1 = psi[2 * m + 2 * c + h];
            bfly_ct(x[4 * h], x[4 * h + 2], w1, K);
            bfly_ct(x[4 * h + 1], x[4 * h + 3], w1, K);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) bfly_ct(x[2 * q], x[2 * q + 1], psi[4 * m + 4 * c + q], K);
}

template <bool FULL>
__device__ __forceinline__ void inv_pass(uint32_t (&x)[8], const uint32_t* ipsi, uint32_t m, uint32_t c,
                                         const FastConst& K) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bfly_gs(x[2 * q], x[2 * q + 1], ipsi[4 * m + 4 * c + q], K);
    if constexpr (FULL) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t w1 = ipsi[2 * m + 2 * c + h];
            bfly_gs(x[4 * h], x[4 * h + 2], w1, K);
            bfly_gs(x[4 * h + 1], x[4 * h + 3], w1, K);
        }
        const uint32_t w = ipsi[m + c];
#pragma unroll
        for (int r = 0; r < 4; ++r) bfly_gs(x[r], x[r + 4], w, K);
    }
}

// forward transform of two polynomials, L1 -> L4 (one cross-wave exchange)
__device__ __forceinline__ void ntt_fwd2(uint32_t (&x0)[8], uint32_t (&x1)[8], uint32_t* buf, const uint32_t* psi,
                                         uint32_t t, const FastConst& K) {
    fwd_pass<true>(x0, psi, 1, 0, K);
    fwd_pass<true>(x1, psi, 1, 0, K);
    __syncthreads();  // the other wavefront has finished reading buf
    lds_store<1>(buf, x0, t);
    lds_store<1>(buf + PFN, x1, t);
    __syncthreads();
    lds_load<2>(buf, x0, t);
    lds_load<2>(buf + PFN, x1, t);
    fwd_pass<true>(x0, psi, 8, t >> 4, K);
    fwd_pass<true>(x1, psi, 8, t >> 4, K);
    wave_sync();
    lds_store<2>(buf, x0, t);
    lds_store<2>(buf + PFN, x1, t);
    wave_sync();
    lds_load<3>(buf, x0, t);
    lds_load<3>(buf + PFN, x1, t);
    fwd_pass<true>(x0, psi, 64, t >> 1, K);
    fwd_pass<true>(x1, psi, 64, t >> 1, K);
    wave_sync();
    lds_store<3>(buf, x0, t);
    lds_store<3>(buf + PFN, x1, t);
    wave_sync();
    lds_load<4>(buf, x0, t);
    lds_load<4>(buf + PFN, x1, t);
    fwd_pass<false>(x0, psi, 128, t, K);
    fwd_pass<false>(x1, psi, 128, t, K);
}

// inverse transform of two polynomials (no N^-1: folded into the BSK), L4 -> L1
__device__ __forceinline__ void ntt_inv2(uint32_t (&x0)[8], uint32_t (&x1)[8], uint32_t* buf, const uint32_t* ipsi,
                                         uint32_t t, const FastConst& K) {
    inv_pass<false>(x0, ipsi, 128, t, K);
    inv_pass<false>(x1, ipsi, 128, t, K);
    wave_sync();
    lds_store<4>(buf, x0, t);
    lds_store<4>(buf + PFN, x1, t);
    wave_sync();
    lds_load<3>(buf, x0, t);
    lds_load<3>(buf + PFN, x1, t);
    inv_pass<true>(x0, ipsi, 64, t >> 1, K);
    inv_pass<true>(x1, ipsi, 64, t >> 1, K);
    wave_sync();
    lds_store<3>(buf, x0, t);
    lds_store<3>(buf + PFN, x1, t);
    wave_sync();
    lds_load<2>(buf, x0, t);
    lds_load<2>(buf + PFN, x1, t);
    inv_pass<true>(x0, ipsi, 8, t >> 4, K);
    inv_pass<true>(x1, ipsi, 8, t >> 4, K);
    wave_sync();
    lds_store<2>(buf, x0, t);  // own half (b9 = wavefront)
    lds_store<2>(buf + PFN, x1, t);
    __syncthreads();
    lds_load<1>(buf, x0, t);
    lds_load<1>(buf + PFN, x1, t);
    inv_pass<true>(x0, ipsi, 1, 0, K);
    inv_pass<true>(x1, ipsi, 1, 0, K);
}

// MINW: minimum waves per SIMD requested from the register allocator;
// ACC32: reduce every digit pair into 32-bit accumulators (fewer VGPRs, +2 ops per term pair);
// RECOMP: recompute digit l from the accumulator in pass l instead of carrying the
//         16-register decomposition state (fewer VGPRs, +3 ops per extra digit step)
template <int MINW, bool ACC32, bool RECOMP = false>
__global__ void __launch_bounds__(THREADS, MINW)
k_blind_rotate_fast(FastConst K, uint32_t n, uint32_t loga, const uint32_t* __restrict__ tabs,
                    const uint32_t* __restrict__ bsk, const uint64_t* __restrict__ a, uint64_t* __restrict__ acc_io,
                    uint32_t B) {
    extern __shared__ __align__(16) uint32_t lds[];
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < T_WORDS; k += THREADS) lds[k] = tabs[k];
    const uint32_t cl = tid / TPC, t = tid % TPC;
    const uint32_t ct = blockIdx.x * CTS + cl;
    const bool active = ct < B;
    uint32_t* buf = lds + T_WORDS + cl * BUF_WORDS;
    const uint32_t* psi = lds + T_PSI;
    const uint32_t* ipsi = lds + T_IPSI;
    const uint32_t* mono = lds + T_MONO;
    const uint32_t* eidx = lds + T_EIDX;

    uint64_t* g = acc_io + (size_t)(active ? ct : 0) * 2 * FN;
    uint32_t acc[2][8];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            uint64_t v = active ? g[p * FN + ix1(t, r)] : 0;
            acc[p][r] = (uint32_t)(v >= K.Q ? v % K.Q : v);
        }
    __syncthreads();

    const uint64_t* ap = a + (size_t)(active ? ct : 0) * n;
    const uint32_t amask = (1u << loga) - 1, ashift = 11 - loga;  // 2N = 2^11
    for (uint32_t i = 0; i < n; ++i) {
        // a'_i = ((amod - a_i) mod amod) * (2N / amod)  (rgsw-acc-cggi.cpp:153)
        const uint32_t ar = active ? (uint32_t)(ap[i] & amask) : 0;
        const uint32_t ai = ((amask + 1 - ar) & amask) << ashift;

        int32_t d[2][8];  // centred coefficients, consumed digit by digit (rgsw-acc.cpp:83-109)
        if constexpr (!RECOMP) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    d[p][r] = acc[p][r] < K.Qhalf ? (int32_t)acc[p][r] : (int32_t)(acc[p][r] - K.Q);
        }

        uint64_t s[2][2][8];   // exact 64-bit sums (ACC32 = false)
        uint32_t s32[2][2][8]; // per-pair reduced sums < 4 * 2.4Q (ACC32 = true)
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    if constexpr (ACC32) s32[k][j][r] = 0;
                    else s[k][j][r] = 0;
                }

        // wave-uniform round base (SGPRs) + 32-bit lane offset: global_load_dwordx4 v, voff, s[base]
        const uint32_t* ek = bsk + (size_t)i * (2 * FDG2 * 2 * FN);
        const uint32_t toff = t * 8;
#pragma unroll 1
        for (uint32_t l = 0; l < FDIG; ++l) {
            uint32_t x0[8], x1[8];
            if constexpr (RECOMP) {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    int32_t e0 = acc[0][r] < K.Qhalf ? (int32_t)acc[0][r] : (int32_t)(acc[0][r] - K.Q);
                    int32_t e1 = acc[1][r] < K.Qhalf ? (int32_t)acc[1][r] : (int32_t)(acc[1][r] - K.Q);
                    for (uint32_t z = 0; z < l; ++z) {  // drop the l lower digits (carries included)
                        e0 = (e0 - ((e0 << (32 - FLOGG)) >> (32 - FLOGG))) >> FLOGG;
                        e1 = (e1 - ((e1 << (32 - FLOGG)) >> (32 - FLOGG))) >> FLOGG;
                    }
                    x0[r] = (uint32_t)(((e0 << (32 - FLOGG)) >> (32 - FLOGG)) + (int32_t)K.Q);
                    x1[r] = (uint32_t)(((e1 << (32 - FLOGG)) >> (32 - FLOGG)) + (int32_t)K.Q);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const int32_t r0 = (d[0][r] << (32 - FLOGG)) >> (32 - FLOGG);  // signed low digit
                    const int32_t r1 = (d[1][r] << (32 - FLOGG)) >> (32 - FLOGG);
                    d[0][r] = (d[0][r] - r0) >> FLOGG;
                    d[1][r] = (d[1][r] - r1) >> FLOGG;
                    x0[r] = (uint32_t)(r0 + (int32_t)K.Q);  // = r mod Q, in [Q-64, Q+64)
                    x1[r] = (uint32_t)(r1 + (int32_t)K.Q);
                }
            }
            ntt_fwd2(x0, x1, buf, psi + opaque_zero(), t, K);
            // rows 2l (poly 0, digit l) and 2l+1 (poly 1, digit l)
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t* r0p = ek + ((k * FDG2 + 2 * l) * 2 + j) * FN;      // uniform
                    const uint32_t* r1p = ek + ((k * FDG2 + 2 * l + 1) * 2 + j) * FN;  // uniform
                    const uint4* e0 = reinterpret_cast<const uint4*>(r0p + toff);
                    const uint4* e1 = reinterpret_cast<const uint4*>(r1p + toff);
                    // one (key, poly) group of BSK words at a time: bounds the staging registers
                    __builtin_amdgcn_sched_barrier(0);
                    const uint4 a0 = e0[0], a1 = e0[1], b0 = e1[0], b1 = e1[1];
                    const uint32_t w0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                    const uint32_t w1[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        if constexpr (ACC32) {
                            const uint64_t T = (uint64_t)x0[r] * w0[r] + (uint64_t)x1[r] * w1[r];
                            s32[k][j][r] += redc(T, K.Q, K.qinv);
                        } else {  // two chained v_mad_u64_u32 into the exact sum
                            s[k][j][r] = (uint64_t)x0[r] * w0[r] + s[k][j][r];
                            s[k][j][r] = (uint64_t)x1[r] * w1[r] + s[k][j][r];
                        }
                    }
                }
        }

        // S_j = A_0j * NTT(X^a' - 1) + A_1j * NTT(X^-a' - 1)
        uint32_t S0[8], S1[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t ip = (eidx[t * 8 + r] * ai) & (2 * FN - 1);
            const uint32_t in = (2 * FN - ip) & (2 * FN - 1);
            const uint32_t mp = mono[ip], mn = mono[in];
            uint32_t A00, A01, A10, A11;
            if constexpr (ACC32) {
                A00 = s32[0][0][r], A01 = s32[0][1][r], A10 = s32[1][0][r], A11 = s32[1][1][r];
            } else {
                A00 = redc(s[0][0][r], K.Q, K.qinv), A01 = redc(s[0][1][r], K.Q, K.qinv);
                A10 = redc(s[1][0][r], K.Q, K.qinv), A11 = redc(s[1][1][r], K.Q, K.qinv);
            }
            S0[r] = redc((uint64_t)A00 * mp + (uint64_t)A10 * mn, K.Q, K.qinv);
            S1[r] = redc((uint64_t)A01 * mp + (uint64_t)A11 * mn, K.Q, K.qinv);
        }
        ntt_inv2(S0, S1, buf, ipsi + opaque_zero(), t, K);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            acc[0][r] = csub32(csub32(acc[0][r] + S0[r], K.twoQ), K.Q);
            acc[1][r] = csub32(csub32(acc[1][r] + S1[r], K.twoQ), K.Q);
        }
    }
    if (active) {
        // acc0 transposed (X -> X^-1, poly.cpp:762-770): out[(N-k) mod N] = -acc0[k]
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t k = ix1(t, r), v = acc[0][r];
            g[(FN - k) & (FN - 1)] = k == 0 ? v : (v == 0 ? 0 : K.Q - v);
            g[FN + k] = acc[1][r];
        }
    }
}

// generic (plain, N^-1-scaled) BSK and tables -> Montgomery-form copies
__global__ void k_pack_fast(uint32_t Q, const uint32_t* __restrict__ bsk, size_t words, const uint32_t* __restrict__ psi,
                            const uint32_t* __restrict__ ipsi, const uint32_t* __restrict__ mono,
                            const uint32_t* __restrict__ eidx, uint32_t* __restrict__ out) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto mont = [Q](uint32_t v) { return (uint32_t)(((uint64_t)v << 32) % Q); };
    if (idx < words) out[T_WORDS + idx] = mont(bsk[idx]);
    if (idx < FN) {
        out[T_PSI + idx] = mont(psi[idx]);
        out[T_IPSI + idx] = mont(ipsi[idx]);
        out[T_EIDX + idx] = eidx[idx];
    }
    if (idx < 2 * FN) out[T_MONO + idx] = mont(mono[idx]);
}

}  // namespace

bool fast_path_supported(const BRParams& P, int word_bits) {
    return word_bits == 32 && P.N == FN && P.dG2 == FDG2 && P.digits == FDIG && P.thr == 0 && P.logG == FLOGG &&
           P.Q < (1ull << 27) && P.n > 0;
}

size_t bsk_fast_bytes(const BRParams& P) { return ((size_t)P.n * 2 * FDG2 * 2 * FN + T_WORDS) * 4; }

hipError_t launch_pack_bsk_fast(const BRParams& P, const DevTables& T, const void* bsk, void* bsk_fast,
                                hipStream_t s) {
    const size_t words = (size_t)P.n * 2 * FDG2 * 2 * FN;
    hipLaunchKernelGGL(k_pack_fast, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, (uint32_t)P.Q,
                       (const uint32_t*)bsk, words, (const uint32_t*)T.psi, (const uint32_t*)T.ipsi,
                       (const uint32_t*)T.mono, T.eidx, (uint32_t*)bsk_fast);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_fast(const BRParams& P, const DevTables&, const void* bsk_fast, const uint64_t* a,
                                    uint64_t amod, uint64_t* acc, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    if (amod == 0 || (amod & (amod - 1)) || amod > 2 * FN) return hipErrorNotSupported;
    uint32_t loga = 0;
    while ((1ull << loga) < amod) ++loga;
    FastConst K;
    K.Q = (uint32_t)P.Q;
    uint32_t inv = 1;  // Q^-1 mod 2^32 by Newton iteration
    for (int it = 0; it < 5; ++it) inv *= 2u - K.Q * inv;
    K.qinv = 0u - inv;
    K.twoQ = 2 * K.Q;
    K.Qhalf = K.Q >> 1;
    const uint32_t* tabs = (const uint32_t*)bsk_fast;
    const uint32_t* bsk = tabs + T_WORDS;
    static const int variant = [] {
        const char* e = std::getenv("TFHE_FAST_VARIANT");
        return e ? std::atoi(e) : 0;
    }();
    // default: 3 waves/SIMD with per-pair 32-bit accumulation (fastest measured,
    // tools/variant_sweep.sh: 68.6 ms vs 75.1 ms for <2,false> per 8192-batch)
    auto k = k_blind_rotate_fast<3, true>;
    switch (variant) {
        case 1: k = k_blind_rotate_fast<3, false>; break;
        case 5: k = k_blind_rotate_fast<2, false>; break;
        case 3: k = k_blind_rotate_fast<4, true>; break;
        case 4: k = k_blind_rotate_fast<2, true>; break;
        case 6: k = k_blind_rotate_fast<4, true, true>; break;
        case 7: k = k_blind_rotate_fast<3, true, true>; break;
        default: break;
    }
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES);
    hipLaunchKernelGGL(k, dim3((unsigned)((B + CTS - 1) / CTS)), dim3(THREADS), LDS_BYTES, s, K, P.n, loga, tabs,
                       bsk, a, acc, (uint32_t)B);
    return hipGetLastError();
}

}  // namespace tfhe
