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
//  * Signed Montgomery arithmetic (R = 2^32) on v_mad_i64_i32, which gfx950 issues
//    at the rate of v_mul_lo_u32 (profiles/r01_valu_rates.txt).  Every value is a
//    signed 32-bit representative; constants (twiddles, BSK, monomials) are stored
//    centred (|w| <= Q/2) in Montgomery form:
//        sredc(T) = hi32(T - m*Q),  m = lo32(T) * Q^-1   (one v_mul_lo + one v_mad_i64_i32)
//    |sredc(T)| <= |T|/2^32 + Q/2.  A twiddle product is 3 instructions, a CT
//    butterfly 5 (no "+2Q" offsets, no conditional subtractions), a GS butterfly 5.
//    Value bounds (tools/bounds_fast.py checks them): forward outputs < 6.3Q + 64;
//    inverse passes keep everything < 16Q by reducing the two a-paths that would
//    double a third time; every 64-bit sum stays < 2^60.
//
//  * The accumulator is kept as the centred canonical representative in
//    [-(Q>>1)-1, Q>>1), exactly OpenFHE's signed view before its digit
//    decomposition (rgsw-acc.cpp:83-109), so a digit is one v_bfe_i32 and the carry
//    two instructions; the top digit is the remainder itself.
//
//  * Monomials: NTT(X^m - 1)[x] = psi^(e_x m) - 1 with e_x = 2 bitrev(x) + 1
//    (checked at setup), so in L4 e = 256 bitrev3(r) + (2 bitrev7(t) + 1): one
//    per-lane product per round plus a wave-uniform stride, and one 2N-entry table.
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

// device table block (int32 words, centred Montgomery): psi[1024] ipsi[1024] mono[2048]
constexpr uint32_t T_PSI = 0, T_IPSI = 1024, T_MONO = 2048, T_WORDS = 4096;
constexpr uint32_t PFN = FN + FN / 8;      // padded polynomial (swz)
constexpr uint32_t BUF_WORDS = 2 * PFN;    // per ciphertext: two polynomials
constexpr size_t lds_bytes(int cts) { return (size_t)(T_WORDS + cts * BUF_WORDS) * 4; }

struct FastConst {
    int32_t Q, nQ, qinv, rM;  // rM = R mod Q (centred): smul(x, rM) reduces x
    uint32_t Q2, Q4, h1, kacc;  // 2Q, 4Q, (Q>>1)+1, (Q>>1)+1+4Q
};

__device__ __forceinline__ int32_t sredc(int64_t T, const FastConst& K) {
    const int32_t m = (int32_t)((uint32_t)T * (uint32_t)K.qinv);
    return (int32_t)(((int64_t)m * K.nQ + T) >> 32);
}
__device__ __forceinline__ int32_t smul(int32_t a, int32_t wM, const FastConst& K) {
    return sredc((int64_t)a * wM, K);
}
__device__ __forceinline__ uint32_t csub32(uint32_t a, uint32_t m) { return min(a, a - m); }

typedef int32_t v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i ld_bsk(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}

// LDS word index of natural index i: 2 pad words per 16.  Affine in the register
// index for all four layouts (address = base(lane) + immediate), and at most
// 2-way bank conflicts per 32-lane group.
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
__device__ __forceinline__ void lds_store(int32_t* buf, const int32_t (&x)[8], uint32_t t) {
#pragma unroll
    for (uint32_t r = 0; r < 8; ++r) buf[swz(ix<L>(t, r))] = x[r];
}
template <int L>
__device__ __forceinline__ void lds_load(const int32_t* buf, int32_t (&x)[8], uint32_t t) {
#pragma unroll
    for (uint32_t r = 0; r < 8; ++r) x[r] = buf[swz(ix<L>(t, r))];
}

// An opaque zero: adding it to a table base stops the compiler from hoisting the
// (loop-invariant) twiddle loads out of the round loop into registers.
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

// Cooley-Tukey: (a, b) -> (a + wb, a - wb);  |out| <= |a| + |b||w|/2^32 + Q/2
__device__ __forceinline__ void bfly_ct(int32_t& a, int32_t& b, int32_t w, const FastConst& K) {
    const int32_t v = smul(b, w, K), u = a;
    a = u + v;
    b = u - v;
}
// Gentleman-Sande: (a, b) -> (a + b, (a - b) w); RED also reduces the sum
template <bool RED = false>
__device__ __forceinline__ void bfly_gs(int32_t& a, int32_t& b, int32_t w, const FastConst& K) {
    const int32_t u = a, v = b;
    a = RED ? smul(u + v, K.rM, K) : u + v;
    b = smul(u - v, w, K);
}

// radix-8 Cooley-Tukey pass over register bits (r2, r1, r0) = three index bits,
// twiddle psi[2^s + block] with block prefix c; FULL=false runs only the r0 stage.
template <bool FULL>
__device__ __forceinline__ void fwd_pass(int32_t (&x)[8], const int32_t* psi, uint32_t m, uint32_t c,
                                         const FastConst& K) {
    if constexpr (FULL) {
        const int32_t w = psi[m + c];
#pragma unroll
        for (int r = 0; r < 4; ++r) bfly_ct(x[r], x[r + 4], w, K);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int32_t w1 = psi[2 * m + 2 * c + h];
            bfly_ct(x[4 * h], x[4 * h + 2], w1, K);
            bfly_ct(x[4 * h + 1], x[4 * h + 3], w1, K);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) bfly_ct(x[2 * q], x[2 * q + 1], psi[4 * m + 4 * c + q], K);
}

// Inverse radix-8 pass.  With inputs < B the doubling a-paths reach 4B after two
// stages; x[0] and x[4] (the only ones) are reduced there, so the outputs stay < 3Q
// for any B <= 3Q (tools/bounds_fast.py).
template <bool FULL>
__device__ __forceinline__ void inv_pass(int32_t (&x)[8], const int32_t* ipsi, uint32_t m, uint32_t c,
                                         const FastConst& K) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bfly_gs(x[2 * q], x[2 * q + 1], ipsi[4 * m + 4 * c + q], K);
    if constexpr (FULL) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int32_t w1 = ipsi[2 * m + 2 * c + h];
            bfly_gs<true>(x[4 * h], x[4 * h + 2], w1, K);
            bfly_gs(x[4 * h + 1], x[4 * h + 3], w1, K);
        }
        const int32_t w = ipsi[m + c];
#pragma unroll
        for (int r = 0; r < 4; ++r) bfly_gs(x[r], x[r + 4], w, K);
    }
}

// forward transform of two polynomials, L1 -> L4 (one cross-wave exchange)
__device__ __forceinline__ void ntt_fwd2(int32_t (&x0)[8], int32_t (&x1)[8], int32_t* buf, const int32_t* psi,
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
__device__ __forceinline__ void ntt_inv2(int32_t (&x0)[8], int32_t (&x1)[8], int32_t* buf, const int32_t* ipsi,
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

// MINW: minimum waves per SIMD requested from the register allocator.
// ACC64: exact 64-bit sums over all 8 rows, one reduction per output (32 more VGPRs);
//        otherwise every digit's row pair is reduced into a 32-bit sum.
// CTS: ciphertexts per workgroup (a workgroup barrier then spans 2*CTS wavefronts).
template <int MINW, bool ACC64, int CTS>
__global__ void __launch_bounds__(TPC * CTS, MINW)
k_blind_rotate_fast(FastConst K, uint32_t n, uint32_t loga, const int32_t* __restrict__ tabs,
                    const int32_t* __restrict__ bsk, const uint64_t* __restrict__ a, uint64_t* __restrict__ acc_io,
                    uint32_t B) {
    extern __shared__ __align__(16) int32_t lds[];
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < T_WORDS; k += TPC * CTS) lds[k] = tabs[k];
    const uint32_t cl = __builtin_amdgcn_readfirstlane(tid / TPC), t = tid % TPC;
    const uint32_t ct = blockIdx.x * CTS + cl;
    const bool active = ct < B;
    int32_t* buf = lds + T_WORDS + cl * BUF_WORDS;
    const int32_t* psi = lds + T_PSI;
    const int32_t* ipsi = lds + T_IPSI;
    const char* mono = reinterpret_cast<const char*>(lds + T_MONO);

    uint64_t* g = acc_io + (size_t)(active ? ct : 0) * 2 * FN;
    const uint32_t Qh = (uint32_t)K.Q >> 1;
    int32_t acc[2][8];  // centred canonical, [-(Q>>1)-1, Q>>1)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint64_t v0 = active ? g[p * FN + ix1(t, r)] : 0;
            const uint32_t v = (uint32_t)(v0 >= (uint64_t)K.Q ? v0 % (uint64_t)K.Q : v0);
            acc[p][r] = v < Qh ? (int32_t)v : (int32_t)v - K.Q;
        }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(bsk), 0, (int)(n * (2 * FDG2 * 2 * FN * 4)), 0x00020000);
    const uint32_t voff = t * 32;  // 8 consecutive words per lane in L4
    // slot exponent of L4 slot 8t + r: e = 256 bitrev3(r) + et, et = 2 bitrev7(t) + 1
    const uint32_t et = 2 * (__builtin_bitreverse32(t) >> 25) + 1;
    const uint64_t* ap = a + (size_t)(active ? ct : 0) * n;
    const uint32_t amask = (1u << loga) - 1, ashift = 11 - loga;  // 2N = 2^11
    for (uint32_t i = 0; i < n; ++i) {
        // a'_i = ((amod - a_i) mod amod) * (2N / amod)  (rgsw-acc-cggi.cpp:153)
        const uint32_t ar = active ? (uint32_t)(ap[i] & amask) : 0;
        const uint32_t ai = ((amask + 1 - ar) & amask) << ashift;

        int64_t s[2][2][8];   // ACC64: exact sums
        int32_t s32[2][2][8]; // otherwise: per-digit reduced sums
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    if constexpr (ACC64) s[k][j][r] = 0;
                    else s32[k][j][r] = 0;
                }

        // BSK rows through a buffer resource: lane offset in a VGPR, row offset in an SGPR
        const uint32_t round_off = i * (2 * FDG2 * 2 * FN * 4);
#pragma unroll
        for (uint32_t l = 0; l < FDIG; ++l) {
            // signed digit l of the centred c (rgsw-acc.cpp:83-109, carries included):
            //   d_l = (c + 64 (1 + 128 + ... + 128^(l-1))) >> 7l,  digit = sext7(d_l);
            //   the top digit |d_3| <= 33 is its own sext7, so one v_bfe_i32 serves all four
            const int32_t kl = (int32_t)(((1u << (FLOGG * l)) - 1) / ((1u << FLOGG) - 1)) << (FLOGG - 1);
            int32_t x0[8], x1[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                x0[r] = __builtin_amdgcn_sbfe(acc[0][r] + kl, FLOGG * l, FLOGG);
                x1[r] = __builtin_amdgcn_sbfe(acc[1][r] + kl, FLOGG * l, FLOGG);
            }
            ntt_fwd2(x0, x1, buf, psi + opaque_zero(), t, K);
            // rows 2l (poly 0, digit l) and 2l+1 (poly 1, digit l)
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t s0 = round_off + ((k * FDG2 + 2 * l) * 2 + j) * FN * 4;      // uniform
                    const uint32_t s1 = round_off + ((k * FDG2 + 2 * l + 1) * 2 + j) * FN * 4;  // uniform
                    // one (key, poly) group of BSK words at a time: bounds the staging registers
                    __builtin_amdgcn_sched_barrier(0);
                    const v4i a0 = ld_bsk(rsrc, voff, s0), a1 = ld_bsk(rsrc, voff + 16, s0);
                    const v4i b0 = ld_bsk(rsrc, voff, s1), b1 = ld_bsk(rsrc, voff + 16, s1);
                    const int32_t w0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                    const int32_t w1[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        if constexpr (ACC64) {
                            s[k][j][r] = (int64_t)x0[r] * w0[r] + s[k][j][r];
                            s[k][j][r] = (int64_t)x1[r] * w1[r] + s[k][j][r];
                        } else {
                            const int64_t T = (int64_t)x0[r] * w0[r] + (int64_t)x1[r] * w1[r];
                            s32[k][j][r] += sredc(T, K);
                        }
                    }
                }
        }

        // S_j = A_0j * NTT(X^a' - 1) + A_1j * NTT(X^-a' - 1)
        const uint32_t b4 = (et * ai) << 2;       // byte offsets into the 2N-entry table
        const uint32_t st4 = (ai << 10) & 8191;   // 256 * ai * 4 mod 8192
        int32_t S0[8], S1[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t c = __builtin_bitreverse32((uint32_t)r) >> 29;
            const uint32_t e4 = b4 + c * st4;
            const int32_t mp = *reinterpret_cast<const int32_t*>(mono + (e4 & 8188));
            const int32_t mn = *reinterpret_cast<const int32_t*>(mono + ((0u - e4) & 8188));
            int32_t A00, A01, A10, A11;
            if constexpr (ACC64) {
                A00 = sredc(s[0][0][r], K), A01 = sredc(s[0][1][r], K);
                A10 = sredc(s[1][0][r], K), A11 = sredc(s[1][1][r], K);
            } else {
                A00 = s32[0][0][r], A01 = s32[0][1][r], A10 = s32[1][0][r], A11 = s32[1][1][r];
            }
            S0[r] = sredc((int64_t)A00 * mp + (int64_t)A10 * mn, K);
            S1[r] = sredc((int64_t)A01 * mp + (int64_t)A11 * mn, K);
        }
        ntt_inv2(S0, S1, buf, ipsi + opaque_zero(), t, K);
        // acc <- centred canonical (acc + S): u = acc + S + (Q>>1) + 1 + 4Q in (0, 8Q)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            uint32_t u0 = (uint32_t)(acc[0][r] + S0[r]) + K.kacc;
            uint32_t u1 = (uint32_t)(acc[1][r] + S1[r]) + K.kacc;
            u0 = csub32(csub32(csub32(u0, K.Q4), K.Q2), (uint32_t)K.Q);
            u1 = csub32(csub32(csub32(u1, K.Q4), K.Q2), (uint32_t)K.Q);
            acc[0][r] = (int32_t)(u0 - K.h1);
            acc[1][r] = (int32_t)(u1 - K.h1);
        }
    }
    if (active) {
        // acc0 transposed (X -> X^-1, poly.cpp:762-770): out[(N-k) mod N] = -acc0[k]
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t k = ix1(t, r);
            const uint32_t v = (uint32_t)(acc[0][r] < 0 ? acc[0][r] + K.Q : acc[0][r]);
            const uint32_t v1 = (uint32_t)(acc[1][r] < 0 ? acc[1][r] + K.Q : acc[1][r]);
            g[(FN - k) & (FN - 1)] = k == 0 ? v : (v == 0 ? 0 : (uint32_t)K.Q - v);
            g[FN + k] = v1;
        }
    }
}

// generic (plain, N^-1-scaled) BSK and tables -> centred Montgomery copies
__global__ void k_pack_fast(uint32_t Q, const uint32_t* __restrict__ bsk, size_t words, const uint32_t* __restrict__ psi,
                            const uint32_t* __restrict__ ipsi, const uint32_t* __restrict__ mono,
                            int32_t* __restrict__ out) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto mont = [Q](uint32_t v) {
        const uint32_t m = (uint32_t)(((uint64_t)v << 32) % Q);
        return m > Q / 2 ? (int32_t)m - (int32_t)Q : (int32_t)m;
    };
    if (idx < words) out[T_WORDS + idx] = mont(bsk[idx]);
    if (idx < FN) {
        out[T_PSI + idx] = mont(psi[idx]);
        out[T_IPSI + idx] = mont(ipsi[idx]);
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
                       (const uint32_t*)T.mono, (int32_t*)bsk_fast);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_fast(const BRParams& P, const DevTables&, const void* bsk_fast, const uint64_t* a,
                                    uint64_t amod, uint64_t* acc, size_t B, hipStream_t s) {
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
    const int32_t* tabs = (const int32_t*)bsk_fast;
    const int32_t* bsk = tabs + T_WORDS;
    static const int variant = [] {
        const char* e = std::getenv("TFHE_FAST_VARIANT");
        return e ? std::atoi(e) : 0;
    }();
    auto launch = [&](auto kern, int cts) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(cts));
        hipLaunchKernelGGL(kern, dim3((unsigned)((B + cts - 1) / cts)), dim3(TPC * cts), lds_bytes(cts), s, K, P.n,
                           loga, tabs, bsk, a, acc, (uint32_t)B);
    };
    switch (variant) {
        case 1: launch(k_blind_rotate_fast<3, false, 2>, 2); break;
        case 2: launch(k_blind_rotate_fast<3, true, 1>, 1); break;
        case 3: launch(k_blind_rotate_fast<2, true, 2>, 2); break;
        case 4: launch(k_blind_rotate_fast<3, false, 1>, 1); break;
        default: launch(k_blind_rotate_fast<3, true, 2>, 2); break;
    }
    return hipGetLastError();
}

}  // namespace tfhe
