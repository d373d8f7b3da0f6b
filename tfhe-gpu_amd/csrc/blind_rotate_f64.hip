// blind_rotate_f64.hip -- CGGI blind rotation in exact FP64 integer arithmetic for
// 2^32 <= Q < 2^50 (STD192(_OPT), STD192Q(_OPT), STD128Q(_OPT); N = 1024 or 2048).
//
// Same math as the generic kernel (rgsw-acc-cggi.cpp:246-307, rgsw-acc.cpp:57-111), but
// every NTT-domain value is an integer held exactly in a double, so a modular product is
// six FP64 instructions instead of a ~18-instruction u64 Shoup product, and keys and
// twiddles need no Shoup companions:
//     h = a*b (rounded), l = fma(a, b, -h)          a*b = h + l exactly
//     q = rint(h / Q),   r = fma(-q, Q, h) + l      r = a*b - qQ exactly, |r| <~ Q/2
// Exactness holds while |a*b| < 2^102 and every sum stays below 2^53.  Q < 2^40 (RED =
// false): the forward transform grows by < Q/2 per stage (< 6Q after 11), the inverse
// doubles per stage from |S| < 1.1Q (< 2^51 after 11); no reduction at all.  Q < 2^50
// (RED = true, STD128Q class): every radix-4 unit reduces its outputs to |x| <~ Q/2
// (x - rint(x/Q) Q, three instructions), which keeps all values below 4Q < 2^52.
// Keys and tables are centred (|x| <= Q/2).  The accumulator stays in int64 registers
// (canonical [0, Q)) for the closed-form digit decomposition of the generic v2 kernel.
#include <cmath>
#include <cstdlib>

#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {
namespace {

constexpr int F64_THREADS = 256;

struct F64Const {
    double Q, Qinv;
    int64_t Qi;
};

__device__ __forceinline__ double fmodmul(double a, double b, const F64Const& K) {
    const double h = __dmul_rn(a, b);
    const double l = __fma_rn(a, b, -h);
    const double q = __builtin_rint(__dmul_rn(h, K.Qinv));
    return __dadd_rn(__fma_rn(-q, K.Q, h), l);
}

__device__ __forceinline__ double fred(double x, const F64Const& K) {
    return __fma_rn(-__builtin_rint(__dmul_rn(x, K.Qinv)), K.Q, x);
}

// CT stages m and 2m fused (radix-4 units); RED: reduce the unit's outputs
template <bool RED>
__device__ __forceinline__ void f64_ntt_fwd(double* buf, uint32_t N, uint32_t logN, const double* psi,
                                            const F64Const& K) {
    uint32_t m = 1, loglen = logN - 1;
    while (m < N) {
        if (m * 2 < N) {
            const uint32_t lh = loglen - 1, h = 1u << lh, units = N >> 2;
            for (uint32_t u = threadIdx.x; u < 2 * units; u += blockDim.x) {
                const uint32_t poly = u >= units, uu = u - poly * units;
                const uint32_t i = uu >> lh, jj = uu & (h - 1);
                double* a = buf + (size_t)poly * N + ((size_t)i << (loglen + 1)) + jj;
                const double w = psi[m + i], w1 = psi[2 * m + 2 * i], w2 = psi[2 * m + 2 * i + 1];
                double a0 = a[0], a1 = a[h], a2 = a[2 * h], a3 = a[3 * h];
                double v = fmodmul(a2, w, K);
                a2 = __dsub_rn(a0, v), a0 = __dadd_rn(a0, v);
                v = fmodmul(a3, w, K);
                a3 = __dsub_rn(a1, v), a1 = __dadd_rn(a1, v);
                v = fmodmul(a1, w1, K);
                a1 = __dsub_rn(a0, v), a0 = __dadd_rn(a0, v);
                v = fmodmul(a3, w2, K);
                a3 = __dsub_rn(a2, v), a2 = __dadd_rn(a2, v);
                if constexpr (RED) a0 = fred(a0, K), a1 = fred(a1, K), a2 = fred(a2, K), a3 = fred(a3, K);
                a[0] = a0, a[h] = a1, a[2 * h] = a2, a[3 * h] = a3;
            }
            m <<= 2;
            loglen -= 2;
        } else {
            const uint32_t half = N >> 1;
            for (uint32_t b = threadIdx.x; b < 2 * half; b += blockDim.x) {
                const uint32_t poly = b >= half, bb = b - poly * half;
                double* a = buf + (size_t)poly * N + 2 * bb;
                const double v = fmodmul(a[1], psi[m + bb], K), u0 = a[0];
                a[0] = RED ? fred(__dadd_rn(u0, v), K) : __dadd_rn(u0, v);
                a[1] = RED ? fred(__dsub_rn(u0, v), K) : __dsub_rn(u0, v);
            }
            m <<= 1;
        }
        __syncthreads();
    }
}

// GS inverse without N^-1 (folded into the BSK); RED: reduce the doubling outputs
template <bool RED>
__device__ __forceinline__ void f64_ntt_inv(double* buf, uint32_t N, uint32_t logN, const double* ipsi,
                                            const F64Const& K) {
    uint32_t m = N >> 1, loglen = 0;
    if (logN & 1) {
        const uint32_t half = N >> 1;
        for (uint32_t b = threadIdx.x; b < 2 * half; b += blockDim.x) {
            const uint32_t poly = b >= half, bb = b - poly * half;
            double* a = buf + (size_t)poly * N + 2 * bb;
            const double u0 = a[0], u1 = a[1];
            a[0] = RED ? fred(__dadd_rn(u0, u1), K) : __dadd_rn(u0, u1);
            a[1] = fmodmul(__dsub_rn(u0, u1), ipsi[m + bb], K);
        }
        __syncthreads();
        m >>= 1;
        loglen = 1;
    }
    while (m > 1) {
        const uint32_t lh = loglen, h = 1u << lh, units = N >> 2;
        for (uint32_t u = threadIdx.x; u < 2 * units; u += blockDim.x) {
            const uint32_t poly = u >= units, uu = u - poly * units;
            const uint32_t i = uu >> lh, jj = uu & (h - 1);
            double* a = buf + (size_t)poly * N + ((size_t)i << (lh + 2)) + jj;
            const double w1 = ipsi[m + 2 * i], w2 = ipsi[m + 2 * i + 1], w = ipsi[(m >> 1) + i];
            const double a0 = a[0], a1 = a[h], a2 = a[2 * h], a3 = a[3 * h];
            const double s0 = __dadd_rn(a0, a1), d0 = fmodmul(__dsub_rn(a0, a1), w1, K);
            const double s1 = __dadd_rn(a2, a3), d1 = fmodmul(__dsub_rn(a2, a3), w2, K);
            a[0] = RED ? fred(__dadd_rn(s0, s1), K) : __dadd_rn(s0, s1);
            a[2 * h] = fmodmul(__dsub_rn(s0, s1), w, K);
            a[h] = RED ? fred(__dadd_rn(d0, d1), K) : __dadd_rn(d0, d1);
            a[3 * h] = fmodmul(__dsub_rn(d0, d1), w, K);
        }
        __syncthreads();
        m >>= 2;
        loglen += 2;
    }
}

// exact double (|x| < 2^52, integer) -> int64
__device__ __forceinline__ int64_t d2ll(double x) {
    const double hi = floor(__dmul_rn(x, 0x1p-32));
    const double lo = __fma_rn(hi, -0x1p32, x);  // in [0, 2^32)
    return ((int64_t)(int32_t)hi << 32) + (int64_t)(uint32_t)lo;
}

// table block (doubles): psi[N] ipsi[N] mono[2N], then the BSK [n][2][dG2][2][N]
template <int CN, bool RED>
__global__ void __launch_bounds__(F64_THREADS, 2)
k_blind_rotate_f64(BRParams P, F64Const K, const double* __restrict__ tabs, const uint32_t* __restrict__ eidx,
                   const uint64_t* __restrict__ a, uint64_t amod, uint64_t* __restrict__ acc_io) {
    extern __shared__ __align__(16) double lds_d[];
    constexpr uint32_t N = F64_THREADS * CN;
    double* psi = lds_d;
    double* ipsi = lds_d + N;
    double* buf = lds_d + 2 * N;  // [2][N]
    const uint32_t t = threadIdx.x, twoN = 2 * N, logG = P.logG;
    for (uint32_t k = t; k < twoN; k += F64_THREADS) lds_d[k] = tabs[k];
    const double* mono = tabs + twoN;
    const double* bsk = tabs + 2 * twoN;
    const uint64_t Qhalf = P.Q >> 1;
    const int64_t Qs = (int64_t)P.Q, Bh = (int64_t)1 << (logG - 1);
    const uint32_t sh = 64 - logG;
    uint64_t* g = acc_io + (size_t)blockIdx.x * twoN;
    const uint64_t* ap = a + (size_t)blockIdx.x * P.n;
    const uint64_t scale = (uint64_t)twoN / amod;
    const size_t round_words = (size_t)4 * P.dG2 * N;

    int64_t acc[2][CN];  // canonical [0, Q)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < CN; ++k) {
            const uint64_t v = g[p * N + t + F64_THREADS * k];
            acc[p][k] = (int64_t)(v >= P.Q ? v % P.Q : v);
        }
    __syncthreads();

    for (uint32_t i = 0; i < P.n; ++i) {
        const uint64_t ar = ap[i] % amod;  // rgsw-acc-cggi.cpp:153
        const uint32_t ai = (uint32_t)((ar == 0 ? 0 : amod - ar) * scale);
        double A[2][2][CN];  // |A| <= dG2 Q/2 (+)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < CN; ++k) A[kk][j][k] = 0.0;
        const double* ek = bsk + (size_t)i * round_words;
        for (uint32_t l = 0; l < P.digits; ++l) {
            const uint32_t lt = l + P.thr, shift = lt * logG;
            int64_t Kd = 0;
            for (uint32_t z = 0; z < lt; ++z) Kd = (Kd << logG) + Bh;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int k = 0; k < CN; ++k) {
                    const int64_t c = (uint64_t)acc[p][k] < Qhalf ? acc[p][k] : acc[p][k] - Qs;
                    const int64_t d = (c + Kd) >> shift;
                    const int32_t r = (int32_t)((int64_t)((uint64_t)d << sh) >> sh);  // |r| <= B/2
                    buf[p * N + t + F64_THREADS * k] = (double)r;
                }
            __syncthreads();
            f64_ntt_fwd<RED>(buf, N, P.logN, psi, K);
#pragma unroll
            for (int k = 0; k < CN; ++k) {
                const uint32_t x = t + F64_THREADS * k;
                const double d0 = buf[x], d1 = buf[N + x];
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const size_t o0 = ((size_t)(kk * P.dG2 + 2 * l) * 2 + j) * N + x;
                        const size_t o1 = ((size_t)(kk * P.dG2 + 2 * l + 1) * 2 + j) * N + x;
                        A[kk][j][k] = __dadd_rn(A[kk][j][k], __dadd_rn(fmodmul(d0, ek[o0], K), fmodmul(d1, ek[o1], K)));
                    }
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < CN; ++k) {
            const uint32_t x = t + F64_THREADS * k;
            const uint32_t ip = (eidx[x] * ai) & (twoN - 1), in = (twoN - ip) & (twoN - 1);
            const double mp = mono[ip], mn = mono[in];
            buf[x] = __dadd_rn(fmodmul(A[0][0][k], mp, K), fmodmul(A[1][0][k], mn, K));
            buf[N + x] = __dadd_rn(fmodmul(A[0][1][k], mp, K), fmodmul(A[1][1][k], mn, K));
        }
        __syncthreads();
        f64_ntt_inv<RED>(buf, N, P.logN, ipsi, K);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int k = 0; k < CN; ++k) {
                const double r = buf[p * N + t + F64_THREADS * k];  // |r| < 2^52
                const double q = __builtin_rint(__dmul_rn(r, K.Qinv));
                int64_t v = acc[p][k] + d2ll(__fma_rn(-q, K.Q, r));  // in (-Q, 2Q)
                v = v < 0 ? v + Qs : v;
                acc[p][k] = v >= Qs ? v - Qs : v;
            }
        __syncthreads();
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < CN; ++k) buf[p * N + t + F64_THREADS * k] = __builtin_bit_cast(double, acc[p][k]);
    __syncthreads();
    for (uint32_t k = t; k < N; k += F64_THREADS) {  // acc0 transposed (poly.cpp:762-770)
        const uint64_t v = __builtin_bit_cast(uint64_t, buf[k == 0 ? 0 : N - k]);
        g[k] = k == 0 ? v : (v == 0 ? 0 : P.Q - v);
        g[N + k] = __builtin_bit_cast(uint64_t, buf[N + k]);
    }
}

// canonical u64 tables / BSK (generic arena) -> centred doubles
__global__ void k_pack_f64(uint64_t Q, uint32_t N, const uint64_t* __restrict__ psi, const uint64_t* __restrict__ ipsi,
                           const uint64_t* __restrict__ mono, const uint64_t* __restrict__ bsk, size_t words,
                           double* __restrict__ out) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto cen = [Q](uint64_t v) { return v > Q / 2 ? (double)(int64_t)(v - Q) : (double)v; };
    if (idx < N) out[idx] = cen(psi[idx]), out[N + idx] = cen(ipsi[idx]);
    if (idx < 2 * (size_t)N) out[2 * N + idx] = cen(mono[idx]);
    if (idx < words) out[4 * (size_t)N + idx] = cen(bsk[idx]);
}

}  // namespace

bool f64_path_supported(const BRParams& P, int word_bits) {
    return word_bits == 64 && P.Q >= (1ull << 32) && P.Q < (1ull << 50) && (P.N == 1024 || P.N == 2048) &&
           P.logG <= 32 && P.n > 0;
}

size_t bsk_f64_bytes(const BRParams& P) { return ((size_t)4 * P.N + (size_t)P.n * 4 * P.dG2 * P.N) * 8; }

hipError_t launch_pack_bsk_f64(const BRParams& P, const DevTables& T, const void* bsk, void* out, hipStream_t s) {
    const size_t words = (size_t)P.n * 4 * P.dG2 * P.N;
    hipLaunchKernelGGL(k_pack_f64, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, (uint64_t)P.Q, P.N,
                       (const uint64_t*)T.psi, (const uint64_t*)T.ipsi, (const uint64_t*)T.mono, (const uint64_t*)bsk,
                       words, (double*)out);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_f64(const BRParams& P, const DevTables& T, const void* keys, const uint64_t* a,
                                   uint64_t amod, uint64_t* acc, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    F64Const K;
    K.Q = (double)P.Q;
    K.Qinv = 1.0 / K.Q;
    K.Qi = (int64_t)P.Q;
    const size_t lds = (size_t)4 * P.N * sizeof(double);  // psi, ipsi, two polynomials
    auto go = [&](auto kern) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(F64_THREADS), lds, s, P, K, (const double*)keys, T.eidx, a,
                           amod, acc);
    };
    const bool red = P.Q >= (1ull << 40);
    if (P.N == 1024) red ? go(k_blind_rotate_f64<4, true>) : go(k_blind_rotate_f64<4, false>);
    else red ? go(k_blind_rotate_f64<8, true>) : go(k_blind_rotate_f64<8, false>);
    return hipGetLastError();
}

}  // namespace tfhe
