// lwe_kernels.hip -- everything around the blind rotation, on device:
//   * MKM: ModSwitch(Q->qKS) -> KeySwitch -> ModSwitch(qKS->fmod)
//     (reference MKMSwitchKernel bootstrapping.cu:73-118; CPU lwe-pke.cpp:204-215,299-321)
//   * test-vector construction (binfhe-base-scheme.cpp:1087-1145, 1147-1192)
//   * RLWE -> LWE extraction (binfhe-base-scheme.cpp:664-672, 1201-1205)
//   * LWE glue of the chained ops (lwe-pke.cpp:175-215, lwe-ciphertext.h:120-124)
//   * CiphertextMulMatrix (lwe-operation.cu:50-137), exact integer form
#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {

// ---------------------------------------------------------------------------
// MKM.  Workgroup = MKM_CTS ciphertexts x MKM_COLS output coordinates.
// Phase 1: every workgroup rounds its ciphertexts' N+1 words to qKS and stores
//          the base-baseKS digits of a'_i in LDS (u8: every baseKS <= 256).
// Phase 2: thread k accumulates the gathered KSK rows' column k (coalesced:
//          consecutive threads read consecutive words of one row), exact u64 sum,
//          one reduction, then RoundqQ to fmod.
// ---------------------------------------------------------------------------
constexpr int MKM_COLS = 256;
constexpr int MKM_CTS = 4;

template <typename KW>
__global__ void __launch_bounds__(MKM_COLS)
k_mkm(KSParams P, const KW* __restrict__ ksk, const uint64_t* __restrict__ ext, uint64_t fmod,
      uint64_t* __restrict__ out, size_t B) {
    extern __shared__ __align__(16) unsigned char smem[];
    const uint32_t N = P.N, n = P.n, dks = P.dKS, bks = P.baseKS, tid = threadIdx.x;
    uint8_t* dig = smem;                                          // [MKM_CTS][N][dKS]
    uint64_t* bq = reinterpret_cast<uint64_t*>(smem + ((size_t)MKM_CTS * N * dks + 15) / 16 * 16);  // [MKM_CTS]
    const size_t ct0 = (size_t)blockIdx.x * MKM_CTS;
    const uint32_t ncts = (uint32_t)min((size_t)MKM_CTS, B - ct0);

    for (uint32_t c = 0; c < ncts; ++c) {
        const uint64_t* e = ext + (ct0 + c) * (N + 1);
        for (uint32_t i = tid; i <= N; i += blockDim.x) {
            uint64_t x = round_qQ(e[i], P.qKS, P.Q);
            if (i == N) {
                bq[c] = x;
            } else {
                uint8_t* d = dig + ((size_t)c * N + i) * dks;
                for (uint32_t j = 0; j < dks; ++j, x /= bks) d[j] = (uint8_t)(x % bks);
            }
        }
    }
    __syncthreads();

    const uint32_t k = blockIdx.y * MKM_COLS + tid;
    if (k > n) return;
    const size_t row_stride = (size_t)n + 1;
    for (uint32_t c = 0; c < ncts; ++c) {
        const uint8_t* d = dig + (size_t)c * N * dks;
        uint64_t sum = 0;
#pragma unroll 4
        for (uint32_t i = 0; i < N; ++i) {
            for (uint32_t j = 0; j < dks; ++j) {
                const uint32_t a0 = d[(size_t)i * dks + j];
                sum += (uint64_t)ksk[(((size_t)i * bks + a0) * dks + j) * row_stride + k];
            }
        }
        const uint64_t qks = P.qKS;
        const uint64_t s = sum % qks;
        uint64_t v;
        if (k == n) v = bq[c] >= s ? bq[c] - s : bq[c] + (qks - s);  // b - sum
        else v = s == 0 ? 0 : qks - s;                              // 0 - sum
        out[(ct0 + c) * row_stride + k] = round_qQ(v, fmod, qks);
    }
}

hipError_t launch_mkm(const KSParams& P, int ksk_bits, const void* ksk, const uint64_t* ext, uint64_t fmod,
                      uint64_t* out, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    if (P.baseKS > 256) return hipErrorNotSupported;
    const size_t lds = ((size_t)MKM_CTS * P.N * P.dKS + 15) / 16 * 16 + MKM_CTS * sizeof(uint64_t);
    if (lds > 160 * 1024) return hipErrorNotSupported;
    dim3 grid((unsigned)((B + MKM_CTS - 1) / MKM_CTS), (unsigned)((P.n + 1 + MKM_COLS - 1) / MKM_COLS));
    dim3 block(MKM_COLS);
    switch (ksk_bits) {
        case 16: {
            auto k = k_mkm<uint16_t>;
            hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            hipLaunchKernelGGL(k, grid, block, lds, s, P, (const uint16_t*)ksk, ext, fmod, out, B);
            break;
        }
        case 32: {
            auto k = k_mkm<uint32_t>;
            hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            hipLaunchKernelGGL(k, grid, block, lds, s, P, (const uint32_t*)ksk, ext, fmod, out, B);
            break;
        }
        default: {
            auto k = k_mkm<uint64_t>;
            hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            hipLaunchKernelGGL(k, grid, block, lds, s, P, (const uint64_t*)ksk, ext, fmod, out, B);
            break;
        }
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// test vectors: acc0 = 0; acc1[j*factor] = f(b - j mod ctmod) for j < ctmod/2
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t tv_value(const TvParams& P, uint64_t x, size_t ct) {
    const uint64_t q = P.ctmod, F = P.fmod;
    switch (P.mode) {
        case TV_GATE:  // binfhe-base-scheme.cpp:1123-1129
            if (P.q1 < P.q2) return (x >= P.q1 && x < P.q2) ? P.Q - P.Q8 : P.Q8;
            return (x >= P.q2 && x < P.q1) ? P.Q8 : P.Q - P.Q8;
        case TV_HALF:  // f0 / f1, :733-738, :954-959
            return x < q / 2 ? F - q / 4 : q / 4;
        case TV_FLOOR2:  // f2, :973-980
            if (x < q / 4) return F - q / 2 - x;
            if (q / 4 <= x && x < 3 * q / 4) return x;
            return F + q / 2 - x;
        case TV_SIGN3:  // f3, :1029-1031
            return x < q / 2 ? F / 4 : F - F / 4;
        case TV_LUT:  // fLUT, :701-703
            return P.lut[ct * P.lut_stride + x];
        case TV_LUT1: {  // fLUT1, :782-787
            const uint64_t* L = P.lut + ct * P.lut_stride;
            return x < q / 2 ? L[x] : F - L[x - q / 2];
        }
        default: {  // TV_LUT2, LUT2 = LUT ++ LUT, :749-754
            const uint64_t* L = P.lut + ct * P.lut_stride;
            return x < q / 2 ? L[x % P.lut_len] : F - L[(x - q / 2) % P.lut_len];
        }
    }
}

__global__ void k_build_testvector(TvParams P, const uint64_t* __restrict__ ct, uint64_t* __restrict__ acc,
                                   uint64_t* __restrict__ a_out) {
    const size_t s = blockIdx.x;
    const uint32_t N = P.N, n = P.n;
    const uint64_t* c = ct + s * (n + 1);
    const uint64_t q = P.ctmod;
    const uint64_t b = c[n] % q;  // NativeInteger::ModSub reduces its operand
    const uint64_t factor = 2ull * N / q;
    const uint64_t scale = P.mode == TV_GATE ? 1 : P.Q / P.fmod;
    uint64_t* a0 = acc + s * 2 * N;
    uint64_t* a1 = a0 + N;
    for (uint32_t k = threadIdx.x; k < N; k += blockDim.x) {
        uint64_t v = 0;
        if (k % factor == 0) {
            const uint64_t j = k / factor;
            if (j < (q >> 1)) {
                const uint64_t x = b >= j ? b - j : b + (q - j);
                v = scale * tv_value(P, x, s);
            }
        }
        a0[k] = 0;
        a1[k] = v;
    }
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) a_out[s * n + k] = c[k];
}

hipError_t launch_build_testvector(const TvParams& P, const uint64_t* ct, uint64_t* acc, uint64_t* a_out, size_t B,
                                   hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_build_testvector, dim3((unsigned)B), dim3(256), 0, s, P, ct, acc, a_out);
    return hipGetLastError();
}

__global__ void k_extract(uint32_t N, uint64_t Q, uint64_t b_add, const uint64_t* __restrict__ acc,
                          uint64_t* __restrict__ ext) {
    const size_t s = blockIdx.x;
    const uint64_t* a0 = acc + s * 2 * N;
    uint64_t* e = ext + s * (N + 1);
    for (uint32_t k = threadIdx.x; k < N; k += blockDim.x) e[k] = a0[k];
    if (threadIdx.x == 0) {
        uint64_t b = b_add + a0[N];  // ModAddFastEq
        e[N] = b >= Q ? b - Q : b;
    }
}

hipError_t launch_extract(uint32_t N, uint64_t Q, uint64_t b_add, const uint64_t* acc, uint64_t* ext, size_t B,
                          hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_extract, dim3((unsigned)B), dim3(256), 0, s, N, Q, b_add, acc, ext);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// LWE glue, element-wise over [B][n+1]
// ---------------------------------------------------------------------------
__global__ void k_lwe_op(uint32_t op, uint32_t n, uint64_t m, uint64_t c, const uint64_t* __restrict__ x,
                         const uint64_t* __restrict__ y, uint64_t* __restrict__ out, size_t total) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const bool isb = (idx % (n + 1)) == n;
    const uint64_t v = x[idx];
    uint64_t r;
    switch (op) {
        case LWE_ADD: r = addm<uint64_t>(v, y[idx], m); break;
        case LWE_SUB: r = subm<uint64_t>(v, y[idx], m); break;
        case LWE_DOUBLE_SUB: {
            const uint64_t d = subm<uint64_t>(v, y[idx], m);
            r = addm<uint64_t>(d, d, m);
            break;
        }
        case LWE_NOT: r = isb ? subm<uint64_t>(m >> 2, v, m) : (v == 0 ? 0 : m - v); break;
        case LWE_ADD_CONST: r = isb ? addm<uint64_t>(v, c, m) : v; break;
        case LWE_SUB_CONST: r = isb ? subm<uint64_t>(v, c, m) : v; break;
        case LWE_SET_MOD: r = v % m; break;
        case LWE_MODSWITCH: r = round_qQ(v, m, c); break;
        default: r = v; break;
    }
    out[idx] = r;
}

hipError_t launch_lwe_op(uint32_t op, uint32_t n, uint64_t m, uint64_t c, const uint64_t* x, const uint64_t* y,
                         uint64_t* out, size_t B, hipStream_t s) {
    const size_t total = B * (size_t)(n + 1);
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_lwe_op, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, op, n, m, c, x, y, out,
                       total);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// CiphertextMulMatrix: the reference computes the product as an FP64 DGEMM and
// fmod (lwe-operation.cu:106-111), exact only while |sums| < 2^53; here the sum
// is exact (__int128) and reduced to [0, modulus).
// ---------------------------------------------------------------------------
__global__ void k_ct_mul_matrix(uint32_t width, size_t K, const uint64_t* __restrict__ ct, size_t cols,
                                const int64_t* __restrict__ mat, uint64_t modulus, uint64_t* __restrict__ out) {
    const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t c = blockIdx.y;
    if (w >= width) return;
    __int128 acc = 0;
    for (size_t k = 0; k < K; ++k) acc += (__int128)mat[k * cols + c] * (__int128)ct[k * width + w];
    __int128 r = acc % (__int128)modulus;
    if (r < 0) r += modulus;
    out[c * width + w] = (uint64_t)r;
}

hipError_t launch_ct_mul_matrix(uint32_t width, size_t K, const uint64_t* ct, size_t cols, const int64_t* matrix,
                                uint64_t modulus, uint64_t* out, hipStream_t s) {
    if (K == 0 || cols == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ct_mul_matrix, dim3((width + 255) / 256, (unsigned)cols), dim3(256), 0, s, width, K, ct,
                       cols, matrix, modulus, out);
    return hipGetLastError();
}

}  // namespace tfhe
