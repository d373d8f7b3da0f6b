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
// MKM.  One wavefront per ciphertext, four per workgroup.
// Phase 1: the wavefront rounds its extract's N+1 words to qKS (RoundqQ) and keeps
//          the base-baseKS digits of a'_i in LDS (u8: every baseKS <= 256).
// Phase 2: for each of the N*dKS gathered rows every lane loads 16 bytes of the
//          row (VEC columns of the packed, 16-byte-padded KSK A part) and adds
//          them into exact per-column sums; the B column lives in its own array
//          and is accumulated wave-uniformly.  One reduction, then RoundqQ to fmod.
// The u32/u64 rows of the larger sets span 5 to 11 chunks of 64*VEC columns.  Below ~4096
// ciphertexts one wave per ciphertext sweeping them in turn leaves the gather
// latency-bound (C5a, 1024 per launch: 19 ms of key switch next to 44 ms of blind rotation),
// so up to ceil(4096 / B) waves share a ciphertext's chunks; at 4096+ more waves per
// ciphertext only widen the per-coefficient row set past L2 (measured: C3 -15 %, C4 -3.5 %).
// The gather is L2/MALL-bandwidth bound: STD128 reads N*dKS rows x 1 KiB per
// ciphertext (SURVEY.md 8(d) "KS gather", 2 MiB u16).
// ---------------------------------------------------------------------------
constexpr int MKM_WAVES = 4;

template <typename KW> struct MkmAcc { using T = uint64_t; };
template <> struct MkmAcc<uint16_t> { using T = uint32_t; };  // N*dKS*2^16 < 2^32

template <typename KW, int WAVES = MKM_WAVES>
__global__ void __launch_bounds__(64 * WAVES)
k_mkm(KSParams P, const KW* __restrict__ kska, const KW* __restrict__ kskb, const uint64_t* __restrict__ ext,
      uint64_t fmod, uint64_t* __restrict__ out, size_t B, uint32_t split) {
    constexpr uint32_t VEC = 16 / sizeof(KW);
    using Acc = typename MkmAcc<KW>::T;
    extern __shared__ __align__(16) unsigned char smem[];
    const uint32_t N = P.N, n = P.n, dks = P.dKS, bks = P.baseKS, npad = P.n_pad;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // `split` wavefronts per ciphertext; wave s sweeps the column chunks s, s + split, ...
    // (chunk = 64 * VEC columns)
    const uint32_t chunks = (npad + 64 * VEC - 1) / (64 * VEC);
    const size_t item = (size_t)blockIdx.x * WAVES + w;
    const size_t ct = item / split;
    const uint32_t first = (uint32_t)(item - ct * split);
    if (ct >= B) return;  // whole wavefront; no workgroup barrier below
    uint8_t* dig = smem + (size_t)w * N * dks;
    const uint64_t* e = ext + ct * (N + 1);

    uint64_t bq = 0;
    for (uint32_t i = lane; i <= N; i += 64) {
        uint64_t x = round_qQ(e[i], P.qKS, P.Q);
        if (i == N) {
            bq = x;
        } else {
            for (uint32_t j = 0; j < dks; ++j, x /= bks) dig[(size_t)i * dks + j] = (uint8_t)(x % bks);
        }
    }
    bq = __shfl(bq, (int)(N & 63));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

    const uint64_t qks = P.qKS;
    uint64_t* o = out + ct * (size_t)(n + 1);
    uint64_t bsum = 0;
    for (uint32_t chunk = first; chunk < chunks; chunk += split) {
        const uint32_t c0 = chunk * 64 * VEC;
        const uint32_t col = c0 + lane * VEC;
        const bool on = col < npad;
        Acc acc[VEC];
#pragma unroll
        for (uint32_t v = 0; v < VEC; ++v) acc[v] = 0;
        const KW* base = kska + (on ? col : 0);
#pragma unroll 4
        for (uint32_t i = 0; i < N; ++i) {
            for (uint32_t j = 0; j < dks; ++j) {
                const uint32_t a0 = dig[(size_t)i * dks + j];
                const size_t row = ((size_t)i * bks + a0) * dks + j;
                if (on) {
                    const uint4 u = *reinterpret_cast<const uint4*>(base + row * npad);
                    const KW* vals = reinterpret_cast<const KW*>(&u);
#pragma unroll
                    for (uint32_t v = 0; v < VEC; ++v) acc[v] += (Acc)vals[v];
                }
                if (chunk == 0) bsum += (uint64_t)kskb[row];
            }
        }
#pragma unroll
        for (uint32_t v = 0; v < VEC; ++v) {
            const uint32_t k = col + v;
            if (on && k < n) {
                const uint64_t r = (uint64_t)acc[v] % qks;
                o[k] = round_qQ(r == 0 ? 0 : qks - r, fmod, qks);  // 0 - sum
            }
        }
    }
    if (first == 0 && lane == 0) {
        const uint64_t r = bsum % qks;
        o[n] = round_qQ(bq >= r ? bq - r : bq + (qks - r), fmod, qks);  // b - sum
    }
}

hipError_t launch_mkm(const KSParams& P, int ksk_bits, const void* kska, const void* kskb, const uint64_t* ext,
                      uint64_t fmod, uint64_t* out, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    if (P.baseKS > 256) return hipErrorNotSupported;
    // u16 keys sum in 32 bits: exact while N dKS (qKS - 1) < 2^32; past that the wrap mod 2^32 is
    // harmless only when qKS divides 2^32
    if (ksk_bits == 16 && (unsigned __int128)P.N * P.dKS * (P.qKS - 1) >= ((unsigned __int128)1 << 32) &&
        (P.qKS & (P.qKS - 1)) != 0)
        return hipErrorNotSupported;
    // one wavefront per workgroup when four digit arrays (N dKS bytes each) exceed the LDS: N = 8192
    const bool one = (size_t)MKM_WAVES * P.N * P.dKS > 160 * 1024;
    const int waves = one ? 1 : MKM_WAVES;
    const size_t lds = (size_t)waves * P.N * P.dKS;
    if (lds > 160 * 1024) return hipErrorNotSupported;
    // enough wavefronts for the gather's latency (~4096), but no more: every extra wave per
    // ciphertext widens the rows in flight per coefficient past what the L2 holds
    const size_t vec = 16 / (ksk_bits / 8), chunks = (P.n_pad + 64 * vec - 1) / (64 * vec);
    const uint32_t split = (uint32_t)std::max<size_t>(1, std::min(chunks, (4096 + B - 1) / B));
    dim3 grid((unsigned)((B * split + waves - 1) / waves)), block(64 * waves);
    auto go = [&](auto kern, auto tag) {
        using KW = decltype(tag);
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, grid, block, lds, s, P, (const KW*)kska, (const KW*)kskb, ext, fmod, out, B, split);
    };
    // one wavefront per workgroup: only the N = 8192 contexts need it, and their keys are u64 (qKS = 2^35)
    if (one && ksk_bits != 64) return hipErrorNotSupported;
    switch (ksk_bits) {
        case 16: go(k_mkm<uint16_t>, uint16_t{}); break;
        case 32: go(k_mkm<uint32_t>, uint32_t{}); break;
        default: one ? go(k_mkm<uint64_t, 1>, uint64_t{}) : go(k_mkm<uint64_t>, uint64_t{}); break;
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

// Sparse test vectors of the drop-in path (tfhe_eval_acc_tv): tv[B][tvlen] -> acc[B][2][N] with
// acc0 = 0 and acc1[j * factor] = tv[j] (the accumulators BootstrapGateCore / BootstrapFuncCore
// build, binfhe-base-scheme.cpp:1110-1138, 1163-1185), every other coefficient 0.
__global__ void k_expand_tv(uint32_t N, uint32_t tvlen, uint32_t factor, const uint64_t* __restrict__ tv,
                            uint64_t* __restrict__ acc) {
    const uint64_t* t = tv + (size_t)blockIdx.x * tvlen;
    uint64_t* g = acc + (size_t)blockIdx.x * 2 * N;
    for (uint32_t x = threadIdx.x; x < N; x += blockDim.x) {
        g[x] = 0;
        g[N + x] = x % factor == 0 ? t[x / factor] : 0;
    }
}

hipError_t launch_expand_tv(uint32_t N, uint32_t tvlen, const uint64_t* tv, uint64_t* acc, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    if (tvlen == 0 || N % tvlen != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_expand_tv, dim3((unsigned)B), dim3(256), 0, s, N, tvlen, N / tvlen, tv, acc);
    return hipGetLastError();
}

// Narrow PCIe wire format of the host-array runner: u64 words <-> u16 / u32 (engine.hip)
template <typename W>
__global__ void k_widen(const W* __restrict__ src, uint64_t* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
template <typename W>
__global__ void k_narrow(const uint64_t* __restrict__ src, W* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = (W)src[i];
}
hipError_t launch_widen(const void* src, int wb, uint64_t* dst, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
    if (wb == 2) hipLaunchKernelGGL(k_widen<uint16_t>, dim3(g), dim3(256), 0, s, (const uint16_t*)src, dst, n);
    else if (wb == 4) hipLaunchKernelGGL(k_widen<uint32_t>, dim3(g), dim3(256), 0, s, (const uint32_t*)src, dst, n);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_narrow(const uint64_t* src, int wb, void* dst, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
    if (wb == 2) hipLaunchKernelGGL(k_narrow<uint16_t>, dim3(g), dim3(256), 0, s, src, (uint16_t*)dst, n);
    else if (wb == 4) hipLaunchKernelGGL(k_narrow<uint32_t>, dim3(g), dim3(256), 0, s, src, (uint32_t*)dst, n);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

// Arena checksum (engine.hip replicate_arena: every replica must equal device 0's image).  Each block
// sums a position-mixed hash of its strided words into partial[blockIdx.x]; the host adds the partials.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void __launch_bounds__(256) k_checksum(const uint64_t* __restrict__ p, size_t words,
                                                  uint64_t* __restrict__ partial) {
    __shared__ uint64_t red[256];
    uint64_t h = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x)
        h += mix64(p[i] ^ (i * 0x9E3779B97F4A7C15ull));
    red[threadIdx.x] = h;
    __syncthreads();
    for (uint32_t w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}
hipError_t launch_checksum(const void* p, size_t bytes, uint64_t* partial, hipStream_t s) {
    hipLaunchKernelGGL(k_checksum, dim3(kChecksumBlocks), dim3(256), 0, s, (const uint64_t*)p, bytes / 8, partial);
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
// fmod (lwe-operation.cu:106-111), exact only while |sums| < 2^53 and non-negative;
// here every operand is first reduced into [0, modulus) (signed matrix entries by
// their mathematical residue), then the sum is exact: unreduced u128 accumulation
// when K (modulus-1)^2 < 2^128, else a modular add per term.
// ---------------------------------------------------------------------------
__global__ void k_reduce_signed(int64_t* __restrict__ v, size_t count, uint64_t modulus) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    __int128 r = (__int128)v[i] % (__int128)modulus;
    if (r < 0) r += modulus;
    reinterpret_cast<uint64_t*>(v)[i] = (uint64_t)r;
}

__global__ void k_reduce_unsigned(uint64_t* __restrict__ v, size_t count, uint64_t modulus) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    v[i] %= modulus;
}

template <bool PER_TERM>
__global__ void k_ct_mul_matrix(uint32_t width, size_t K, const uint64_t* __restrict__ ct, size_t cols,
                                const uint64_t* __restrict__ mat, uint64_t modulus, uint64_t* __restrict__ out) {
    const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t c = blockIdx.y;
    if (w >= width) return;
    unsigned __int128 acc = 0;
    for (size_t k = 0; k < K; ++k) {
        const unsigned __int128 t = (unsigned __int128)mat[k * cols + c] * ct[k * width + w];
        if (PER_TERM) {
            acc += t % modulus;  // acc < modulus before, so no overflow
            if (acc >= modulus) acc -= modulus;
        } else {
            acc += t;
        }
    }
    out[c * width + w] = (uint64_t)(acc % modulus);
}

hipError_t launch_ct_mul_matrix(uint32_t width, size_t K, uint64_t* ct, size_t cols, int64_t* matrix,
                                uint64_t modulus, uint64_t* out, hipStream_t s) {
    if (K == 0 || cols == 0) return hipSuccess;
    if (modulus == 0) return hipErrorInvalidValue;
    const size_t nm = K * cols, nc = K * (size_t)width;
    hipLaunchKernelGGL(k_reduce_signed, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, s, matrix, nm, modulus);
    hipLaunchKernelGGL(k_reduce_unsigned, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, ct, nc, modulus);
    const unsigned __int128 sq = (unsigned __int128)(modulus - 1) * (modulus - 1);
    const bool per_term = sq != 0 && sq > ~(unsigned __int128)0 / K;
    const uint64_t* m = reinterpret_cast<const uint64_t*>(matrix);
    if (per_term)
        hipLaunchKernelGGL(k_ct_mul_matrix<true>, dim3((width + 255) / 256, (unsigned)cols), dim3(256), 0, s, width,
                           K, ct, cols, m, modulus, out);
    else
        hipLaunchKernelGGL(k_ct_mul_matrix<false>, dim3((width + 255) / 256, (unsigned)cols), dim3(256), 0, s,
                           width, K, ct, cols, m, modulus, out);
    return hipGetLastError();
}

}  // namespace tfhe
