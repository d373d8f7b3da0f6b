// VALU throughput microbenchmark for gfx950: which instructions can carry
// exact modular arithmetic for the blind-rotation NTT ("modmul").
// Each kernel runs 8 independent dependency chains per lane of one instruction
// (inline asm, so the compiler cannot fold them) and reports lane-ops/s and
// cycles per wave-instruction per SIMD at the measured clock.
//
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#include "../../tfhe-gpu_amd/csrc/device_math.hpp"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int UNROLL = 16;

#define CHAINS8(STMT) STMT(a0) STMT(a1) STMT(a2) STMT(a3) STMT(a4) STMT(a5) STMT(a6) STMT(a7)

#define DEF_U32_KERNEL(NAME, ASM)                                                   \
__global__ void NAME(uint32_t* out, int iters, uint32_t seed) {                     \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;                             \
    uint32_t a0 = seed + t, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u;               \
    uint32_t a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;            \
    uint32_t c = seed | 1u;                                                         \
    for (int i = 0; i < iters; ++i) {                                               \
        _Pragma("unroll")                                                           \
        for (int u = 0; u < UNROLL; ++u) {                                          \
            _Pragma("") CHAINS8(ASM)                                                \
        }                                                                           \
    }                                                                               \
    out[t] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                 \
}

#define S_MUL_LO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_MUL_HI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_MUL24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_MULHI24(x) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_MAD24(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x) : "v"(c));
#define S_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_SUBMIN(x) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %1, 5" : "+v"(x) : "v"(c));
#define S_CVT(x) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));
#define S_BFE(x) asm volatile("v_bfe_i32 %0, %0, 0, 7" : "+v"(x));
#define S_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x) : "v"(c));
#define S_SUB(x) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_ASHR(x) asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(x));

DEF_U32_KERNEL(k_mul_lo_u32, S_MUL_LO)
DEF_U32_KERNEL(k_mul_hi_u32, S_MUL_HI)
DEF_U32_KERNEL(k_mul_u32_u24, S_MUL24)
DEF_U32_KERNEL(k_mul_hi_u32_u24, S_MULHI24)
DEF_U32_KERNEL(k_mad_u32_u24, S_MAD24)
DEF_U32_KERNEL(k_add_u32, S_ADD)
DEF_U32_KERNEL(k_min_u32, S_SUBMIN)
DEF_U32_KERNEL(k_alignbit, S_ALIGN)
DEF_U32_KERNEL(k_cvt_f32_u32, S_CVT)
DEF_U32_KERNEL(k_bfe_i32, S_BFE)
DEF_U32_KERNEL(k_add3_u32, S_ADD3)
DEF_U32_KERNEL(k_sub_u32, S_SUB)
DEF_U32_KERNEL(k_ashr_i32, S_ASHR)

#define DEF_U64_KERNEL(NAME, ASM)                                                   \
__global__ void NAME(uint64_t* out, int iters, uint32_t seed) {                     \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;                             \
    uint64_t a0 = seed + t, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u;               \
    uint64_t a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;            \
    uint32_t c = seed | 1u, d = seed ^ 0x5555u;                                     \
    for (int i = 0; i < iters; ++i) {                                               \
        _Pragma("unroll")                                                           \
        for (int u = 0; u < UNROLL; ++u) {                                          \
            CHAINS8(ASM)                                                            \
        }                                                                           \
    }                                                                               \
    out[t] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                 \
}
#define S_MAD64(x) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"(c), "v"(d) : "vcc");
#define S_LSHR64(x) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(x));
#define S_ADD64(x) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(x));
#define S_MADI64(x) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"(c), "v"(d) : "vcc");
DEF_U64_KERNEL(k_mad_u64_u32, S_MAD64)
DEF_U64_KERNEL(k_mad_i64_i32, S_MADI64)
DEF_U64_KERNEL(k_lshrrev_b64, S_LSHR64)
DEF_U64_KERNEL(k_lshl_add_u64, S_ADD64)

#define DEF_F64_KERNEL(NAME, ASM)                                                   \
__global__ void NAME(double* out, int iters, uint32_t seed) {                       \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;                             \
    double a0 = seed + t, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;                    \
    double a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                  \
    double c = 0.999999, d = 1e-7;                                                  \
    for (int i = 0; i < iters; ++i) {                                               \
        _Pragma("unroll")                                                           \
        for (int u = 0; u < UNROLL; ++u) {                                          \
            CHAINS8(ASM)                                                            \
        }                                                                           \
    }                                                                               \
    out[t] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                 \
}
#define S_FMA64(x) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(c), "v"(d));
#define S_MUL64F(x) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(c));
#define S_RND64(x) asm volatile("v_rndne_f64 %0, %0" : "+v"(x));
DEF_F64_KERNEL(k_fma_f64, S_FMA64)
DEF_F64_KERNEL(k_mul_f64, S_MUL64F)
DEF_F64_KERNEL(k_rndne_f64, S_RND64)

#define DEF_F32_KERNEL(NAME, ASM)                                                   \
__global__ void NAME(float* out, int iters, uint32_t seed) {                        \
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;                             \
    float a0 = seed + t, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;                     \
    float a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                   \
    float c = 0.999999f, d = 1e-7f;                                                 \
    for (int i = 0; i < iters; ++i) {                                               \
        _Pragma("unroll")                                                           \
        for (int u = 0; u < UNROLL; ++u) {                                          \
            CHAINS8(ASM)                                                            \
        }                                                                           \
    }                                                                               \
    out[t] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                 \
}
#define S_FMA32(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c), "v"(d));
DEF_F32_KERNEL(k_fma_f32, S_FMA32)

// Whole modmul candidates, written in plain HIP so the compiler's real code is timed.
// Q = 2^27 - 2^11 + 1 (STD128). 8 independent chains x = x*w mod Q.
__device__ __forceinline__ uint32_t shoup_mul(uint32_t a, uint32_t w, uint32_t wp, uint32_t Q) {
    uint32_t qt = __umulhi(a, wp);
    uint32_t r = a * w - qt * Q;
    return r >= Q ? r - Q : r;
}
__device__ __forceinline__ uint32_t barrett_mul(uint32_t a, uint32_t b, uint32_t Q, uint64_t mu /*floor(2^58/Q)*/) {
    uint64_t p = (uint64_t)a * b;
    uint64_t qt = ((p >> 26) * mu) >> 32;
    uint32_t r = (uint32_t)p - (uint32_t)qt * Q;
    r = r >= Q ? r - Q : r;
    return r >= Q ? r - Q : r;
}
__device__ __forceinline__ double f64_mul(double a, double b, double Q, double Qinv) {
    // centred |a|,|b| < 2^26  =>  a*b exact in binary64
    double p = a * b;
    double qt = __builtin_rint(p * Qinv);
    return __builtin_fma(-qt, Q, p);
}

__global__ void k_modmul_shoup(uint32_t* out, int iters, uint32_t seed) {
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    const uint32_t Q = 134215681u, w = 12345677u;
    const uint32_t wp = (uint32_t)(((uint64_t)w << 32) / Q);
    uint32_t x[8];
    for (int k = 0; k < 8; ++k) x[k] = (seed + t * 8 + k) % Q;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = shoup_mul(x[k], w, wp, Q);
    }
    uint32_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= x[k];
    out[t] = s;
}
// signed Montgomery (R = 2^32) as in blind_rotate_fast.hip: v_mad_i64_i32, v_mul_lo_u32, v_mad_i64_i32
__global__ void k_modmul_smont(int32_t* out, int iters, uint32_t seed) {
    int32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    const int32_t Q = 134215681, nQ = -Q, w = 12345677;
    uint32_t inv = 1;
    for (int it = 0; it < 5; ++it) inv *= 2u - (uint32_t)Q * inv;
    int32_t x[8];
    for (int k = 0; k < 8; ++k) x[k] = (int32_t)((seed + t * 8 + k) % (uint32_t)Q) - Q / 2;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int64_t T = (int64_t)x[k] * w;
                const int32_t m = (int32_t)((uint32_t)T * inv);
                x[k] = (int32_t)(((int64_t)m * nQ + T) >> 32);
            }
    }
    int32_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= x[k];
    out[t] = s;
}
__global__ void k_modmul_barrett(uint32_t* out, int iters, uint32_t seed) {
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    const uint32_t Q = 134215681u;
    const uint64_t mu = (1ull << 58) / Q;
    uint32_t x[8], y[8];
    for (int k = 0; k < 8; ++k) { x[k] = (seed + t * 8 + k) % Q; y[k] = (seed * 7 + t + k * 3) % Q; }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = barrett_mul(x[k], y[k], Q, mu);
    }
    uint32_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= x[k];
    out[t] = s;
}
__global__ void k_modmul_f64(double* out, int iters, uint32_t seed) {
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    const double Q = 134215681.0, Qinv = 1.0 / 134215681.0;
    double x[8], y[8];
    for (int k = 0; k < 8; ++k) { x[k] = (double)((seed + t * 8 + k) % 134215681u) - 67107840.0;
                                  y[k] = (double)((seed * 7 + t + k * 3) % 134215681u) - 67107840.0; }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = f64_mul(x[k], y[k], Q, Qinv);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += x[k];
    out[t] = s;
}

// The products the N = 2048 kernels actually issue, from the kernels' own header (device_math.hpp):
// fmodmul_f64 (blind_rotate_f64.hip: 6 FP64 instructions) at STD192's Q = 2^37 - 2^17 + 1 and
// STD128Q's Q = 2^50 - 2^14 + 1 with full-width centred operands, and sf_mul (the sf kernels of
// blind_rotate_generic.hip: five v_mad_u64_u32 + four more VALU) at Q = 2^54 - 77823 with lazy operands.
// Each lane runs 8 independent chains x = x * w mod Q, w a per-chain constant (a key / twiddle).
template <uint64_t QV>
__global__ void k_modmul_fmod(double* out, int iters, uint32_t seed) {
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    const double Q = (double)QV, Qinv = 1.0 / Q, half = (double)(QV >> 1);
    double x[8], w[8];
    for (int k = 0; k < 8; ++k) {
        const uint64_t h = (uint64_t)(seed + t * 8 + k) * 0x9E3779B97F4A7C15ull;
        x[k] = (double)(int64_t)((h >> 7) % QV) - half;
        w[k] = (double)(int64_t)(((h * 0xBF58476D1CE4E5B9ull) >> 9) % QV) - half;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = tfhe::fmodmul_f64(x[k], w[k], Q, Qinv);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += x[k];
    out[t] = s;
}
__global__ void k_modmul_sf54(uint64_t* out, int iters, uint32_t seed) {
    uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
    constexpr uint64_t Q = (1ull << 54) - 77823;
    constexpr uint32_t c = 77823;
    uint64_t x[8], w0[8], w1[8];
    for (int k = 0; k < 8; ++k) {
        const uint64_t h = (uint64_t)(seed + t * 8 + k) * 0x9E3779B97F4A7C15ull;
        x[k] = (h >> 3) % Q;
        w0[k] = ((h * 0xBF58476D1CE4E5B9ull) >> 9) % Q;
        // W1 = w 2^32 mod Q, the form k_pack_sf stores
        const uint64_t y = ((w0[k] & ((1ull << 22) - 1)) << 32) + (w0[k] >> 22) * c;
        w1[k] = y >= Q ? y - Q : y;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = tfhe::sf_mul(x[k], w0[k], w1[k], 2 * c);
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; ++k) s ^= x[k];
    out[t] = s;
}

template <typename T, typename K>
static void run(const char* name, K kern, int ops_per_iter_lane, double peak_lane_ops) {
    const int blocks = 256 * 8, threads = 256, iters = 2000;
    T* out;
    CHK(hipMalloc(&out, sizeof(T) * blocks * threads));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 10, 7u);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    double lane_ops = (double)blocks * threads * iters * ops_per_iter_lane;
    double rate = lane_ops / (ms * 1e-3);
    printf("%-22s %9.3f ms  %10.3f Glane-ops/s  %6.3f of fp32-fma lane rate\n", name, ms, rate * 1e-9,
           rate / peak_lane_ops);
    CHK(hipFree(out));
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    printf("device %s CUs=%d clock=%d kHz\n", p.name, p.multiProcessorCount, p.clockRate);
    // fp32 FMA lane rate at max clock: CUs * 4 SIMD * 32 lanes * clock
    double peak = (double)p.multiProcessorCount * 128.0 * p.clockRate * 1e3;
    const int ops = UNROLL * 8;
    run<float>("v_fma_f32", k_fma_f32, ops, peak);
    run<uint32_t>("v_add_u32", k_add_u32, ops, peak);
    run<uint32_t>("v_min_u32", k_min_u32, ops, peak);
    run<uint32_t>("v_alignbit_b32", k_alignbit, ops, peak);
    run<uint32_t>("v_cvt_f32_u32", k_cvt_f32_u32, ops, peak);
    run<uint32_t>("v_mul_u32_u24", k_mul_u32_u24, ops, peak);
    run<uint32_t>("v_mul_hi_u32_u24", k_mul_hi_u32_u24, ops, peak);
    run<uint32_t>("v_mad_u32_u24", k_mad_u32_u24, ops, peak);
    run<uint32_t>("v_mul_lo_u32", k_mul_lo_u32, ops, peak);
    run<uint32_t>("v_mul_hi_u32", k_mul_hi_u32, ops, peak);
    run<uint64_t>("v_mad_u64_u32", k_mad_u64_u32, ops, peak);
    run<uint64_t>("v_mad_i64_i32", k_mad_i64_i32, ops, peak);
    run<uint32_t>("v_bfe_i32", k_bfe_i32, ops, peak);
    run<uint32_t>("v_add3_u32", k_add3_u32, ops, peak);
    run<uint32_t>("v_sub_u32", k_sub_u32, ops, peak);
    run<uint32_t>("v_ashrrev_i32", k_ashr_i32, ops, peak);
    run<uint64_t>("v_lshrrev_b64", k_lshrrev_b64, ops, peak);
    run<uint64_t>("v_lshl_add_u64", k_lshl_add_u64, ops, peak);
    run<double>("v_fma_f64", k_fma_f64, ops, peak);
    run<double>("v_mul_f64", k_mul_f64, ops, peak);
    run<double>("v_rndne_f64", k_rndne_f64, ops, peak);
    // whole modmuls: rate reported as modmul/s (lane), fraction vs fp32 lane rate = 1/slots
    run<uint32_t>("modmul_shoup_u32", k_modmul_shoup, ops, peak);
    run<uint32_t>("modmul_barrett_u32", k_modmul_barrett, ops, peak);
    run<int32_t>("modmul_smont_i32", k_modmul_smont, ops, peak);
    run<double>("modmul_f64_centred", k_modmul_f64, ops, peak);
    run<double>("modmul_fmod_q37", k_modmul_fmod<(1ull << 37) - (1ull << 17) + 1>, ops, peak);
    run<double>("modmul_fmod_q50", k_modmul_fmod<(1ull << 50) - (1ull << 14) + 1>, ops, peak);
    run<uint64_t>("modmul_sf_q54", k_modmul_sf54, ops, peak);
    return 0;
}
