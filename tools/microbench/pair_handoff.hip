// Price of the per-round hand-off a two-workgroup ("duo") blind rotation would need: one
// ciphertext's round split over two 512-thread workgroups on two CUs, each publishing 16 KiB
// (2048 u64 coefficients, 8 per thread of one half) to its partner every round.
//
// P pairs, R rounds.  Per round every workgroup runs W iterations of dependent special-form
// products (a stand-in for the round's VALU work, device_math.hpp sf_mul), then, with EXCHANGE:
//   half the threads store 8 u64 each with sc1 (write-through) stores, every wave waits
//   vmcnt(0), workgroup barrier, lane 0 stores the round number to its flag (sc1);
//   lane 0 polls the partner's flag with sc1 loads (s_sleep between polls, bounded), barrier,
//   every thread loads the partner's 8 u64 with sc1 loads and folds them into its state.
// This is the consumer/producer form of MI355X_MICROARCH.md's hand-off table (first row).
// Pairing: blocks b and b + 8 (one XCD under round-robin dispatch) or b and b + 1 (two XCDs).
// Output: one JSON line per (pairs, W, pairing) with ms per launch without / with the exchange
// and the difference per round.  A poll that runs out counts as a timeout (reported; the
// kernel still finishes: every wave reaches the end of the round loop).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../tfhe-gpu_amd/csrc pair_handoff.hip -o pair_handoff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "../../tfhe-gpu_amd/csrc/device_math.hpp"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int TH = 512;
constexpr int N = 2048;
constexpr uint32_t kMaxPolls = 1u << 22;

__device__ __forceinline__ void sc1_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t sc1_load(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t flag_load(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// xbuf [pairs][2 members][2 parities][N] u64; flags [pairs][2] u32, one 128-B line each
template <bool EXCHANGE, bool SAME_XCD>
__global__ void __launch_bounds__(TH, 2)
k_pair(int pairs, int rounds, int work, uint64_t* __restrict__ xbuf, uint32_t* __restrict__ flags,
       uint32_t* __restrict__ timeouts, uint64_t* __restrict__ out) {
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t pair = SAME_XCD ? (b >> 4) * 8 + (b & 7) : b >> 1;
    const uint32_t x = SAME_XCD ? (b >> 3) & 1 : b & 1;
    if ((int)pair >= pairs) return;  // both members of a pair take this branch together
    __shared__ uint32_t ok;
    uint64_t s[8];
    for (int k = 0; k < 8; ++k) s[k] = (uint64_t)(pair * 977 + t * 131 + k) * 0x9E3779B97F4A7C15ull >> 11;
    const uint64_t w0 = 0x2F0C1D5A3B77ull, w1 = 0x1A2B3C4D5E6Full;
    uint32_t* myflag = flags + (pair * 2 + x) * 32;
    const uint32_t* peerflag = flags + (pair * 2 + (1 - x)) * 32;
    for (int r = 0; r < rounds; ++r) {
        for (int i = 0; i < work; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k) s[k] = tfhe::sf_mul(s[k], w0, w1, 155646u);
        if constexpr (EXCHANGE) {
            uint64_t* mine = xbuf + (((size_t)pair * 2 + x) * 2 + (r & 1)) * N;
            const uint64_t* theirs = xbuf + (((size_t)pair * 2 + (1 - x)) * 2 + (r & 1)) * N;
            if ((t >> 8) == 1 - x)
#pragma unroll
                for (int k = 0; k < 8; ++k) sc1_store(mine + (t & 255) + 256 * k, s[k]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) {
                flag_store(myflag, (uint32_t)r + 1);
                uint32_t polls = 0;
                while (flag_load(peerflag) < (uint32_t)r + 1 && ++polls < kMaxPolls) __builtin_amdgcn_s_sleep(1);
                ok = polls < kMaxPolls;
                if (!ok) atomicAdd(timeouts, 1u);
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 8; ++k) s[k] += sc1_load(theirs + (t & 255) + 256 * k) & 0xFFFF;
        }
    }
    uint64_t acc = 0;
    for (int k = 0; k < 8; ++k) acc ^= s[k];
    out[(size_t)b * TH + t] = acc;
}

template <bool EX, bool SX>
static float run(int pairs, int rounds, int work, uint64_t* xbuf, uint32_t* flags, uint32_t* to, uint64_t* out,
                 int reps) {
    const int blocks = SX ? ((pairs + 7) / 8) * 16 : pairs * 2;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < reps + 1; ++rep) {
        CHK(hipMemset(flags, 0, (size_t)pairs * 2 * 32 * 4));
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_pair<EX, SX>), dim3(blocks), dim3(TH), 0, 0, pairs, rounds, work, xbuf, flags, to, out);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;  // first launch warms up
    }
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    return best;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 1000;
    const int reps = 3;
    const int max_pairs = 256;
    uint64_t *xbuf, *out;
    uint32_t *flags, *to;
    CHK(hipMalloc(&xbuf, (size_t)max_pairs * 4 * N * 8));
    CHK(hipMalloc(&flags, (size_t)max_pairs * 2 * 32 * 4));
    CHK(hipMalloc(&to, 4));
    CHK(hipMalloc(&out, (size_t)max_pairs * 2 * 16 * TH * 8));
    CHK(hipMemset(to, 0, 4));
    const int pair_counts[] = {64, 128, 256};
    const int works[] = {0, 8, 32};
    for (int P : pair_counts)
        for (int W : works)
            for (int sx = 1; sx >= 0; --sx) {
                const float t0 = sx ? run<false, true>(P, rounds, W, xbuf, flags, to, out, reps)
                                    : run<false, false>(P, rounds, W, xbuf, flags, to, out, reps);
                const float t1 = sx ? run<true, true>(P, rounds, W, xbuf, flags, to, out, reps)
                                    : run<true, false>(P, rounds, W, xbuf, flags, to, out, reps);
                uint32_t nto = 0;
                CHK(hipMemcpy(&nto, to, 4, hipMemcpyDeviceToHost));
                printf("{\"pairs\": %d, \"workgroups\": %d, \"rounds\": %d, \"work_iters\": %d, \"pairing\": \"%s\", "
                       "\"ms_compute_only\": %.3f, \"ms_with_exchange\": %.3f, \"us_per_round_compute\": %.3f, "
                       "\"us_per_round_exchange\": %.3f, \"timeouts\": %u}\n",
                       P, 2 * P, rounds, W, sx ? "b,b+8 (one XCD)" : "b,b+1 (two XCDs)", t0, t1,
                       1000.0 * t0 / rounds, 1000.0 * (t1 - t0) / rounds, nto);
                fflush(stdout);
            }
    CHK(hipFree(xbuf));
    CHK(hipFree(flags));
    CHK(hipFree(to));
    CHK(hipFree(out));
    return 0;
}
