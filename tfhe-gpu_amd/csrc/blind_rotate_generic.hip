// blind_rotate_generic.hip -- LDS-resident CGGI blind rotation for any supported
// (N, Q, dG2): one 256-thread workgroup per ciphertext, polynomials in LDS,
// radix-2 transforms with workgroup barriers.  This is the path for the >32-bit
// moduli (STD192, STD128Q, logQ/arbFunc contexts) and the cross-check for the
// specialised STD128 kernel (blind_rotate_fast.hip).
//
// Math per round i (rgsw-acc-cggi.cpp:246-307, restated in the oracle):
//   dct   = SignedDigitDecompose(acc)                 rgsw-acc.cpp:57-111
//   A_kj  = sum_l NTT(dct_l) * BSK[i][k][l][j]        (BSK pre-scaled by N^-1)
//   S_j   = A_0j * NTT(X^a' - 1) + A_1j * NTT(X^-a' - 1),  NTT(X^m - 1)[x] = psi^(e_x m) - 1
//   acc_j += INTT(S_j)
// acc stays in coefficient form, so the kernel input/output is the reference's
// EvalAcc_CUDA coefficient form (acc0 transposed on exit, bootstrapping.cu:675-686).
#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {

constexpr int GEN_THREADS = 256;

template <typename W>
__device__ __forceinline__ void lds_ntt_fwd(W* buf, uint32_t polys, uint32_t N, uint32_t logN, W Q,
                                            const W* __restrict__ psi, const W* __restrict__ psi_sh) {
    const uint32_t half = N >> 1, total = polys * half;
    uint32_t len = N, loglen = logN;
    for (uint32_t m = 1; m < N; m <<= 1) {
        len >>= 1;
        --loglen;
        for (uint32_t b = threadIdx.x; b < total; b += blockDim.x) {
            const uint32_t poly = b >> (logN - 1), bb = b & (half - 1);
            const uint32_t i = bb >> loglen;
            const uint32_t j = (i << (loglen + 1)) | (bb & (len - 1));
            W* a = buf + (size_t)poly * N;
            const W U = a[j];
            const W V = shoup<W>(a[j + len], psi[m + i], psi_sh[m + i], Q);
            a[j] = addm<W>(U, V, Q);
            a[j + len] = subm<W>(U, V, Q);
        }
        __syncthreads();
    }
}

// Gentleman-Sande inverse without the N^-1 scaling (folded into the BSK)
template <typename W>
__device__ __forceinline__ void lds_ntt_inv(W* buf, uint32_t polys, uint32_t N, uint32_t logN, W Q,
                                            const W* __restrict__ ipsi, const W* __restrict__ ipsi_sh) {
    const uint32_t half = N >> 1, total = polys * half;
    uint32_t len = 1, loglen = 0;
    for (uint32_t m = N; m > 1; m >>= 1) {
        const uint32_t h = m >> 1;
        for (uint32_t b = threadIdx.x; b < total; b += blockDim.x) {
            const uint32_t poly = b >> (logN - 1), bb = b & (half - 1);
            const uint32_t i = bb >> loglen;
            const uint32_t j = (i << (loglen + 1)) | (bb & (len - 1));
            W* a = buf + (size_t)poly * N;
            const W U = a[j], V = a[j + len];
            a[j] = addm<W>(U, V, Q);
            a[j + len] = shoup<W>(subm<W>(U, V, Q), ipsi[h + i], ipsi_sh[h + i], Q);
        }
        __syncthreads();
        len <<= 1;
        ++loglen;
    }
}

template <typename W>
__global__ void __launch_bounds__(GEN_THREADS)
k_blind_rotate_generic(BRParams P, const W* __restrict__ psi, const W* __restrict__ psi_sh,
                       const W* __restrict__ ipsi, const W* __restrict__ ipsi_sh, const W* __restrict__ mono,
                       const W* __restrict__ mono_sh, const uint32_t* __restrict__ eidx, const W* __restrict__ bsk,
                       const W* __restrict__ bsk_sh, const uint64_t* __restrict__ a, uint64_t amod,
                       uint64_t* __restrict__ acc_io) {
    extern __shared__ __align__(16) unsigned char smem[];
    const uint32_t N = P.N, twoN = 2 * N, tid = threadIdx.x, T = blockDim.x;
    W* acc = reinterpret_cast<W*>(smem);  // [2][N] coefficient form
    W* buf = acc + twoN;                  // [dG2][N]
    const W Q = (W)P.Q, r1 = (W)P.r1;
    const uint64_t Qhalf = P.Q >> 1;
    const int64_t Qs = (int64_t)P.Q;
    const uint32_t sh = 64 - P.logG;
    uint64_t* g = acc_io + (size_t)blockIdx.x * twoN;
    const uint64_t* ap = a + (size_t)blockIdx.x * P.n;
    const uint64_t scale = (uint64_t)twoN / amod;
    const size_t round_words = (size_t)4 * P.dG2 * N;

    for (uint32_t k = tid; k < twoN; k += T) acc[k] = (W)g[k];
    __syncthreads();

    for (uint32_t i = 0; i < P.n; ++i) {
        // a'_i = ((amod - a_i) mod amod) * (2N / amod)   (rgsw-acc-cggi.cpp:153, bootstrapping.cu:1623)
        const uint64_t ar = ap[i] % amod;
        const uint32_t ai = (uint32_t)((ar == 0 ? 0 : amod - ar) * scale);

        // signed digit decomposition, row = poly + 2*digit (rgsw-acc.cpp:80-110)
        for (uint32_t k = tid; k < twoN; k += T) {
            const uint32_t p = k >= N, x = k - p * N;
            const uint64_t t = (uint64_t)acc[k];
            int64_t d = t < Qhalf ? (int64_t)t : (int64_t)t - Qs;
            for (uint32_t z = 0; z < P.thr; ++z) {
                const int64_t r = (int64_t)((uint64_t)d << sh) >> sh;
                d = (d - r) >> P.logG;
            }
            for (uint32_t l = 0; l < P.digits; ++l) {
                int64_t r = (int64_t)((uint64_t)d << sh) >> sh;
                d = (d - r) >> P.logG;
                if (r < 0) r += Qs;
                buf[(size_t)(p + 2 * l) * N + x] = (W)r;
            }
        }
        __syncthreads();
        lds_ntt_fwd<W>(buf, P.dG2, N, P.logN, Q, psi, psi_sh);

        // external product with the two ternary keys, times the NTT-domain monomials
        const W* ek = bsk + (size_t)i * round_words;
        const W* eks = bsk_sh + (size_t)i * round_words;
        for (uint32_t x = tid; x < N; x += T) {
            W A00 = 0, A01 = 0, A10 = 0, A11 = 0;  // A_kj, lazily reduced (< 2*dG2*Q)
            for (uint32_t l = 0; l < P.dG2; ++l) {
                const W d = buf[(size_t)l * N + x];
                const size_t o00 = ((size_t)(0 * P.dG2 + l) * 2 + 0) * N + x;
                const size_t o10 = ((size_t)(1 * P.dG2 + l) * 2 + 0) * N + x;
                A00 += shoup_lazy<W>(d, ek[o00], eks[o00], Q);
                A01 += shoup_lazy<W>(d, ek[o00 + N], eks[o00 + N], Q);
                A10 += shoup_lazy<W>(d, ek[o10], eks[o10], Q);
                A11 += shoup_lazy<W>(d, ek[o10 + N], eks[o10 + N], Q);
            }
            A00 = reduce_full<W>(A00, r1, Q);
            A01 = reduce_full<W>(A01, r1, Q);
            A10 = reduce_full<W>(A10, r1, Q);
            A11 = reduce_full<W>(A11, r1, Q);
            const uint32_t ip = (eidx[x] * ai) & (twoN - 1);
            const uint32_t in = (twoN - ip) & (twoN - 1);
            const W mp = mono[ip], mps = mono_sh[ip], mn = mono[in], mns = mono_sh[in];
            // this thread has consumed every buf[l][x]; rows 0/1 at x now hold S_0/S_1
            buf[x] = addm<W>(shoup<W>(A00, mp, mps, Q), shoup<W>(A10, mn, mns, Q), Q);
            buf[N + x] = addm<W>(shoup<W>(A01, mp, mps, Q), shoup<W>(A11, mn, mns, Q), Q);
        }
        __syncthreads();
        lds_ntt_inv<W>(buf, 2, N, P.logN, Q, ipsi, ipsi_sh);
        for (uint32_t k = tid; k < twoN; k += T) acc[k] = addm<W>(acc[k], buf[k], Q);
        __syncthreads();
    }
    // acc0 -> transpose (automorphism X -> X^-1, poly.cpp:762-770), reduced values
    for (uint32_t k = tid; k < N; k += T) {
        const W v = acc[k == 0 ? 0 : N - k];
        g[k] = (uint64_t)(k == 0 ? v : (v == 0 ? (W)0 : (W)(Q - v)));
        g[N + k] = (uint64_t)acc[N + k];
    }
}

hipError_t launch_blind_rotate_generic(int word_bits, const BRParams& P, const DevTables& T, const void* bsk,
                                       const void* bsk_sh, const uint64_t* a, uint64_t amod, uint64_t* acc, size_t B,
                                       hipStream_t s) {
    if (B == 0) return hipSuccess;
    const size_t wb = word_bits == 32 ? 4 : 8;
    const size_t lds = (size_t)(2 + P.dG2) * P.N * wb;
    if (lds > 160 * 1024) return hipErrorNotSupported;
    dim3 grid((unsigned)B), block(GEN_THREADS);
    if (word_bits == 32) {
        auto k = k_blind_rotate_generic<uint32_t>;
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, grid, block, lds, s, P, (const uint32_t*)T.psi, (const uint32_t*)T.psi_sh,
                           (const uint32_t*)T.ipsi, (const uint32_t*)T.ipsi_sh, (const uint32_t*)T.mono,
                           (const uint32_t*)T.mono_sh, T.eidx, (const uint32_t*)bsk, (const uint32_t*)bsk_sh, a, amod,
                           acc);
    } else {
        auto k = k_blind_rotate_generic<uint64_t>;
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, grid, block, lds, s, P, (const uint64_t*)T.psi, (const uint64_t*)T.psi_sh,
                           (const uint64_t*)T.ipsi, (const uint64_t*)T.ipsi_sh, (const uint64_t*)T.mono,
                           (const uint64_t*)T.mono_sh, T.eidx, (const uint64_t*)bsk, (const uint64_t*)bsk_sh, a, amod,
                           acc);
    }
    return hipGetLastError();
}

}  // namespace tfhe
