// blind_rotate_rns.hip -- CGGI blind rotation for the 2^50 <= Q < 2^58 contexts whose Q has the
// form 2^k - c with a small c (the logQ / arbFunc contexts of binfhecontext.cpp:51-113, Q =
// 2^54 - 77823: SURVEY 8(d) C3 and C5b), in a residue number system of four NTT primes.
//
// Math per round (rgsw-acc-cggi.cpp:246-307, the same element of Z_Q[X]/(X^N+1) as every
// other kernel): with signed digits d (rgsw-acc.cpp:57-111) and the centred integer keys k
// (|k| < Q/2), the external product and the monomial factors
//     R = sum_l d_l * k0_l * (X^a' - 1) + sum_l d_l * k1_l * (X^-a' - 1)
// are computed EXACTLY as an integer polynomial: |R| <= 4 dG2 N max|d| Q/2 < 2^94 (C3), below
// M/2 for M = p0 p1 p2 p3 ~ 2^104 (primes p = 1 mod 2N below 2^26).  Each residue ring
// Z_p[X]/(X^N+1) runs the gen3 schedule of blind_rotate_generic.hip (512 threads, radix-8
// register passes over the XOR-swizzled LDS buffer, accumulator in pass A's layout) on signed
// 32-bit Montgomery arithmetic (a product is three multiplies, as in blind_rotate_fast4.hip)
// instead of the u64 Shoup product (~16 instructions and a 64-bit companion per constant).  Two
// primes share a pass as the halves of one 64-bit LDS element (int2), so the buffer and its
// conflict-free swizzle are gen3's.  After the inverse transforms, Garner's mixed radix gives
// R = u0 + p0 (u1 + p1 (u2 + p2 u3)) with u3 centred; R mod Q follows by Horner with Q's special
// form (qt = x >> k, x - qt Q = (x mod 2^k) + qt c), and acc += R mod Q.
// Magnitudes (every int32 value < 2^31, final residues < 2p) are checked by tools/bounds_rns.py
// for this schedule and its reductions (RED_* below).
#include <cstdlib>
#include <vector>

#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {
namespace {

constexpr uint32_t RN = 2048, RTH = 512, RCN = 4;

struct RnsConst {
    int32_t p[4], np[4], qinv[4], rM[4];  // prime, -prime, prime^-1 mod 2^32, 2^32 mod prime (centred)
    int32_t g1;                           // Mont(p0^-1 mod p1)
    int32_t g2a, g2;                      // Mont(p0 mod p2), Mont((p0 p1)^-1 mod p2)
    int32_t g3a, g3b, g3;                 // Mont(p0 mod p3), Mont(p0 p1 mod p3), Mont((p0 p1 p2)^-1 mod p3)
    uint64_t Q;
    uint32_t kq, c;                       // Q = 2^kq - c
};

// table block at the head of the RNS key buffer (int2 = primes (2J, 2J+1) of pair J)
struct RnsTables {
    static constexpr size_t psi = 0;                  // int2 [2][N] forward twiddles, Montgomery, centred
    static constexpr size_t ipsi = psi + 2 * RN;      // int2 [2][N] inverse twiddles
    static constexpr size_t mono = ipsi + 2 * RN;     // int2 [2][2N] psi^k - 1
    static constexpr size_t ninv = mono + 4 * RN;     // int2 [2] Mont(N^-1 R) (key packing)
    static constexpr size_t words = ninv + 2;         // int2 elements; keys follow (16-byte aligned)
};
constexpr size_t rns_keys_off = (RnsTables::words + 1) / 2 * 2;

__device__ __forceinline__ int32_t sredc(int64_t T, int32_t qinv, int32_t np) {
    const int32_t m = (int32_t)((uint32_t)T * (uint32_t)qinv);
    return (int32_t)(((int64_t)m * np + T) >> 32);
}
template <int J>
__device__ __forceinline__ int2 smul2(int2 a, int2 w, const RnsConst& K) {
    return make_int2(sredc((int64_t)a.x * w.x, K.qinv[2 * J], K.np[2 * J]),
                     sredc((int64_t)a.y * w.y, K.qinv[2 * J + 1], K.np[2 * J + 1]));
}
template <int J>
__device__ __forceinline__ int2 red2(int2 a, const RnsConst& K) {
    return smul2<J>(a, make_int2(K.rM[2 * J], K.rM[2 * J + 1]), K);
}
__device__ __forceinline__ int2 add2(int2 a, int2 b) { return make_int2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ int2 sub2(int2 a, int2 b) { return make_int2(a.x - b.x, a.y - b.y); }

template <int J>
__device__ __forceinline__ void ct2(int2& a, int2& b, int2 w, const RnsConst& K) {
    const int2 v = smul2<J>(b, w, K);
    b = sub2(a, v);
    a = add2(a, v);
}
template <int J>
__device__ __forceinline__ void gs2(int2& a, int2& b, int2 w, const RnsConst& K) {
    const int2 d = sub2(a, b);
    a = add2(a, b);
    b = smul2<J>(d, w, K);
}

// ---- gen3 addressing (blind_rotate_generic.hip / tools/lds_layouts_f64.py) ----
__device__ __forceinline__ uint32_t rswz(uint32_t x) {
    const uint32_t c = (x >> 5) & 7;
    return x ^ (c << 2) ^ (c & 3);
}
__device__ __forceinline__ uint32_t rswzf(uint32_t c) { return (c << 2) ^ (c & 3); }
__device__ __forceinline__ void r_ad(int pass, uint32_t tau, uint32_t (&ad)[8]) {
    if (pass == 0) {
        const uint32_t a0 = rswz(tau);
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) ad[k] = a0 + 256 * k;
    } else if (pass == 1) {
        const uint32_t b0 = ((tau >> 5) << 8) + (tau & 31);
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) ad[k] = (b0 ^ rswzf(k)) + 32 * k;
    } else {
        const uint32_t c0 = rswz(((tau >> 2) << 5) + (tau & 3));
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) ad[k] = c0 ^ (4 * k);
    }
}
__device__ __forceinline__ uint32_t r_tau() {
    uint32_t tau = threadIdx.x & 255;
    asm volatile("" : "+v"(tau));  // keep the passes' addresses out of the round loop
    return tau;
}

// forward CT stages s0 .. s0+2 (m0 = 2^s0) on 8 elements; g = block
template <int J>
__device__ __forceinline__ void r_fwd_core(int2 (&v)[8], uint32_t m0, uint32_t g, const int2* T, const RnsConst& K) {
#pragma unroll
    for (int k = 0; k < 4; ++k) ct2<J>(v[k], v[k + 4], T[m0 + g], K);
    ct2<J>(v[0], v[2], T[2 * m0 + 2 * g], K), ct2<J>(v[1], v[3], T[2 * m0 + 2 * g], K);
    ct2<J>(v[4], v[6], T[2 * m0 + 2 * g + 1], K), ct2<J>(v[5], v[7], T[2 * m0 + 2 * g + 1], K);
#pragma unroll
    for (int j = 0; j < 4; ++j) ct2<J>(v[2 * j], v[2 * j + 1], T[4 * m0 + 4 * g + j], K);
}
// inverse GS stages h0, 2h0, 4h0 on 8 elements; g = block, m = N / (2 h0).  v[0] is the pure sum
// (8x growth): RED_PASS reduces it (tools/bounds_rns.py)
template <int J>
__device__ __forceinline__ void r_inv_core(int2 (&v)[8], uint32_t m, uint32_t g, const int2* T, const RnsConst& K) {
#pragma unroll
    for (int j = 0; j < 4; ++j) gs2<J>(v[2 * j], v[2 * j + 1], T[m + 4 * g + j], K);
    gs2<J>(v[0], v[2], T[(m >> 1) + 2 * g], K), gs2<J>(v[1], v[3], T[(m >> 1) + 2 * g], K);
    gs2<J>(v[4], v[6], T[(m >> 1) + 2 * g + 1], K), gs2<J>(v[5], v[7], T[(m >> 1) + 2 * g + 1], K);
#pragma unroll
    for (int k = 0; k < 4; ++k) gs2<J>(v[k], v[k + 4], T[(m >> 2) + g], K);
}

// forward transform of polynomial t >> 8; v = its pass-A elements (registers), outputs in LDS
template <int J>
__device__ __forceinline__ void r_ntt_fwd(int2* buf, int2 (&v)[8], const int2* T, const RnsConst& K) {
    const uint32_t tau = r_tau();
    int2* p = buf + (threadIdx.x >> 8) * RN;
    {
        uint32_t ad[8];
        r_ad(0, tau, ad);
        r_fwd_core<J>(v, 1, 0, T, K);
#pragma unroll
        for (int k = 0; k < 8; ++k) p[ad[k]] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int pass = 1; pass <= 2; ++pass) {
        uint32_t ad[8];
        r_ad(pass, tau, ad);
        int2 w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = p[ad[k]];
        if (pass == 1) r_fwd_core<J>(w, 8, tau >> 5, T, K);
        else r_fwd_core<J>(w, 64, tau >> 2, T, K);
#pragma unroll
        for (int k = 0; k < 8; ++k) p[ad[k]] = w[k];
        __syncthreads();
    }
#pragma unroll
    for (uint32_t r = 0; r < 2; ++r) {  // stages 9 (h = 2) and 10 (h = 1) on units 4u .. 4u+3
        const uint32_t u = tau + 256 * r, u0 = rswz(4 * u);
        int2 v0 = p[u0], v1 = p[u0 ^ 1], v2 = p[u0 ^ 2], v3 = p[u0 ^ 3];
        ct2<J>(v0, v2, T[RN / 4 + u], K), ct2<J>(v1, v3, T[RN / 4 + u], K);
        ct2<J>(v0, v1, T[RN / 2 + 2 * u], K), ct2<J>(v2, v3, T[RN / 2 + 2 * u + 1], K);
        p[u0] = v0, p[u0 ^ 1] = v1, p[u0 ^ 2] = v2, p[u0 ^ 3] = v3;
    }
    __syncthreads();
}

// inverse transform of polynomial t >> 8 from LDS; v = its pass-A outputs (registers), each
// |v| < 2p (no trailing barrier: the last pass only read this thread's own entries)
template <int J>
__device__ __forceinline__ void r_ntt_inv(int2* buf, int2 (&v)[8], const int2* __restrict__ T, const RnsConst& K) {
    const uint32_t tau = r_tau();
    int2* p = buf + (threadIdx.x >> 8) * RN;
#pragma unroll
    for (uint32_t r = 0; r < 2; ++r) {  // h = 1 then h = 2 on units 4u .. 4u+3; RED_UNITS = {0}
        const uint32_t u = tau + 256 * r, u0 = rswz(4 * u);
        int2 v0 = p[u0], v1 = p[u0 ^ 1], v2 = p[u0 ^ 2], v3 = p[u0 ^ 3];
        gs2<J>(v0, v1, T[RN / 2 + 2 * u], K), gs2<J>(v2, v3, T[RN / 2 + 2 * u + 1], K);
        gs2<J>(v0, v2, T[RN / 4 + u], K), gs2<J>(v1, v3, T[RN / 4 + u], K);
        p[u0] = red2<J>(v0, K), p[u0 ^ 1] = v1, p[u0 ^ 2] = v2, p[u0 ^ 3] = v3;
    }
    __syncthreads();
#pragma unroll
    for (int pass = 2; pass >= 1; --pass) {  // RED_PASS = {0}
        uint32_t ad[8];
        r_ad(pass, tau, ad);
        int2 w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = p[ad[k]];
        if (pass == 2) r_inv_core<J>(w, 256, tau >> 2, T, K);
        else r_inv_core<J>(w, 32, tau >> 5, T, K);
        w[0] = red2<J>(w[0], K);
#pragma unroll
        for (int k = 0; k < 8; ++k) p[ad[k]] = w[k];
        __syncthreads();
    }
    uint32_t ad[8];
    r_ad(0, tau, ad);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p[ad[k]];
    r_inv_core<J>(v, 4, 0, T, K);
    v[0] = red2<J>(v[0], K), v[1] = red2<J>(v[1], K);  // RED_FINAL = {0, 1}: every output < 2p
}

// x in (-2p, 2p) -> [0, p)
__device__ __forceinline__ int32_t canon2p(int32_t x, int32_t p) {
    uint32_t t = (uint32_t)(x + 2 * p);
    t = min(t, t - 2 * (uint32_t)p);
    return (int32_t)min(t, t - (uint32_t)p);
}
// x in (-p, p) -> [0, p)
__device__ __forceinline__ int32_t canon1p(int32_t x, int32_t p) { return x + ((x >> 31) & p); }
__device__ __forceinline__ int32_t smul1(int32_t a, int32_t w, const RnsConst& K, int i) {
    return sredc((int64_t)a * w, K.qinv[i], K.np[i]);
}
// a value = P z (mod Q) below 2^kq + 2^(104 - kq), for P < 2^26, z < 2^58 and Q = 2^kq - c (c < 2^20):
// with x = P z = qt 2^kq + (x mod 2^kq) and 2^kq = c (mod Q), x = (x mod 2^kq) + qt c (mod Q)
__device__ __forceinline__ uint64_t mulc(uint64_t z, uint32_t P, const RnsConst& K) {
    const uint64_t X = (uint64_t)P * (uint32_t)z;                       // < 2^58
    const uint64_t Y = (uint64_t)P * (uint32_t)(z >> 32) + (X >> 32);   // product >> 32, < 2^52
    const uint64_t qt = Y >> (K.kq - 32);                               // < 2^(84 - kq)
    const uint64_t lo = ((Y & ((1ull << (K.kq - 32)) - 1)) << 32) | (uint32_t)X;
    return lo + qt * K.c;                                               // < 2^kq + 2^(104 - kq)
}

// one pair of primes for the round: digits -> forward transforms (digit l into buf + 2lN) ->
// products -> monomials -> inverse transform; R = the pair's residues of the round's increment
// in pass A's layout.  The products of slot x sum all DIG digits' rows in int64, so no partial
// sums stay live across a transform (DIG = 2 keeps both digits' transforms in LDS instead).
template <int J, int DIG>
__device__ __forceinline__ void r_pair(const BRParams& P, const RnsConst& K, int2* buf, const int2* psi,
                                       const int2* __restrict__ ipsi, const int2* __restrict__ mono,
                                       const uint32_t (&ex)[RCN], const int2* __restrict__ keys, uint32_t i,
                                       uint32_t ai, const uint64_t (&acc)[2][RCN], int2 (&R)[8]) {
    constexpr uint32_t N = RN, TH = RTH, CN = RCN;
    const uint32_t t = threadIdx.x, ts = rswz(t), twoN = 2 * N;
    const uint64_t Qhalf = P.Q >> 1;
    const int64_t Qs = (int64_t)P.Q, Bh = (int64_t)1 << (P.logG - 1);
    const uint32_t sh = 64 - P.logG;
    const size_t rowN = (size_t)2 * N;  // int2 elements per key row (both pairs)
    const int2* ek = keys + (size_t)i * 4 * P.dG2 * rowN + (size_t)J * N;
#pragma unroll
    for (uint32_t l = 0; l < DIG; ++l) {
        const uint32_t lt = l + P.thr, shift = lt * P.logG;
        int64_t Kd = 0;
        for (uint32_t z = 0; z < lt; ++z) Kd = (Kd << P.logG) + Bh;
        int2 v[8];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int k = 0; k < CN; ++k) {
                const uint64_t x = acc[p][k];
                const int64_t c = x < Qhalf ? (int64_t)x : (int64_t)x - Qs;
                const int64_t d = (c + Kd) >> shift;
                const int32_t r = (int32_t)((int64_t)((uint64_t)d << sh) >> sh);  // |r| <= 2^(logG-1)
                v[p * CN + k] = make_int2(r, r);
            }
        r_ntt_fwd<J>(buf + l * twoN, v, psi, K);  // pass A writes this thread's own entries: no barrier before
    }
    // group g = (slot k, key kk, column j): rows (digit l, polynomial p) = 2l + p, 2 DIG key words;
    // the next group's words are loaded before this group's arithmetic
    constexpr int NG = CN * 4, GW = 2 * DIG;
    auto kload = [&](int g, int2 (&kv)[GW]) {
        const uint32_t x = t + TH * (g >> 2), kk = (g >> 1) & 1, j = g & 1;
#pragma unroll
        for (int r = 0; r < GW; ++r) kv[r] = ek[((size_t)(kk * P.dG2 + r) * 2 + j) * rowN + x];
    };
    int2 kv[2][GW];
    int2 A[2][2];  // A_kj of the current slot
    kload(0, kv[0]);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (g + 1 < NG) kload(g + 1, kv[(g + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const int k = g >> 2, kk = (g >> 1) & 1, j = g & 1;
        int64_t sx = 0, sy = 0;
#pragma unroll
        for (int r = 0; r < GW; ++r) {
            const int2 d = buf[(r >> 1) * twoN + (r & 1) * N + ts + TH * k];
            sx += (int64_t)d.x * kv[g & 1][r].x;
            sy += (int64_t)d.y * kv[g & 1][r].y;
        }
        A[kk][j] = make_int2(sredc(sx, K.qinv[2 * J], K.np[2 * J]), sredc(sy, K.qinv[2 * J + 1], K.np[2 * J + 1]));
        if (kk == 1 && j == 1) {
            // S_j = A_0j NTT(X^a' - 1) + A_1j NTT(X^-a' - 1) at slot x; this thread has consumed
            // every digit's entries of x; digit 0's now hold S_0 / S_1
            const uint32_t ip = (ex[k] * ai) & (twoN - 1), in = (twoN - ip) & (twoN - 1);
            const int2 mp = mono[ip], mn = mono[in];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const int2 a0 = A[0][jj], a1 = A[1][jj];
                buf[jj * N + ts + TH * k] =
                    make_int2(sredc((int64_t)a0.x * mp.x + (int64_t)a1.x * mn.x, K.qinv[2 * J], K.np[2 * J]),
                              sredc((int64_t)a0.y * mp.y + (int64_t)a1.y * mn.y, K.qinv[2 * J + 1], K.np[2 * J + 1]));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // the inverse reads entries other threads wrote
    r_ntt_inv<J>(buf, R, ipsi, K);
}

template <int DIG>
__global__ void __launch_bounds__(RTH, 4)
k_blind_rotate_rns(BRParams P, RnsConst K, const int2* __restrict__ rns,
                   const uint64_t* __restrict__ a, uint64_t amod, uint64_t* __restrict__ acc_io) {
    extern __shared__ __align__(16) int2 lds_r[];
    constexpr uint32_t N = RN, TH = RTH, CN = RCN;
    int2* buf = lds_r;  // [DIG][2][N], swizzled
    const uint32_t t = threadIdx.x, twoN = 2 * N;
    // forward twiddles [2 pairs][N]: in LDS beside one digit's buffer (64 KiB per workgroup), from
    // memory when two digits' buffers take the 64 KiB
    const int2* psiT = rns + RnsTables::psi;
    if constexpr (DIG == 1) {
        int2* psiL = lds_r + 2 * N;
        for (uint32_t k = t; k < 2 * N; k += TH) psiL[k] = psiT[k];
        psiT = psiL;
    }
    const int2* ipsi = rns + RnsTables::ipsi;
    const int2* mono = rns + RnsTables::mono;
    const int2* keys = rns + rns_keys_off;
    uint64_t* g = acc_io + (size_t)blockIdx.x * twoN;
    const uint64_t* ap = a + (size_t)blockIdx.x * P.n;
    const uint64_t scale = (uint64_t)twoN / amod;
    const uint64_t Q = P.Q, kmask = (1ull << K.kq) - 1;
    auto lpos = [t](int p, int k) -> uint32_t { return (t >> 8) * N + (t & 255) + 256 * (p * CN + k); };
    uint32_t ex[CN];  // slot x of the transform evaluates at psi^(2 bitrev(x) + 1), for every prime
#pragma unroll
    for (int k = 0; k < CN; ++k) ex[k] = 2 * (__builtin_bitreverse32(t + TH * k) >> 21) + 1;

    uint64_t acc[2][CN];  // canonical [0, Q), pass A's layout
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < CN; ++k) {
            const uint64_t v = g[lpos(p, k)];
            acc[p][k] = v >= Q ? v % Q : v;
        }
    __syncthreads();  // forward twiddles in LDS

    for (uint32_t i = 0; i < P.n; ++i) {
        const uint64_t ar = ap[i] % amod;  // rgsw-acc-cggi.cpp:153
        const uint32_t ai = (uint32_t)((ar == 0 ? 0 : amod - ar) * scale);
        int2 R0[8], R1[8];
        r_pair<0, DIG>(P, K, buf, psiT, ipsi, mono, ex, keys, i, ai, acc, R0);
        r_pair<1, DIG>(P, K, buf, psiT + N, ipsi + N, mono + twoN, ex, keys, i, ai, acc, R1);
        // Garner: R = u0 + p0 (u1 + p1 (u2 + p2 u3)), u3 centred (|R| < M/2), then mod Q
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int32_t u0 = canon2p(R0[e].x, K.p[0]);
            const int32_t u1 = canon1p(smul1(canon2p(R0[e].y, K.p[1]) - u0, K.g1, K, 1), K.p[1]);
            const int32_t r2 = canon2p(R1[e].x, K.p[2]);
            const int32_t u2 = canon1p(smul1(r2 - u0 - smul1(u1, K.g2a, K, 2), K.g2, K, 2), K.p[2]);
            const int32_t r3 = canon2p(R1[e].y, K.p[3]);
            int32_t u3 = canon1p(smul1(r3 - u0 - smul1(u1, K.g3a, K, 3) - smul1(u2, K.g3b, K, 3), K.g3, K, 3),
                                 K.p[3]);
            u3 = u3 > (K.p[3] >> 1) ? u3 - K.p[3] : u3;
            const int64_t Z = (int64_t)u3 * K.p[2] + u2;                 // |Z| < 2^51
            const uint64_t Zq = Z < 0 ? (uint64_t)(Z + (int64_t)Q) : (uint64_t)Z;
            const uint64_t Z1 = mulc(Zq, (uint32_t)K.p[1], K) + (uint32_t)u1;
            const uint64_t R = mulc(Z1, (uint32_t)K.p[0], K) + (uint32_t)u0;  // = R mod Q, < 2^kq + 2^51
            const int p = e / CN, k = e % CN;
            uint64_t x = acc[p][k] + R;                                   // < 2^(kq+1) + 2^51
            x = (x & kmask) + (x >> K.kq) * K.c;                          // < 2^kq + 2^22
            acc[p][k] = x >= Q ? x - Q : x;
        }
    }
    __syncthreads();  // every last inverse pass has read its entries
    uint64_t* out = reinterpret_cast<uint64_t*>(lds_r);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < CN; ++k) out[lpos(p, k)] = acc[p][k];
    __syncthreads();
    for (uint32_t k = t; k < N; k += TH) {  // acc0 transposed (poly.cpp:762-770)
        const uint64_t v = out[k == 0 ? 0 : N - k];
        g[k] = k == 0 ? v : (v == 0 ? 0 : Q - v);
        g[N + k] = out[N + k];
    }
}

// ---- setup: arena BSK (NTT mod Q, scaled by N^-1) -> centred integer keys -> RNS NTT ----
// One workgroup per key polynomial: the GS inverse mod Q without scaling gives back the key
// k mod Q (the arena holds NTT(k) N^-1); centred, reduced mod each prime, forward-transformed
// with the kernel's own twiddles, scaled by N^-1 (Montgomery form): K = Mont(NTT_p(k) N^-1).
__device__ __forceinline__ int32_t canon_any(int64_t x, int32_t p) {
    int64_t r = x % p;
    return (int32_t)(r < 0 ? r + p : r);
}
__global__ void __launch_bounds__(256)
k_pack_rns(RnsConst K, uint32_t N, uint64_t Q, const uint64_t* __restrict__ ipsiQ, const uint64_t* __restrict__ ipsiQ_sh,
           const uint64_t* __restrict__ bsk, int2* __restrict__ rns) {
    __shared__ uint64_t q[RN];
    __shared__ int32_t w[RN];
    const uint32_t t = threadIdx.x, T = blockDim.x, half = N / 2;
    const size_t poly = blockIdx.x;
    for (uint32_t x = t; x < N; x += T) q[x] = bsk[poly * N + x] % Q;
    __syncthreads();
    for (uint32_t m = N, len = 1; m > 1; m >>= 1, len <<= 1) {  // GS inverse, no N^-1 (host_ntt_inv)
        const uint32_t h = m >> 1;
        for (uint32_t b = t; b < half; b += T) {
            const uint32_t i = b / len, j = 2 * i * len + b % len;
            const uint64_t U = q[j], V = q[j + len];
            q[j] = addm<uint64_t>(U, V, Q);
            q[j + len] = shoup<uint64_t>(subm<uint64_t>(U, V, Q), ipsiQ[h + i], ipsiQ_sh[h + i], Q);
        }
        __syncthreads();
    }
    const int2* psi = rns + RnsTables::psi;
    const int2* nv = rns + RnsTables::ninv;
    for (int pr = 0; pr < 4; ++pr) {
        const int J = pr >> 1, comp = pr & 1;
        const int32_t p = K.p[pr];
        for (uint32_t x = t; x < N; x += T) {
            const int64_t kc = q[x] > Q / 2 ? (int64_t)q[x] - (int64_t)Q : (int64_t)q[x];
            w[x] = canon_any(kc, p);
        }
        __syncthreads();
        for (uint32_t m = 1, len = N >> 1; m < N; m <<= 1, len >>= 1) {  // CT forward (host_ntt_fwd)
            for (uint32_t b = t; b < half; b += T) {
                const uint32_t i = b / len, j = 2 * i * len + b % len;
                const int2 tw = psi[(size_t)J * RN + m + i];
                const int32_t U = w[j];
                const int32_t V = canon1p(sredc((int64_t)w[j + len] * (comp ? tw.y : tw.x), K.qinv[pr], K.np[pr]), p);
                w[j] = canon1p(U + V - p, p);
                w[j + len] = canon1p(U - V, p);
            }
            __syncthreads();
        }
        const int32_t c = comp ? nv[J].y : nv[J].x;
        int32_t* dst = reinterpret_cast<int32_t*>(rns + rns_keys_off + (poly * 2 + J) * N) + comp;
        for (uint32_t x = t; x < N; x += T) {
            int32_t v = canon1p(sredc((int64_t)w[x] * c, K.qinv[pr], K.np[pr]), p);
            dst[2 * (size_t)x] = v > p / 2 ? v - p : v;
        }
        __syncthreads();
    }
}

// ---- host side ----
uint64_t pw(uint64_t b, uint64_t e, uint64_t m) {
    unsigned __int128 r = 1 % m, x = b % m;
    for (; e; e >>= 1, x = x * x % m)
        if (e & 1) r = r * x % m;
    return (uint64_t)r;
}
bool prime32(uint64_t p) {
    if (p < 2) return false;
    for (uint64_t d = 2; d * d <= p; ++d)
        if (p % d == 0) return false;
    return true;
}
uint32_t bitrev_n(uint32_t x, uint32_t bits) {
    uint32_t r = 0;
    for (uint32_t b = 0; b < bits; ++b) r |= ((x >> b) & 1) << (bits - 1 - b);
    return r;
}
int32_t mont_c(uint64_t v, uint64_t p) {  // v 2^32 mod p, centred
    const uint64_t m = (uint64_t)(((unsigned __int128)(v % p) << 32) % p);
    return m > p / 2 ? (int32_t)((int64_t)m - (int64_t)p) : (int32_t)m;
}
uint64_t inv_mod(uint64_t a, uint64_t p) { return pw(a % p, p - 2, p); }

struct RnsHost {
    RnsConst K{};
    std::vector<int2> tables;  // RnsTables::words
    bool ok = false;
};

// The four primes (largest p = 1 mod 2N below 2^26), their Montgomery constants and tables, and
// the CRT range check: 4 dG2 N max|digit| (Q-1)/2 < M/2 (tools/bounds_rns.py).
RnsHost rns_host(const BRParams& P) {
    RnsHost H;
    if (P.N != RN || P.Q < (1ull << 50) || P.Q >= (1ull << 58) || P.logG > 27 || P.logG < 2 || P.digits < 1 ||
        P.digits > 2)
        return H;
    uint32_t kq = 0;
    while ((1ull << kq) < P.Q) ++kq;
    const uint64_t c = (1ull << kq) - P.Q;
    if (kq < 53 || kq > 58 || c >= (1ull << 20)) return H;
    std::vector<uint64_t> pr;
    for (uint64_t p = ((1ull << 26) - 1) / (2 * RN) * (2 * RN) + 1; pr.size() < 4 && p > (1ull << 25); p -= 2 * RN)
        if (p < (1ull << 26) && prime32(p)) pr.push_back(p);
    if (pr.size() < 4) return H;
    // max |digit|: B/2 for the full digits, the top digit of a centred |c| < Q/2 otherwise
    const unsigned __int128 B = (unsigned __int128)1 << P.logG;
    unsigned __int128 top = (unsigned __int128)(P.Q / 2);
    for (uint32_t z = 0; z + 1 < P.thr + P.digits; ++z) top /= B;
    const unsigned __int128 maxd = std::max<unsigned __int128>(B / 2 + 1, top + 2);
    const long double bound = 4.0L * P.dG2 * P.N * (long double)maxd * (long double)(P.Q / 2);
    long double M = 1;
    for (uint64_t p : pr) M *= (long double)p;
    if (!(bound < M / 2 / 1.0001L)) return H;
    RnsConst& K = H.K;
    for (int i = 0; i < 4; ++i) {
        const uint32_t p = (uint32_t)pr[i];
        uint32_t inv = 1;
        for (int it = 0; it < 5; ++it) inv *= 2u - p * inv;
        K.p[i] = (int32_t)p, K.np[i] = -(int32_t)p, K.qinv[i] = (int32_t)inv;
        K.rM[i] = mont_c(1, p);
    }
    const uint64_t p0 = pr[0], p1 = pr[1], p2 = pr[2], p3 = pr[3];
    K.g1 = mont_c(inv_mod(p0, p1), p1);
    K.g2a = mont_c(p0 % p2, p2);
    K.g2 = mont_c(inv_mod(p0 * p1 % p2, p2), p2);
    K.g3a = mont_c(p0 % p3, p3);
    K.g3b = mont_c(p0 * p1 % p3, p3);
    K.g3 = mont_c(inv_mod((unsigned __int128)p0 * p1 % p3 * p2 % p3, p3), p3);
    K.Q = P.Q, K.kq = kq, K.c = (uint32_t)c;
    // tables: twiddles psi^bitrev(k) (any primitive 2N-th root: the slot exponents e_x =
    // 2 bitrev(x) + 1 depend only on the transform's structure), monomials psi^k - 1
    H.tables.assign(RnsTables::words, make_int2(0, 0));
    const uint32_t logN = 11;
    for (int i = 0; i < 4; ++i) {
        const uint64_t p = pr[i];
        uint64_t psi = 0;
        for (uint64_t gq = 2;; ++gq) {
            psi = pw(gq, (p - 1) / (2 * RN), p);
            if (pw(psi, RN, p) == p - 1) break;
        }
        const uint64_t ipsi = inv_mod(psi, p);
        const int J = i >> 1, comp = i & 1;
        auto put = [&](size_t idx, int32_t v) { (comp ? H.tables[idx].y : H.tables[idx].x) = v; };
        for (uint32_t k = 0; k < RN; ++k) {
            const uint32_t e = bitrev_n(k, logN);
            put(RnsTables::psi + (size_t)J * RN + k, mont_c(pw(psi, e, p), p));
            put(RnsTables::ipsi + (size_t)J * RN + k, mont_c(pw(ipsi, e, p), p));
        }
        uint64_t x = 1;
        for (uint32_t k = 0; k < 2 * RN; ++k, x = x * psi % p) put(RnsTables::mono + (size_t)J * 2 * RN + k, mont_c((x + p - 1) % p, p));
        // keys: Mont(k N^-1) = sredc(k * ninv) with ninv = N^-1 R^2 mod p
        const uint64_t ninvR = (uint64_t)(((unsigned __int128)inv_mod(RN, p) << 32) % p);
        put(RnsTables::ninv + J, mont_c(ninvR, p));
    }
    H.ok = true;
    return H;
}

}  // namespace

bool rns_path_supported(const BRParams& P) { return rns_host(P).ok; }

size_t rns_keys_bytes(const BRParams& P) { return (rns_keys_off + (size_t)P.n * 4 * P.dG2 * 2 * RN) * sizeof(int2); }

hipError_t launch_pack_bsk_rns(const BRParams& P, const DevTables& T, const void* bsk, void* out, hipStream_t s) {
    const RnsHost H = rns_host(P);
    if (!H.ok) return hipErrorNotSupported;
    hipError_t e = hipMemcpyAsync(out, H.tables.data(), H.tables.size() * sizeof(int2), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(s);  // H.tables is host memory that goes out of scope
    if (e != hipSuccess) return e;
    const size_t polys = (size_t)P.n * 2 * P.dG2 * 2;
    hipLaunchKernelGGL(k_pack_rns, dim3((unsigned)polys), dim3(256), 0, s, H.K, P.N, P.Q, (const uint64_t*)T.ipsi,
                       (const uint64_t*)T.ipsi_sh, (const uint64_t*)bsk, (int2*)out);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_rns(const BRParams& P, const DevTables& T, const void* keys, const uint64_t* a,
                                   uint64_t amod, uint64_t* acc, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    static thread_local BRParams lastP{};
    static thread_local RnsConst lastK{};
    const bool same = lastP.N == P.N && lastP.n == P.n && lastP.dG2 == P.dG2 && lastP.digits == P.digits &&
                      lastP.thr == P.thr && lastP.logG == P.logG && lastP.Q == P.Q;
    if (!same) {
        const RnsHost H = rns_host(P);
        if (!H.ok) return hipErrorNotSupported;
        lastK = H.K, lastP = P;
    }
    const size_t lds = (size_t)4 * RN * sizeof(int2);  // DIG 1: buffer [2][N] + twiddles [2][N]; DIG 2: [2][2][N]
    auto go = [&](auto kern) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(RTH), lds, s, P, lastK, (const int2*)keys, a, amod, acc);
    };
    if (P.digits == 1) go(k_blind_rotate_rns<1>);
    else go(k_blind_rotate_rns<2>);
    return hipGetLastError();
}

}  // namespace tfhe
