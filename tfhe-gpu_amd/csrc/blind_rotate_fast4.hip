// blind_rotate_fast4.hip -- STD128-class blind rotation, four wavefronts per ciphertext.
//
// Same round as k_blind_rotate_fast2 (blind_rotate_fast.hip: top digit eliminated through the
// NTT-domain accumulator C, digit-folded key rows, signed Montgomery arithmetic), laid out for
// four waves per SIMD instead of three:
//
//  * 256 lanes per ciphertext (one workgroup), 4 coefficients of each polynomial per lane, so
//    the per-lane state halves (row sums 32 VGPRs, accumulator 8, C 8) and the kernel fits
//    128 VGPRs.  A 1024-point transform is five radix-4 register passes over the index-bit
//    pairs (b9 b8) (b7 b6) (b5 b4) (b3 b2) (b1 b0) with four LDS exchanges; only the last
//    one crosses wavefronts (tools/lds_layouts4.py models and checks all eight exchanges):
//        L1 regs (b8 b9)  lanes (b2 b3 b4 b6 b7 b5)  waves (b0 b1)   coefficient order
//        L2 regs (b6 b7)  lanes (b2 b3 b8 b9 b4 b5)  waves (b0 b1)
//        L3 regs (b4 b5)  lanes (b2 b3 b6 b8 b9 b7)  waves (b0 b1)
//        L4 regs (b2 b3)  lanes (b4 b5 b6 b8 b9 b7)  waves (b0 b1)
//        L5 regs (b0 b1)  lanes (b2 .. b7)           waves (b8 b9)   MAC: lane t owns slots 4t..4t+3
//    Every exchange stores lane-contiguous rows (ds_write_addtid_b32) and gathers with
//    conflict-free ds_read_b32.  The cross-wavefront exchange uses one LDS area (XB = 1, the
//    default: a barrier after its stores and a plain one before them) or alternates between
//    two (XB = 2: no barrier before the stores, 18 KiB more LDS; measured no faster).
//  * Key rows stream through a ring: while the MAC consumes group g of one digit, group g of
//    the next digit (or of the next round's C rows) is loaded into the freed registers, so
//    every row has a whole transform to arrive.
//  * Twiddles of pass 4 are per-lane constants kept in registers, pass 0's are uniform
//    (SGPRs), passes 1-3 come from LDS (ds_read_b128).  Pass 0 of a digit polynomial (7-bit
//    inputs) reads all its products from three 128-entry LDS tables.
//  * Inverse passes on L4 and L2 reduce their second-stage sums (tools/bounds_fast4.py).
#include "device_math.hpp"
#include "kernels.hpp"

namespace tfhe {
namespace f4 {

constexpr uint32_t FN = 1024;
constexpr int TPC = 256;

// Global table block written by k_pack_fast (blind_rotate_fast.hip), int32 centred Montgomery:
//   pass p >= 1 block c (m = 4^p): [psi[m+c], psi[2m+2c], psi[2m+2c+1], 0]; pass 0 = block 0 of m = 1
constexpr uint32_t P0F = 0, P1F = 4, P2F = 20, P3F = 84, P4F = 340, PF_END = 1364;
constexpr uint32_t P0I = PF_END, P1I = P0I + P1F, P4I = P0I + P4F;
constexpr uint32_t T4_MONO = 2 * PF_END, T4_T1 = T4_MONO + 2 * FN, T4_T23 = T4_T1 + 128, T4_T2131 = T4_T23 + 256,
                   T4_WORDS = T4_T2131 + 256;
// LDS (words): pass 1-3 twiddles (fwd, inv), monomials, 4 local regions, 2 cross areas
constexpr uint32_t L_TW = 0, L_TWI = P4F - P1F, L_MONO = 2 * L_TWI;  // passes 1-3 (fwd, inv)
// then, for P polynomials per wavefront: 4 local regions of P x LP words, 2 cross areas of P x XP
// T1[d + 64] = d psi[1] mod Q for digits d in [-64, 64): pass 0's first stage on a digit polynomial
// T23[d] = (d psi[2], d psi[3]), T2131[d] = (d psi[2] psi[1], d psi[3] psi[1]): the rest of pass 0
// P4F: pass-4 forward twiddles, lane order (one ds_read_b128 per lane, conflict-free)
constexpr uint32_t L_T1 = L_MONO + 2 * FN, L_T23 = L_T1 + 128, L_T2131 = L_T23 + 256, L_P4F = L_T2131 + 256;
constexpr uint32_t LP = 304, XP = 1152, L_CT = L_P4F + 4 * 256;
constexpr size_t lds_bytes(int P, int XB = 2, int CTS = 1) { return (size_t)(L_CT + CTS * (4 * P * LP + XB * P * XP)) * 4; }

struct Lay {
    int reg[2];
    int lane[6];
    int wave[2];
};
__host__ __device__ constexpr Lay lay(int L) {
    return L == 1   ? Lay{{8, 9}, {2, 3, 4, 6, 7, 5}, {0, 1}}
           : L == 2 ? Lay{{6, 7}, {2, 3, 8, 9, 4, 5}, {0, 1}}
           : L == 3 ? Lay{{4, 5}, {2, 3, 6, 8, 9, 7}, {0, 1}}
           : L == 4 ? Lay{{2, 3}, {4, 5, 6, 8, 9, 7}, {0, 1}}
                    : Lay{{0, 1}, {2, 3, 4, 5, 6, 7}, {8, 9}};
}
// (row stride of the writer's register rows, stride of its wavefront blocks; 0 = local)
__host__ __device__ constexpr int rstride(int A, int B) {
    return (A == 1 && B == 2) ? 72 : (A == 2 && B == 3) ? 80 : (A == 3 && B == 4) ? 65
         : (A == 2 && B == 1) ? 68 : (A == 3 && B == 2) ? 68 : (A == 4 && B == 3) ? 65
         : (A == 4 && B == 5) ? 72 : 64;
}
__host__ __device__ constexpr int wstride(int A, int B) { return (A == 4 && B == 5) ? 288 : (A == 5 && B == 4) ? 257 : 0; }
// LDS words contributed by index bit b in exchange A -> B (its position in the writer's layout)
__host__ __device__ constexpr int wt(int A, int B, int b) {
    for (int k = 0; k < 2; ++k)
        if (lay(A).reg[k] == b) return rstride(A, B) << k;
    for (int k = 0; k < 6; ++k)
        if (lay(A).lane[k] == b) return 1 << k;
    for (int k = 0; k < 2; ++k)
        if (lay(A).wave[k] == b) return wstride(A, B) << k;
    return 1 << 24;
}
template <int L>
__device__ __forceinline__ uint32_t elem(uint32_t w, uint32_t lane, uint32_t r) {
    uint32_t i = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) i |= ((r >> k) & 1) << lay(L).reg[k];
#pragma unroll
    for (int k = 0; k < 6; ++k) i |= ((lane >> k) & 1) << lay(L).lane[k];
#pragma unroll
    for (int k = 0; k < 2; ++k) i |= ((w >> k) & 1) << lay(L).wave[k];
    return i;
}
// writer register r: row offset (words); reader register r: gather offset (words)
__host__ __device__ constexpr int st_reg(int A, int B, int r) {
    int o = 0;
    for (int k = 0; k < 2; ++k)
        if ((r >> k) & 1) o += wt(A, B, lay(A).reg[k]);
    return o;
}
__host__ __device__ constexpr int ld_reg(int A, int B, int r) {
    int o = 0;
    for (int k = 0; k < 2; ++k)
        if ((r >> k) & 1) o += wt(A, B, lay(B).reg[k]);
    return o;
}
// reader lane/wave part of a gather address (words)
template <int A, int B>
__device__ __forceinline__ uint32_t ld_lane(uint32_t w, uint32_t lane) {
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) o += ((lane >> k) & 1) * (uint32_t)wt(A, B, lay(B).lane[k]);
    if (wstride(A, B) != 0) {
#pragma unroll
        for (int k = 0; k < 2; ++k) o += ((w >> k) & 1) * (uint32_t)wt(A, B, lay(B).wave[k]);
    }
    return o;
}
// writer wavefront part of a cross-exchange row address (words)
template <int A, int B>
__host__ __device__ constexpr uint32_t st_wave(uint32_t w) {
    uint32_t o = 0;
    for (int k = 0; k < 2; ++k) o += ((w >> k) & 1) * (uint32_t)wt(A, B, lay(A).wave[k]);
    return o;
}

struct FastConst {  // same layout as blind_rotate_fast.hip's
    int32_t Q, nQ, qinv, rM;
    uint32_t Q2, Q4, h1, kacc;
    int32_t ninv;
    uint32_t bm;  // floor(2^32 / Q)
};
__device__ __forceinline__ int32_t sredc(int64_t T, const FastConst& K) {
    const int32_t m = (int32_t)((uint32_t)T * (uint32_t)K.qinv);
    return (int32_t)(((int64_t)m * K.nQ + T) >> 32);
}
__device__ __forceinline__ int32_t smul(int32_t a, int32_t wM, const FastConst& K) { return sredc((int64_t)a * wM, K); }
__device__ __forceinline__ uint32_t csub32(uint32_t a, uint32_t m) { return min(a, a - m); }
// s + a b as one v_mad_i64_i32: s passes through an empty asm so the compiler cannot
// re-associate a row sum's terms into (a b + c d) + s, which costs a separate 64-bit add per pair
// (24 per wave-round)
__device__ __forceinline__ int64_t mac64(int32_t a, int32_t b, int64_t s) {
    asm("" : "+v"(s));  // opaque: the sum is formed in this order
    return (int64_t)a * b + s;
}

typedef int32_t v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i ld_bsk(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}

__device__ __forceinline__ void bfly_ct(int32_t& a, int32_t& b, int32_t w, const FastConst& K) {
    const int32_t v = smul(b, w, K), u = a;
    a = u + v;
    b = u - v;
}
template <bool RED = false>
__device__ __forceinline__ void bfly_gs(int32_t& a, int32_t& b, int32_t w, const FastConst& K) {
    const int32_t u = a, v = b;
    a = RED ? smul(u + v, K.rM, K) : u + v;
    b = smul(u - v, w, K);
}
// radix-4 CT pass over register bits (1, 0): w = [psi[m+c], psi[2m+2c], psi[2m+2c+1]]
__device__ __forceinline__ void fwd4(int32_t (&x)[4], int32_t w1, int32_t w2, int32_t w3, const FastConst& K) {
    bfly_ct(x[0], x[2], w1, K);
    bfly_ct(x[1], x[3], w1, K);
    bfly_ct(x[0], x[1], w2, K);
    bfly_ct(x[2], x[3], w3, K);
}
template <bool RED>
__device__ __forceinline__ void inv4(int32_t (&x)[4], int32_t w1, int32_t w2, int32_t w3, const FastConst& K) {
    bfly_gs(x[0], x[1], w2, K);
    bfly_gs(x[2], x[3], w3, K);
    bfly_gs<RED>(x[0], x[2], w1, K);
    bfly_gs<RED>(x[1], x[3], w1, K);
}

// ---- LDS traffic (inline asm: counted lgkmcnt waits, addtid stores) ----
// one polynomial's 4 registers as 4 lane-contiguous rows at M0 + OFF
template <int A, int B, uint32_t OFF>
__device__ __forceinline__ void store_rows(const int32_t (&x)[4], uint32_t m0, const int32_t* lds) {
    asm volatile(
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "ds_write_addtid_b32 %0 offset:%6\n\t"
        "ds_write_addtid_b32 %1 offset:%7\n\t"
        "ds_write_addtid_b32 %2 offset:%8\n\t"
        "ds_write_addtid_b32 %3 offset:%9" ::"v"(x[0]),
        "v"(x[1]), "v"(x[2]), "v"(x[3]), "s"(m0), "s"(lds), "i"((OFF + st_reg(A, B, 0)) * 4),
        "i"((OFF + st_reg(A, B, 1)) * 4), "i"((OFF + st_reg(A, B, 2)) * 4), "i"((OFF + st_reg(A, B, 3)) * 4)
        : "memory");
}
template <int A, int B, uint32_t OFF>
__device__ __forceinline__ void gather_rows(int32_t (&x)[4], uint32_t base, const int32_t* lds) {
    asm volatile(
        "ds_read_b32 %0, %4 offset:%6\n\t"
        "ds_read_b32 %1, %4 offset:%7\n\t"
        "ds_read_b32 %2, %4 offset:%8\n\t"
        "ds_read_b32 %3, %4 offset:%9"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
        : "v"(base), "s"(lds), "i"((OFF + ld_reg(A, B, 0)) * 4), "i"((OFF + ld_reg(A, B, 1)) * 4),
          "i"((OFF + ld_reg(A, B, 2)) * 4), "i"((OFF + ld_reg(A, B, 3)) * 4)
        : "memory");
}
template <uint32_t OFF>
__device__ __forceinline__ void tw_load(v4i& w, uint32_t addr, const int32_t* lds) {
    asm volatile("ds_read_b128 %0, %1 offset:%3" : "=&v"(w) : "v"(addr), "s"(lds), "i"(OFF * 4) : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait(int32_t (&x)[4]) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait(int32_t (&x)[4], v4i& w) {
    asm volatile("s_waitcnt lgkmcnt(%5)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(w)
                 : "i"(N)
                 : "memory");
}
__device__ __forceinline__ void lds_drain_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
}

// per-lane constants of the transforms
struct LaneCtx {
    uint32_t g12, g23, g34, g45, g54, g43, g32, g21;  // gather bases (bytes; local ones include the region)
    uint32_t m_loc;                                   // this wavefront's local region (bytes, uniform)
    uint32_t m45, m54;                                // cross-store wave offsets (bytes, uniform)
    uint32_t t1, t2, t3, t4;                          // pass 1 / 2 / 3 / 4 twiddle block addresses (bytes)
    int32_t w0f[3], w0i[3];                           // pass 0 (uniform)
    v4i w4f, w4i;                                     // pass 4 (per lane)
};

// ---- transforms of P polynomials (P = 2 per ciphertext of the wavefront) ----
// Every exchange step runs, per polynomial: wait for its gathered rows, its radix-4 pass, its
// row stores; then (cross steps: drain + barrier) all gathers.  While polynomial p's pass
// runs, the rows of p+1.. are still in flight: the wait for polynomial p always leaves the
// 4 (P-1) younger operations outstanding (the gathers of p+1.. plus the stores of ..p-1).
// EXP (timing experiments, results invalid): bit 0 no barriers, bit 1 no key loads, bit 3 no
// transforms at all.
// FOR_P(body): body once per polynomial with a compile-time constant p
#define FOR_P(...)                                   \
    {                                                \
        { constexpr int p = 0; __VA_ARGS__ }         \
        if constexpr (P > 1) {                       \
            { constexpr int p = 1; __VA_ARGS__ }     \
        }                                            \
        if constexpr (P > 2) {                       \
            { constexpr int p = 2; __VA_ARGS__ }     \
            { constexpr int p = 3; __VA_ARGS__ }     \
        }                                            \
    }
// wait for polynomial p's gathered rows at the end of a transform (no stores follow)
template <int P, int p>
constexpr int tail_wait() { return 4 * (P - 1 - p); }

// SMALL (inputs are digits in [-64, 64)): 1 = pass 0's first-stage products from T1, 2 = all of
// pass 0's products from T1, T23, T2131 (3 address computations + 8 additions per polynomial).
// P4L: pass-4 twiddles from LDS (L_P4F) instead of registers.
// PRE: one cross area only, so every wavefront must have finished reading its previous
// contents before anyone stores (a plain barrier: those reads completed long ago)
template <uint32_t XA, int P, int EXP = 0, int SMALL = 0, bool PRE = false, bool P4L = false>
__device__ __forceinline__ void ntt_fwd(int32_t (&X)[P][4], const int32_t* lds, const LaneCtx& C, const FastConst& K) {
    if constexpr ((EXP & 8) != 0) return;
    constexpr int W = 4 * (P - 1);
    v4i w;
    // pass 0 (L1), exchange 1 -> 2
    if constexpr (SMALL == 2) {
        const int32_t* t1 = lds + L_T1 + 64;
        const int2* t23 = reinterpret_cast<const int2*>(lds + L_T23) + 64;
        const int2* t2131 = reinterpret_cast<const int2*>(lds + L_T2131) + 64;
        int32_t a[P];
        int2 u23[P], u2131[P];
        FOR_P(a[p] = t1[X[p][2]]; u23[p] = t23[X[p][1]]; u2131[p] = t2131[X[p][3]];)
        FOR_P(const int32_t x0 = X[p][0], u = u23[p].x + u2131[p].x, v = u23[p].y - u2131[p].y;
              const int32_t e0 = x0 + a[p], e2 = x0 - a[p];
              X[p][0] = e0 + u; X[p][1] = e0 - u; X[p][2] = e2 + v; X[p][3] = e2 - v;
              store_rows<1, 2, p * LP>(X[p], C.m_loc, lds);)
    } else if constexpr (SMALL == 1) {
        const int32_t* t1 = lds + L_T1 + 64;
        int32_t v[P][2];
        FOR_P(v[p][0] = t1[X[p][2]]; v[p][1] = t1[X[p][3]];)
        FOR_P(const int32_t a0 = X[p][0], a1 = X[p][1];
              X[p][0] = a0 + v[p][0]; X[p][2] = a0 - v[p][0]; X[p][1] = a1 + v[p][1]; X[p][3] = a1 - v[p][1];
              bfly_ct(X[p][0], X[p][1], C.w0f[1], K); bfly_ct(X[p][2], X[p][3], C.w0f[2], K);
              store_rows<1, 2, p * LP>(X[p], C.m_loc, lds);)
    } else {
        FOR_P(fwd4(X[p], C.w0f[0], C.w0f[1], C.w0f[2], K); store_rows<1, 2, p * LP>(X[p], C.m_loc, lds);)
    }
    tw_load<L_TW>(w, C.t1, lds);
    FOR_P(gather_rows<1, 2, p * LP>(X[p], C.g12, lds);)
    // pass 1 (L2), exchange 2 -> 3
    FOR_P(if constexpr (p == 0) lds_wait<W>(X[0], w); else lds_wait<W>(X[p]);
          fwd4(X[p], w.x, w.y, w.z, K); store_rows<2, 3, p * LP>(X[p], C.m_loc, lds);)
    tw_load<L_TW + 16>(w, C.t2, lds);
    FOR_P(gather_rows<2, 3, p * LP>(X[p], C.g23, lds);)
    // pass 2 (L3), exchange 3 -> 4
    FOR_P(if constexpr (p == 0) lds_wait<W>(X[0], w); else lds_wait<W>(X[p]);
          fwd4(X[p], w.x, w.y, w.z, K); store_rows<3, 4, p * LP>(X[p], C.m_loc, lds);)
    tw_load<L_TW + 80>(w, C.t3, lds);
    FOR_P(gather_rows<3, 4, p * LP>(X[p], C.g34, lds);)
    // pass 3 (L4), cross exchange 4 -> 5
    FOR_P(if constexpr (p == 0) lds_wait<W>(X[0], w); else lds_wait<W>(X[p]);
          fwd4(X[p], w.x, w.y, w.z, K);
          if constexpr (PRE && p == 0) __builtin_amdgcn_s_barrier();
          store_rows<4, 5, XA + p * XP>(X[p], C.m45, lds);)
    if constexpr (!(EXP & 1)) lds_drain_barrier();
    if constexpr (P4L) tw_load<L_P4F>(w, C.t4, lds);
    FOR_P(gather_rows<4, 5, XA + p * XP>(X[p], C.g45, lds);)
    // pass 4 (L5)
    if constexpr (P4L) {
        FOR_P(if constexpr (p == 0) lds_wait<tail_wait<P, 0>()>(X[0], w); else lds_wait<tail_wait<P, p>()>(X[p]);
              fwd4(X[p], w.x, w.y, w.z, K);)
    } else {
        FOR_P(lds_wait<tail_wait<P, p>()>(X[p]); fwd4(X[p], C.w4f.x, C.w4f.y, C.w4f.z, K);)
    }
}

// inverse (N^-1 folded into the keys), L5 -> L1
template <uint32_t XA, int P, int EXP = 0, bool PRE = false>
__device__ __forceinline__ void ntt_inv(int32_t (&X)[P][4], const int32_t* lds, const LaneCtx& C, const FastConst& K) {
    if constexpr ((EXP & 8) != 0) return;
    constexpr int W = 4 * (P - 1);
    v4i w;
    // (b0 b1) (L5), cross exchange 5 -> 4
    FOR_P(inv4<false>(X[p], C.w4i.x, C.w4i.y, C.w4i.z, K); if constexpr (PRE && p == 0) __builtin_amdgcn_s_barrier();
          store_rows<5, 4, XA + p * XP>(X[p], C.m54, lds);)
    if constexpr (!(EXP & 1)) lds_drain_barrier();
    tw_load<L_TWI + 80>(w, C.t3, lds);
    FOR_P(gather_rows<5, 4, XA + p * XP>(X[p], C.g54, lds);)
    // (b2 b3) (L4, reduced), exchange 4 -> 3
    FOR_P(if constexpr (p == 0) lds_wait<W>(X[0], w); else lds_wait<W>(X[p]);
          inv4<true>(X[p], w.x, w.y, w.z, K);
          store_rows<4, 3, p * LP>(X[p], C.m_loc, lds);)
    tw_load<L_TWI + 16>(w, C.t2, lds);
    FOR_P(gather_rows<4, 3, p * LP>(X[p], C.g43, lds);)
    // (b4 b5) (L3), exchange 3 -> 2
    FOR_P(if constexpr (p == 0) lds_wait<W>(X[0], w); else lds_wait<W>(X[p]);
          inv4<false>(X[p], w.x, w.y, w.z, K); store_rows<3, 2, p * LP>(X[p], C.m_loc, lds);)
    tw_load<L_TWI>(w, C.t1, lds);
    FOR_P(gather_rows<3, 2, p * LP>(X[p], C.g32, lds);)
    // (b6 b7) (L2, reduced), exchange 2 -> 1
    FOR_P(if constexpr (p == 0) lds_wait<W>(X[0], w); else lds_wait<W>(X[p]);
          inv4<true>(X[p], w.x, w.y, w.z, K); store_rows<2, 1, p * LP>(X[p], C.m_loc, lds);)
    FOR_P(gather_rows<2, 1, p * LP>(X[p], C.g21, lds);)
    // (b8 b9) (L1)
    FOR_P(lds_wait<tail_wait<P, p>()>(X[p]); inv4<false>(X[p], C.w0i[0], C.w0i[1], C.w0i[2], K);)
}

// NCT ciphertexts per wavefront (the same slots of each): every key row loaded feeds NCT
// ciphertexts, halving the vector-memory traffic per bootstrap at NCT = 2.
// OPT bit 0: T1 lookups in the digit transforms (bit 2: all of pass 0 from tables); bit 1: Barrett
// accumulator update; bit 3: pass-4 forward twiddles from LDS
// XB: cross-exchange areas (2: alternate, no barrier before the stores; 1: one area + a barrier)
// CTS (NCT = 1): ciphertexts per workgroup, in lockstep through the transforms' barriers, so
// their wavefronts read each key row at about the same time (L1 reuse instead of L2 traffic).
// SPLIT (small batches; CHES-experiments.cpp's 256-gate calls): one ciphertext per 512-thread workgroup, its
// two polynomials on two groups of four wavefronts -- group g runs this kernel's round on accumulator
// polynomial g alone (digits, forward transforms, C_g, the inverse of column g, the update of acc_g) --
// and the external product is split by polynomial: group g forms the row sums of its own polynomial's
// digit / C rows for BOTH columns, reduces them (sredc), and hands the other column's 8 partial sums per
// lane to the other group through LDS (one barrier); each then finishes column g.  Half of every
// transform, product and monomial step per wavefront, twice the wavefronts per ciphertext: at 256
// ciphertexts a CU runs 2 waves per SIMD instead of 1.
// Digit shape (any N = 1024 set with Q < 2^27 and baseG <= 2^9; tools/bounds_fast4.py): DIG digits
// per polynomial (dG2 = 2 DIG), baseG = 2^LOGG, THR thrown digits.  FOLD: the top digit is
// eliminated (its rows carry C = N^-1 NTT(acc), k_pack_fast folds it into the other rows), valid
// when THR = 0 and the top digit never wraps (the host checks); otherwise every digit is
// transformed.  Pass 0's lookup tables hold digits in [-64, 64), so they need LOGG <= 7.
template <int MINW, int NCT = 1, int EXP = 0, int OPT = 7, int XB = 2, int CTS = 1, int DIG = 4, int LOGG = 7,
          int THR = 0, bool FOLD = true, bool FLAG = false, bool SPLIT = false>
__global__ void __launch_bounds__(TPC * (SPLIT ? 2 : CTS), MINW)
k_blind_rotate_fast4(FastConst K, uint32_t n, uint32_t loga, const int32_t* __restrict__ tabs,
                     const int32_t* __restrict__ bsk, const uint64_t* __restrict__ a, uint64_t* __restrict__ acc_io,
                     uint32_t B, uint32_t* __restrict__ done) {
    constexpr int NPOL = SPLIT ? 1 : 2;   // accumulator polynomials per lane
    constexpr int P = NPOL * NCT;         // polynomials per transform
    constexpr int GR = SPLIT ? 2 : CTS;   // 256-thread groups per workgroup
    extern __shared__ __align__(16) int32_t lds[];
    static_assert(CTS == 1 || NCT == 1, "CTS > 1 needs NCT = 1");
    static_assert(!SPLIT || (NCT == 1 && CTS == 1 && FOLD && !FLAG && XB == 1), "SPLIT: the folded one-ciphertext build");
    constexpr uint32_t RW = 2 * DIG;                  // key rows per (key, column)
    constexpr int TOP = DIG - 1;                       // FOLD: the eliminated digit (its rows: the C products)
    constexpr int NT = FOLD ? DIG - 1 : DIG;           // transformed digits per round
    static_assert(!FOLD || THR == 0, "top-digit elimination needs every digit");
    static_assert(LOGG * (THR + NT) <= 32, "digit field beyond 32 bits");
    // XB = 2 alternates cross areas between consecutive transforms: laid out for STD128's order only
    static_assert(XB == 1 || (DIG == 4 && FOLD), "two cross areas need the STD128 digit order");
    const uint32_t cl = __builtin_amdgcn_readfirstlane(threadIdx.x / TPC);  // group: ciphertext (SPLIT: polynomial)
    const uint32_t tid = threadIdx.x % TPC;
    const uint32_t wg_ct = SPLIT ? blockIdx.x : blockIdx.x * CTS * NCT + cl;  // first ciphertext of this lane
    const uint32_t pol = SPLIT ? cl : 0;                                      // SPLIT: this group's polynomial
    for (uint32_t k = threadIdx.x; k < L_TWI; k += TPC * GR) lds[L_TW + k] = tabs[P1F + k], lds[L_TWI + k] = tabs[P1I + k];
    for (uint32_t k = threadIdx.x; k < 2 * FN + 640; k += TPC * GR) lds[L_MONO + k] = tabs[T4_MONO + k];  // monomials, T1/T23/T2131
    if constexpr ((OPT & 8) != 0)
        for (uint32_t k = threadIdx.x; k < 4 * 256; k += TPC * GR) lds[L_P4F + k] = tabs[P4F + k];
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    constexpr uint32_t LOCW = P * LP, XAW = P * XP;       // local region per wave, cross area (words)
    constexpr uint32_t XA0 = 4 * LOCW, XA1 = XB == 2 ? XA0 + XAW : XA0;  // cross areas, relative to L_CT
    constexpr bool PRE = XB == 1;

    LaneCtx C;
    constexpr uint32_t CTW = 4 * LOCW + XB * XAW;        // LDS words per ciphertext group
    const uint32_t ctb = (L_CT + cl * CTW) * 4;         // bytes, uniform
    C.m_loc = ctb + w * LOCW * 4;
    C.g12 = C.m_loc + ld_lane<1, 2>(w, lane) * 4, C.g23 = C.m_loc + ld_lane<2, 3>(w, lane) * 4;
    C.g34 = C.m_loc + ld_lane<3, 4>(w, lane) * 4, C.g43 = C.m_loc + ld_lane<4, 3>(w, lane) * 4;
    C.g32 = C.m_loc + ld_lane<3, 2>(w, lane) * 4, C.g21 = C.m_loc + ld_lane<2, 1>(w, lane) * 4;
    C.g45 = ctb + ld_lane<4, 5>(w, lane) * 4, C.g54 = ctb + ld_lane<5, 4>(w, lane) * 4;
    C.m45 = ctb + st_wave<4, 5>(w) * 4, C.m54 = ctb + st_wave<5, 4>(w) * 4;
    C.t1 = (elem<2>(w, lane, 0) >> 8) * 16, C.t2 = (elem<3>(w, lane, 0) >> 6) * 16;
    C.t3 = (elem<4>(w, lane, 0) >> 4) * 16, C.t4 = tid * 16;
    const v4i* tv = reinterpret_cast<const v4i*>(tabs);
    if constexpr ((OPT & 8) == 0) C.w4f = tv[P4F / 4 + tid];
    C.w4i = tv[P4I / 4 + tid];
#pragma unroll
    for (int k = 0; k < 3; ++k) C.w0f[k] = tabs[P0F + k], C.w0i[k] = tabs[P0I + k];

    const uint32_t Qh = (uint32_t)K.Q >> 1;
    int32_t acc[NCT][NPOL][4];  // L1, centred canonical
#pragma unroll
    for (int q = 0; q < NCT; ++q) {
        const uint32_t ct = wg_ct + q;
        const uint64_t* g = acc_io + (size_t)(ct < B ? ct : 0) * 2 * FN;
#pragma unroll
        for (int p = 0; p < NPOL; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint64_t v0 = ct < B ? g[(SPLIT ? pol : p) * FN + elem<1>(w, lane, r)] : 0;
                const uint32_t v = (uint32_t)(v0 >= (uint64_t)K.Q ? v0 % (uint64_t)K.Q : v0);
                acc[q][p][r] = v < Qh ? (int32_t)v : (int32_t)v - K.Q;
            }
    }
    __syncthreads();

    // C = N^-1 NTT(acc) in L5
    int32_t Cp[P][4];
    if constexpr (FOLD) {
        if constexpr (SPLIT) {
#pragma unroll
            for (int r = 0; r < 4; ++r) Cp[0][r] = acc[0][0][r];
        } else {
#pragma unroll
            for (int q = 0; q < NCT; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) Cp[2 * q][r] = acc[q][0][r], Cp[2 * q + 1][r] = acc[q][NPOL - 1][r];
        }
        ntt_fwd<XA1, P, EXP, 0, PRE, (OPT & 8) != 0>(Cp, lds, C, K);
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r) Cp[p][r] = smul(Cp[p][r], K.ninv, K);
    }

    constexpr uint32_t ROWB = 2 * RW * 2 * FN * 4;  // key bytes per round
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(bsk), 0, (int)(n * ROWB), 0x00020000);
    const uint32_t voff = tid * 16;  // 4 consecutive slots per lane
    const uint32_t et = 2 * (__builtin_bitreverse32(tid) >> 24) + 1;  // slot 4t + r: e = 512 bitrev2(r) + et
    const uint32_t amask = (1u << loga) - 1, ashift = 11 - loga;

    // group gi = (key k, column j) of digit l (FOLD, l = TOP: the C rows): rows 2l (poly 0), 2l + 1 (poly 1)
    auto issue = [&](v4i (&pw)[2], uint32_t round_off, int l, int gi) {
        const int k = gi >> 1, j = gi & 1;
        if constexpr ((EXP & 2) != 0) {
            pw[0] = v4i{(int)round_off, l, gi, 4}, pw[1] = pw[0] + 1;
            return;
        }
        if constexpr (SPLIT) {  // this group's polynomial's row only
            pw[0] = ld_bsk(rsrc, voff, round_off + ((k * RW + 2 * l + pol) * 2 + j) * FN * 4);
            return;
        }
        pw[0] = ld_bsk(rsrc, voff, round_off + ((k * RW + 2 * l) * 2 + j) * FN * 4);
        pw[1] = ld_bsk(rsrc, voff, round_off + ((k * RW + 2 * l + 1) * 2 + j) * FN * 4);
    };
    // first: the round's first terms (s = 0 until now)
    auto mac = [&](int64_t (&s)[NCT][2][2][4], const int32_t (&X)[P][4], const v4i (&pw)[2], int gi, bool first) {
        const int k = gi >> 1, j = gi & 1;
        const int32_t w0[4] = {pw[0].x, pw[0].y, pw[0].z, pw[0].w};
        const int32_t w1[4] = {pw[1].x, pw[1].y, pw[1].z, pw[1].w};
#pragma unroll
        for (int q = 0; q < NCT; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                s[q][k][j][r] = first ? (int64_t)X[NPOL * q][r] * w0[r] : mac64(X[NPOL * q][r], w0[r], s[q][k][j][r]);
                if constexpr (!SPLIT) s[q][k][j][r] = mac64(X[2 * q + 1][r], w1[r], s[q][k][j][r]);
            }
    };

    v4i pw[4][2];  // key ring: the rows of the digit being consumed / about to be
    // FOLD: the C rows of round 0.  Otherwise digit 0's rows are issued at the start of each
    // round (not during the previous round's last products), so the ring is dead across the
    // monomial step and the inverse transform: fewer live registers (no spills in the loop).
    if constexpr (FOLD) {
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) issue(pw[gi], 0, TOP, gi);
    }

    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t round_off = i * ROWB;
        uint32_t ai[NCT];  // a'_i = ((amod - a_i) mod amod) * (2N / amod)  (rgsw-acc-cggi.cpp:153)
#pragma unroll
        for (int q = 0; q < NCT; ++q) {
            const uint32_t ct = wg_ct + q;
            const uint32_t ar = ct < B ? (uint32_t)(a[(size_t)ct * n + i] & amask) : 0;
            ai[q] = __builtin_amdgcn_readfirstlane(((amask + 1 - ar) & amask) << ashift);
        }
        int64_t s[NCT][2][2][4];
#pragma unroll
        for (int q = 0; q < NCT; ++q)
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) s[q][k][j][r] = 0;

        // the C digit (no transform); its groups' registers take digit 0's rows
        if constexpr (FOLD) {
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                __builtin_amdgcn_sched_barrier(0);
                mac(s, Cp, pw[gi], gi, true);
                issue(pw[gi], round_off, 0, gi);
            }
        } else {
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) issue(pw[gi], round_off, 0, gi);
        }
#pragma unroll
        for (uint32_t l = 0; l < NT; ++l) {
            // closed-form signed digit lt (thrown digits counted): sext_LOGG((c + K_lt) >> LOGG lt)
            const uint32_t lt = l + THR;
            const int32_t kl = (int32_t)(((1u << (LOGG * lt)) - 1) / ((1u << LOGG) - 1)) << (LOGG - 1);
            int32_t X[P][4];
            if constexpr (SPLIT) {
#pragma unroll
                for (int r = 0; r < 4; ++r) X[0][r] = __builtin_amdgcn_sbfe(acc[0][0][r] + kl, LOGG * lt, LOGG);
            } else {
#pragma unroll
                for (int q = 0; q < NCT; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        X[2 * q][r] = __builtin_amdgcn_sbfe(acc[q][0][r] + kl, LOGG * lt, LOGG);
                        X[2 * q + 1][r] = __builtin_amdgcn_sbfe(acc[q][NPOL - 1][r] + kl, LOGG * lt, LOGG);
                    }
            }
            __builtin_amdgcn_sched_barrier(0);
            constexpr int SM = LOGG > 7 ? 0 : (OPT & 4) ? 2 : (OPT & 1) ? 1 : 0;
            if (l & 1) ntt_fwd<XA1, P, EXP, SM, PRE, (OPT & 8) != 0>(X, lds, C, K);
            else ntt_fwd<XA0, P, EXP, SM, PRE, (OPT & 8) != 0>(X, lds, C, K);
            // next digit's rows (after the last, FOLD: the next round's C rows; the last round
            // re-fetches)
            const bool last = l + 1 == NT;
            const uint32_t noff = !last ? round_off : (i + 1 < n ? i + 1 : i) * ROWB;
            const int nl = !last ? (int)l + 1 : TOP;
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                __builtin_amdgcn_sched_barrier(0);
                mac(s, X, pw[gi], gi, !FOLD && l == 0);
                if (FOLD || !last) issue(pw[gi], noff, nl, gi);
            }
        }

        // S_j = A_0j * NTT(X^a' - 1) + A_1j * NTT(X^-a' - 1); rotated monomial table
        __builtin_amdgcn_sched_barrier(0);
        const char* mono = reinterpret_cast<const char*>(lds + L_MONO);
        int32_t S[P][4];
        if constexpr (SPLIT) {
            // partial sums of this polynomial's rows; the other column's go to the other group (LDS word
            // ((writer group * 2 + key) * 4 + r) * 256 + lane: conflict-free), this column's come back
            int32_t* xch = lds + L_CT + GR * (4 * P * LP + XB * P * XP);
            const uint32_t bp = (et * ai[0]) & 2047, bn = (0u - bp) & 2047;
            const uint32_t F4p = ((bp >> 4) & 0x1C) | ((bp & 63) << 7), F4n = ((bn >> 4) & 0x1C) | ((bn & 63) << 7);
            const uint32_t hp = (bp >> 4) & 0x60, hn = (bn >> 4) & 0x60;
            int32_t Am[2][4];
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    xch[((pol * 2 + k) * 4 + r) * TPC + tid] = sredc(pol ? s[0][k][0][r] : s[0][k][1][r], K);
                    Am[k][r] = sredc(pol ? s[0][k][1][r] : s[0][k][0][r], K);
                }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t c = ((r & 1) << 1) | (r >> 1);  // bitrev2(r)
                const uint32_t cs = c * 32 * ai[0];             // uniform
                const int32_t mp = *reinterpret_cast<const int32_t*>(mono + ((((hp + cs) & 0x60)) | F4p));
                const int32_t mn = *reinterpret_cast<const int32_t*>(mono + ((((hn - cs) & 0x60)) | F4n));
                const int32_t A0 = Am[0][r] + xch[(((1 - pol) * 2 + 0) * 4 + r) * TPC + tid];
                const int32_t A1 = Am[1][r] + xch[(((1 - pol) * 2 + 1) * 4 + r) * TPC + tid];
                S[0][r] = sredc((int64_t)A0 * mp + (int64_t)A1 * mn, K);
            }
        }
#pragma unroll
        for (int q = 0; q < (SPLIT ? 0 : NCT); ++q) {
            const uint32_t bp = (et * ai[q]) & 2047, bn = (0u - bp) & 2047;
            const uint32_t F4p = ((bp >> 4) & 0x1C) | ((bp & 63) << 7), F4n = ((bn >> 4) & 0x1C) | ((bn & 63) << 7);
            const uint32_t hp = (bp >> 4) & 0x60, hn = (bn >> 4) & 0x60;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t c = ((r & 1) << 1) | (r >> 1);  // bitrev2(r)
                const uint32_t cs = c * 32 * ai[q];             // uniform
                const int32_t mp = *reinterpret_cast<const int32_t*>(mono + ((((hp + cs) & 0x60)) | F4p));
                const int32_t mn = *reinterpret_cast<const int32_t*>(mono + ((((hn - cs) & 0x60)) | F4n));
                const int32_t A00 = sredc(s[q][0][0][r], K), A01 = sredc(s[q][0][1][r], K);
                const int32_t A10 = sredc(s[q][1][0][r], K), A11 = sredc(s[q][1][1][r], K);
                S[2 * q][r] = sredc((int64_t)A00 * mp + (int64_t)A10 * mn, K);
                S[2 * q + 1][r] = sredc((int64_t)A01 * mp + (int64_t)A11 * mn, K);
            }
        }
        // C <- C + S, reduced every 8 rounds
        if constexpr (FOLD) {
#pragma unroll
            for (int p = 0; p < P; ++p)
#pragma unroll
                for (int r = 0; r < 4; ++r) Cp[p][r] += S[p][r];
        }
        if (FOLD && (i & 7) == 7) {
#pragma unroll
            for (int p = 0; p < P; ++p)
#pragma unroll
                for (int r = 0; r < 4; ++r) Cp[p][r] = smul(Cp[p][r], K.rM, K);
        }
        __builtin_amdgcn_sched_barrier(0);
        ntt_inv<XA1, P, EXP, PRE>(S, lds, C, K);
#pragma unroll
        for (int q = 0; q < NCT; ++q)
#pragma unroll
            for (int p = 0; p < NPOL; ++p)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    uint32_t u = (uint32_t)(acc[q][p][r] + S[NPOL * q + p][r]) + K.kacc;  // in (0, 8Q)
                    if constexpr ((OPT & 2) != 0) {
                        // u - floor(u / Q) Q, off by at most one Q (u < 2^30): one mul_hi + one mad
                        const uint32_t qt = __umulhi(u, K.bm);
                        uint64_t t;
                        asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(t) : "v"(qt), "s"(K.nQ), "v"((uint64_t)u) : "vcc");
                        u = csub32((uint32_t)t, (uint32_t)K.Q);
                    } else {
                        u = csub32(csub32(csub32(u, K.Q4), K.Q2), (uint32_t)K.Q);
                    }
                    acc[q][p][r] = (int32_t)(u - K.h1);
                }
    }
#pragma unroll
    for (int q = 0; q < NCT; ++q) {
        const uint32_t ct = wg_ct + q;
        if (ct >= B) continue;
        uint64_t* g = acc_io + (size_t)ct * 2 * FN;
        // acc0 transposed (X -> X^-1, poly.cpp:762-770): out[(N-k) mod N] = -acc0[k]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t k = elem<1>(w, lane, r);
            const uint32_t v = (uint32_t)(acc[q][0][r] < 0 ? acc[q][0][r] + K.Q : acc[q][0][r]);
            if constexpr (SPLIT) {
                if (pol == 0) g[(FN - k) & (FN - 1)] = k == 0 ? v : (v == 0 ? 0 : (uint32_t)K.Q - v);
                else g[FN + k] = v;
            } else {
                const uint32_t v1 = (uint32_t)(acc[q][NPOL - 1][r] < 0 ? acc[q][NPOL - 1][r] + K.Q : acc[q][NPOL - 1][r]);
                g[(FN - k) & (FN - 1)] = k == 0 ? v : (v == 0 ? 0 : (uint32_t)K.Q - v);
                g[FN + k] = v1;
            }
        }
    }
    // FLAG (host-array EvalAcc, engine.hip d2h_flagged): done[4 ct + w] = 1 in pinned host memory once
    // wave w's accumulator words are in HBM -- its system-scope release waits for its stores and writes
    // the XCD's L2 back -- so the host can DMA finished ciphertexts while later workgroups still run.
    // A separate instantiation: the store after the loop changes the loop's register allocation (5
    // scratch loads per round, +43 instructions), so the device-resident path keeps FLAG = false.
    if constexpr (FLAG) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0)  // lane 0, not `lane`: kept live
            __hip_atomic_store(done + wg_ct * 4 + w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#ifndef TFHE_FAST4_KERNEL_ONLY  // blind_rotate_fast4_d6.hip includes the kernel template only
// generic psi / ipsi / mono tables (plain u32) -> the table block above (centred Montgomery)
__global__ void k_pack_tables4(uint32_t Q, const uint32_t* __restrict__ psi, const uint32_t* __restrict__ ipsi,
                               const uint32_t* __restrict__ mono, int32_t* __restrict__ out) {
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    auto mont = [Q](uint32_t v) {
        const uint32_t m = (uint32_t)(((uint64_t)v << 32) % Q);
        return m > Q / 2 ? (int32_t)m - (int32_t)Q : (int32_t)m;
    };
    if (idx < PF_END) {
        uint32_t m, base;
        if (idx < P1F) m = 1, base = P0F;
        else if (idx < P2F) m = 4, base = P1F;
        else if (idx < P3F) m = 16, base = P2F;
        else if (idx < P4F) m = 64, base = P3F;
        else m = 256, base = P4F;
        const uint32_t c = (idx - base) >> 2, e = (idx - base) & 3;
        const uint32_t k = e == 0 ? m + c : 2 * m + 2 * c + (e - 1);
        out[idx] = e == 3 ? 0 : mont(psi[k]);
        out[P0I + idx] = e == 3 ? 0 : mont(ipsi[k]);
    }
    if (idx < 2 * FN) out[T4_MONO + ((idx >> 6) | ((idx & 63) << 5))] = mont(mono[idx]);
    if (idx < 128) {  // pass 0 of a digit polynomial: d w mod Q, centred (plain: smul(d, mont(w)) = d w)
        const int32_t d = (int32_t)idx - 64;
        auto dmul = [Q, d](uint64_t w) {
            const uint32_t v = (uint32_t)((uint64_t)(uint32_t)(d < 0 ? -d : d) * (w % Q) % Q);
            const uint32_t m = d < 0 ? (v ? Q - v : 0) : v;
            return m > Q / 2 ? (int32_t)m - (int32_t)Q : (int32_t)m;
        };
        const uint64_t p21 = (uint64_t)psi[2] * psi[1] % Q, p31 = (uint64_t)psi[3] * psi[1] % Q;
        out[T4_T1 + idx] = dmul(psi[1]);
        out[T4_T23 + 2 * idx] = dmul(psi[2]), out[T4_T23 + 2 * idx + 1] = dmul(psi[3]);
        out[T4_T2131 + 2 * idx] = dmul(p21), out[T4_T2131 + 2 * idx + 1] = dmul(p31);
    }
}

#endif  // TFHE_FAST4_KERNEL_ONLY
}  // namespace f4
#ifndef TFHE_FAST4_KERNEL_ONLY

size_t fast4_table_words() { return f4::T4_WORDS; }

hipError_t launch_pack_tables_fast4(uint32_t Q, const DevTables& T, void* out, hipStream_t s) {
    hipLaunchKernelGGL(f4::k_pack_tables4, dim3((f4::T4_WORDS + 255) / 256), dim3(256), 0, s, Q,
                       (const uint32_t*)T.psi, (const uint32_t*)T.ipsi, (const uint32_t*)T.mono, (int32_t*)out);
    return hipGetLastError();
}

bool fast4_shape_supported(const Fast4Shape& sh) {
    return (sh.dig == 4 && sh.logg == 7 && sh.thr == 0 && sh.fold) ||   // STD128, STD128_OPT
           (sh.dig == 6 && sh.logg == 5 && sh.thr == 0 && sh.fold) ||   // logQ = 11, no thrown digit
           (sh.dig == 5 && sh.logg == 5 && sh.thr == 1 && !sh.fold) ||  // logQ = 11, one thrown digit
           (sh.dig == 3 && sh.logg == 9 && sh.thr == 0 && !sh.fold);    // STD128_AP (top digit wraps)
}

// blind_rotate_fast4_d6.hip: the logQ = 11 folded shape (6 digits of 5 bits), built with the default
// LLVM scheduler (29 % slower under iterative-ilp, profiles/r02bh)
hipError_t launch_blind_rotate_fast4_d6(const f4::FastConst& K, uint32_t n, uint32_t loga, const int32_t* tabs4,
                                        const int32_t* bsk, const uint64_t* a, uint64_t* acc, size_t B, hipStream_t s);

hipError_t launch_blind_rotate_fast4(int variant, const Fast4Shape& sh, const void* K, uint32_t n, uint32_t loga,
                                     const int32_t* tabs4, const int32_t* bsk, const uint64_t* a, uint64_t* acc,
                                     size_t B, hipStream_t s, BRDone* dn, int split_max) {
    const f4::FastConst Kc = *reinterpret_cast<const f4::FastConst*>(K);
    auto launch = [&](auto kern, int nct, int xb = 2, int cts = 1, uint32_t* done = nullptr) {
        const size_t lb = f4::lds_bytes(2 * nct, xb, cts);
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
        hipLaunchKernelGGL(kern, dim3((unsigned)((B + nct * cts - 1) / (nct * cts))), dim3(f4::TPC * cts), lb, s, Kc,
                           n, loga, tabs4, bsk, a, acc, (uint32_t)B, done);
    };
    // other digit shapes: the default build (variant 60's template arguments) at that shape
    if (sh.dig == 6 && sh.logg == 5 && sh.thr == 0 && sh.fold)  // own translation unit (Makefile)
        return launch_blind_rotate_fast4_d6(Kc, n, loga, tabs4, bsk, a, acc, B, s);
    if (sh.dig == 5 && sh.logg == 5 && sh.thr == 1 && !sh.fold) {
        launch(f4::k_blind_rotate_fast4<4, 1, 0, 7, 1, 1, 5, 5, 1, false>, 1, 1);
        return hipGetLastError();
    }
    if (sh.dig == 3 && sh.logg == 9 && sh.thr == 0 && !sh.fold) {
        launch(f4::k_blind_rotate_fast4<4, 1, 0, 7, 1, 1, 3, 9, 0, false>, 1, 1);
        return hipGetLastError();
    }
    if (!(sh.dig == 4 && sh.logg == 7 && sh.thr == 0 && sh.fold)) return hipErrorNotSupported;
    if (variant == 60 && B <= (size_t)split_max && !(dn && dn->flags)) {
        // small batches: one ciphertext per 512-thread workgroup, its two polynomials on two groups (SPLIT)
        auto kern = f4::k_blind_rotate_fast4<4, 1, 0, 7, 1, 1, 4, 7, 0, true, false, true>;
        const size_t lb = f4::lds_bytes(1, 1, 2) + (size_t)2 * 8 * f4::TPC * 4;  // + the partial-sum exchange
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
        hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(2 * f4::TPC), lb, s, Kc, n, loga, tabs4, bsk, a, acc, (uint32_t)B,
                           (uint32_t*)nullptr);
        return hipGetLastError();
    }
    if (dn && dn->flags && variant == 60) {  // the default build with completion flags (FLAG)
        launch(f4::k_blind_rotate_fast4<4, 1, 0, 7, 1, 1, 4, 7, 0, true, true>, 1, 1, 1, dn->flags);
        dn->written = true;
        return hipGetLastError();
    }
    switch (variant) {  // cross-check builds (blind_rotate_fast.hip known_variant)
        case 70: launch(f4::k_blind_rotate_fast4<2, 2>, 2); break;                    // two ciphertexts per wavefront
        case 86: launch(f4::k_blind_rotate_fast4<4, 1, 0, 7, 1, 4>, 1, 1, 4); break;  // four per workgroup
        default: launch(f4::k_blind_rotate_fast4<4, 1, 0, 7, 1>, 1, 1); break;  // = 60
    }
    return hipGetLastError();
}

#endif  // TFHE_FAST4_KERNEL_ONLY
}  // namespace tfhe
