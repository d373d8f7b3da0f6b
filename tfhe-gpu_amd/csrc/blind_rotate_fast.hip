// blind_rotate_fast.hip -- CGGI blind rotation specialised for the STD128 class
// (N = 1024, dG2 = 8, baseG = 2^7, Q < 2^27; STD128, STD128_OPT): the key/table packing
// shared by both specialised kernels, the two-wavefront kernel k_blind_rotate_fast2 and the
// launcher, which runs the four-wavefront kernel of blind_rotate_fast4.hip by default.  The
// four-wavefront kernel and the packing also take the other N = 1024, Q < 2^27 digit shapes
// fast4_shape_supported lists (logQ = 11 contexts, STD128_AP).
//
// Same math as the generic kernel and the oracle (rgsw-acc-cggi.cpp:246-307 and
// rgsw-acc.cpp:57-111), re-organised for gfx950 (k_blind_rotate_fast2's layout below;
// blind_rotate_fast4.hip describes its own):
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
#include <atomic>
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

// Table block (int32 words, centred Montgomery form).  Twiddles are packed per radix-8
// pass so that a lane fetches the 7 twiddles of its block with two ds_read_b128:
//   TW1  [lo 4][hi 4]           pass on (b9 b8 b7), one block
//   TW2  [lo 8][4] [hi 8][4]    pass on (b6 b5 b4), block c = i >> 7
//   TW3  [lo 64][4] [hi 64][4]  pass on (b3 b2 b1), block c = i >> 4
//   TW4  [128 lanes][4]         single stage on b0: psi[512 + (i >> 1)], in L4 lane order
// block c of a pass with stride m: lo = psi[m+c], psi[2m+2c], psi[2m+2c+1], psi[4m+4c],
// hi = psi[4m+4c+1 .. +3], 0.  Separate lo/hi arrays and the lane-ordered TW4 keep every
// 16-lane ds_read_b128 group on one 256-byte bank row (no conflicts).
// Forward (psi) and inverse (psi^-1) sets, then mono[2N] = psi^k - 1.
constexpr uint32_t TW1 = 0, TW2 = 8, TW3 = 72, TW4 = 584, TW_WORDS = 1096;
constexpr uint32_t T_FWD = 0, T_INV = TW_WORDS, T_MONO = 2 * TW_WORDS, T_WORDS = 2 * TW_WORDS + 2 * FN;
// Exchange buffers per ciphertext: two alternating buffers, each 2 regions (one per
// reading wavefront) x 2 polynomials x PS words.
// (NB = 1: one buffer and an extra barrier before each cross-wavefront store)
constexpr uint32_t PS = 576, WS = 2 * PS, XBUF = 2 * WS;
// the fast key buffer: [T_WORDS tables][4-wave kernel tables (blind_rotate_fast4.hip)][key rows]
constexpr uint32_t T4W = 5416, TB_WORDS = T_WORDS + T4W;

struct FastConst {
    int32_t Q, nQ, qinv, rM;  // rM = R mod Q (centred): smul(x, rM) reduces x
    uint32_t Q2, Q4, h1, kacc;  // 2Q, 4Q, (Q>>1)+1, (Q>>1)+1+4Q
    int32_t ninv;               // N^-1 (centred Montgomery form)
    uint32_t bm;                // floor(2^32 / Q) (blind_rotate_fast4.hip's Barrett update)
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

// ---- layouts and exchanges (model and proof: tools/lds_layouts.py) ----
// A layout names the index bit (b9..b0 of the natural index i) carried by each register
// bit (r = 0..7) and lane bit (lane = 0..127 of the ciphertext, bit 6 = wavefront):
//   L1 regs (b7 b8 b9)  lanes (b4 b5 b1 b2 b3 b0 | b6)   coefficient order, pass on b9 b8 b7
//   L2 regs (b4 b5 b6)  lanes (b1 b2 b3 b7 b8 b0 | b9)   pass on b6 b5 b4
//   L3 regs (b1 b2 b3)  lanes (b4 b5 b6 b7 b8 b0 | b9)   pass on b3 b2 b1
//   L4 regs (b0 b1 b2)  lanes (b4 b5 b6 b7 b8 b3 | b9)   stage on b0; MAC (8 consecutive slots)
// Only L1 <-> L2 crosses wavefronts.  An exchange A -> B stores each register of A as one
// lane-contiguous row (ds_write_addtid_b32: no address VGPR, 2 cycles) and B gathers with
// ds_read_b32 at F(lane) + G(register).  Rows are placed in the region of the wavefront
// that reads them, with strides chosen so every 32-lane read group hits 32 distinct banks.
struct Lay {
    int reg[3];
    int lane[7];
};
__host__ __device__ constexpr Lay lay(int L) {
    return L == 1   ? Lay{{7, 8, 9}, {4, 5, 1, 2, 3, 0, 6}}
           : L == 2 ? Lay{{4, 5, 6}, {1, 2, 3, 7, 8, 0, 9}}
           : L == 3 ? Lay{{1, 2, 3}, {4, 5, 6, 7, 8, 0, 9}}
                    : Lay{{0, 1, 2}, {4, 5, 6, 7, 8, 3, 9}};
}
__host__ __device__ constexpr int row_bit(int A, int B, int k) {
    return (A == 1 && B == 2)   ? (k == 0 ? 7 : k == 1 ? 8 : 6)
           : (A == 2 && B == 1) ? (k == 0 ? 4 : k == 1 ? 5 : 9)
                                : lay(A).reg[k];
}
__host__ __device__ constexpr int row_stride(int A, int B) { return (A == 2 && B == 1) ? 72 : 65; }
// words contributed to the LDS address by index bit b in exchange A -> B
__host__ __device__ constexpr int wt(int A, int B, int b) {
    if (b == lay(B).lane[6]) return (int)WS;
    for (int k = 0; k < 3; ++k)
        if (row_bit(A, B, k) == b) return row_stride(A, B) << k;
    for (int k = 0; k < 6; ++k)
        if (lay(A).lane[k] == b) return 1 << k;
    return 1 << 24;  // unreachable for the layouts above
}
__host__ __device__ constexpr int st_off(int A, int B, int r, int p) {  // bytes, writer register r
    int o = p * (int)PS;
    for (int k = 0; k < 3; ++k)
        if ((r >> k) & 1) o += wt(A, B, lay(A).reg[k]);
    return o * 4;
}
__host__ __device__ constexpr int ld_off(int A, int B, int r, int p) {  // bytes, reader register r
    int o = p * (int)PS;
    for (int k = 0; k < 3; ++k)
        if ((r >> k) & 1) o += wt(A, B, lay(B).reg[k]);
    return o * 4;
}
template <int A, int B>
__device__ __forceinline__ uint32_t ld_lane(uint32_t t) {  // bytes, reader lane t
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) o += ((t >> k) & 1) * (uint32_t)wt(A, B, lay(B).lane[k]);
    return o * 4;
}
template <int L>
__device__ __forceinline__ uint32_t elem(uint32_t t, uint32_t r) {  // natural index of (lane, register)
    uint32_t i = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) i |= ((r >> k) & 1) << lay(L).reg[k];
#pragma unroll
    for (int k = 0; k < 7; ++k) i |= ((t >> k) & 1) << lay(L).lane[k];
    return i;
}

// one polynomial's 8 registers as 8 lane-contiguous rows (M0 = this wavefront's base)
template <int A, int B, int P>
__device__ __forceinline__ void store_rows(const int32_t (&x)[8], uint32_t m0, const int32_t* lds) {
    asm volatile(
        "s_mov_b32 m0, %8\n\t"
        "s_nop 0\n\t"
        "ds_write_addtid_b32 %0 offset:%10\n\t"
        "ds_write_addtid_b32 %1 offset:%11\n\t"
        "ds_write_addtid_b32 %2 offset:%12\n\t"
        "ds_write_addtid_b32 %3 offset:%13\n\t"
        "ds_write_addtid_b32 %4 offset:%14\n\t"
        "ds_write_addtid_b32 %5 offset:%15\n\t"
        "ds_write_addtid_b32 %6 offset:%16\n\t"
        "ds_write_addtid_b32 %7 offset:%17" ::"v"(x[0]),
        "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]), "s"(m0), "s"(lds),
        "i"(st_off(A, B, 0, P)), "i"(st_off(A, B, 1, P)), "i"(st_off(A, B, 2, P)), "i"(st_off(A, B, 3, P)),
        "i"(st_off(A, B, 4, P)), "i"(st_off(A, B, 5, P)), "i"(st_off(A, B, 6, P)), "i"(st_off(A, B, 7, P))
        : "memory");
}

// LDS traffic of the transforms is issued from inline asm so that its completion can be
// awaited with counted waits (LDS operations complete in order): one polynomial's pass runs
// while the other one's rows are in flight.  The wait statements take the awaited
// registers as read-write operands, which orders every consumer after the wait.
//
// 8 single-dword gathers from one base address (16-bit immediates, one address VGPR)
template <int A, int B, int P>
__device__ __forceinline__ void gather_rows(int32_t (&x)[8], uint32_t base, const int32_t* lds) {
    asm volatile(
        "ds_read_b32 %0, %8 offset:%10\n\t"
        "ds_read_b32 %1, %8 offset:%11\n\t"
        "ds_read_b32 %2, %8 offset:%12\n\t"
        "ds_read_b32 %3, %8 offset:%13\n\t"
        "ds_read_b32 %4, %8 offset:%14\n\t"
        "ds_read_b32 %5, %8 offset:%15\n\t"
        "ds_read_b32 %6, %8 offset:%16\n\t"
        "ds_read_b32 %7, %8 offset:%17"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7])
        : "v"(base), "s"(lds), "i"(ld_off(A, B, 0, P)), "i"(ld_off(A, B, 1, P)), "i"(ld_off(A, B, 2, P)),
          "i"(ld_off(A, B, 3, P)), "i"(ld_off(A, B, 4, P)), "i"(ld_off(A, B, 5, P)), "i"(ld_off(A, B, 6, P)),
          "i"(ld_off(A, B, 7, P))
        : "memory");
}
// packed twiddles of one block: two ds_read_b128 (one for the single-stage pass)
template <uint32_t OFF, uint32_t NBLK>
__device__ __forceinline__ void tw_load(v4i& lo, v4i& hi, uint32_t addr, const int32_t* lds) {
    asm volatile("ds_read_b128 %0, %2 offset:%4\n\tds_read_b128 %1, %2 offset:%5"
                 : "=&v"(lo), "=&v"(hi)
                 : "v"(addr), "s"(lds), "i"(OFF), "i"(OFF + NBLK * 16)
                 : "memory");
}
template <uint32_t OFF>
__device__ __forceinline__ void tw_load(v4i& lo, uint32_t addr, const int32_t* lds) {
    asm volatile("ds_read_b128 %0, %1 offset:%3" : "=&v"(lo) : "v"(addr), "s"(lds), "i"(OFF) : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait(int32_t (&x)[8]) {
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
                 : "i"(N)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait(int32_t (&x)[8], v4i& lo, v4i& hi) {
    asm volatile("s_waitcnt lgkmcnt(%10)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                   "+v"(lo), "+v"(hi)
                 : "i"(N)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait(int32_t (&x)[8], v4i& lo) {
    asm volatile("s_waitcnt lgkmcnt(%9)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                   "+v"(lo)
                 : "i"(N)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait(v4i& lo, v4i& hi) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(lo), "+v"(hi) : "i"(N) : "memory");
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

// radix-8 CT pass over register bits (2, 1, 0); lo/hi = packed twiddles of the block
__device__ __forceinline__ void fwd_pass8(int32_t (&x)[8], v4i lo, v4i hi, const FastConst& K) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bfly_ct(x[r], x[r + 4], lo.x, K);
    bfly_ct(x[0], x[2], lo.y, K);
    bfly_ct(x[1], x[3], lo.y, K);
    bfly_ct(x[4], x[6], lo.z, K);
    bfly_ct(x[5], x[7], lo.z, K);
    bfly_ct(x[0], x[1], lo.w, K);
    bfly_ct(x[2], x[3], hi.x, K);
    bfly_ct(x[4], x[5], hi.y, K);
    bfly_ct(x[6], x[7], hi.z, K);
}
__device__ __forceinline__ void fwd_pass1(int32_t (&x)[8], v4i w, const FastConst& K) {
    bfly_ct(x[0], x[1], w.x, K);
    bfly_ct(x[2], x[3], w.y, K);
    bfly_ct(x[4], x[5], w.z, K);
    bfly_ct(x[6], x[7], w.w, K);
}
// Inverse radix-8 pass.  With inputs < B the doubling a-paths reach 4B after two
// stages; x[0] and x[4] (the only ones) are reduced there, so the outputs stay < 3Q
// for any B <= 3Q (tools/bounds_fast.py).
__device__ __forceinline__ void inv_pass8(int32_t (&x)[8], v4i lo, v4i hi, const FastConst& K) {
    bfly_gs(x[0], x[1], lo.w, K);
    bfly_gs(x[2], x[3], hi.x, K);
    bfly_gs(x[4], x[5], hi.y, K);
    bfly_gs(x[6], x[7], hi.z, K);
    bfly_gs<true>(x[0], x[2], lo.y, K);
    bfly_gs(x[1], x[3], lo.y, K);
    bfly_gs<true>(x[4], x[6], lo.z, K);
    bfly_gs(x[5], x[7], lo.z, K);
#pragma unroll
    for (int r = 0; r < 4; ++r) bfly_gs(x[r], x[r + 4], lo.x, K);
}
__device__ __forceinline__ void inv_pass1(int32_t (&x)[8], v4i w, const FastConst& K) {
    bfly_gs(x[0], x[1], w.x, K);
    bfly_gs(x[2], x[3], w.y, K);
    bfly_gs(x[4], x[5], w.z, K);
    bfly_gs(x[6], x[7], w.w, K);
}

// per-lane constants of the transforms
struct LaneCtx {
    uint32_t w;                               // wavefront of the ciphertext (uniform)
    uint32_t f12, f23, f34, f43, f32, f21;    // gather offsets (bytes)
    uint32_t a2, a3, a4;                      // twiddle block offsets (bytes)
    uint32_t zero;                            // 0, as an address VGPR
};

// Forward transform of two polynomials, L1 -> L4; sbuf = the ciphertext's current
// exchange buffer (bytes).  The two polynomials are staggered: while one polynomial's
// rows travel through LDS, the other one's radix-8 pass runs.  Wait counts are the LDS
// operations issued after the awaited ones (15 = the counter's maximum, at most one
// operation stricter than needed).
// BAR bit 0: barrier before the cross-wavefront stores (NB = 1), bit 1: after them
// (timing experiments clear them; results are then invalid)
template <int NB, int BAR = 3>
__device__ __forceinline__ void ntt_fwd2(int32_t (&x0)[8], int32_t (&x1)[8], const int32_t* lds, uint32_t sbuf,
                                         const LaneCtx& C, const FastConst& K) {
    constexpr uint32_t T = T_FWD * 4;
    const uint32_t m12 = sbuf + C.w * (uint32_t)(wt(1, 2, 6) * 4);  // uniform
    const uint32_t mloc = sbuf + C.w * WS * 4;                      // uniform: own region
    v4i lo, hi;
    tw_load<T + TW1 * 4, 1>(lo, hi, C.zero, lds);
    lds_wait<0>(lo, hi);
    fwd_pass8(x0, lo, hi, K);
    if constexpr (NB == 1) {  // the other wavefront has finished reading this buffer
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (BAR & 1) __syncthreads();
    }
    store_rows<1, 2, 0>(x0, m12, lds);
    fwd_pass8(x1, lo, hi, K);
    store_rows<1, 2, 1>(x1, m12, lds);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (BAR & 2) __syncthreads();
    tw_load<T + TW2 * 4, 8>(lo, hi, C.a2, lds);
    gather_rows<1, 2, 0>(x0, sbuf + C.f12, lds);
    gather_rows<1, 2, 1>(x1, sbuf + C.f12, lds);
    lds_wait<8>(x0, lo, hi);
    fwd_pass8(x0, lo, hi, K);
    store_rows<2, 3, 0>(x0, mloc, lds);
    gather_rows<2, 3, 0>(x0, sbuf + C.f23, lds);
    lds_wait<15>(x1);
    fwd_pass8(x1, lo, hi, K);
    tw_load<T + TW3 * 4, 64>(lo, hi, C.a3, lds);
    store_rows<2, 3, 1>(x1, mloc, lds);
    gather_rows<2, 3, 1>(x1, sbuf + C.f23, lds);
    lds_wait<15>(x0, lo, hi);
    fwd_pass8(x0, lo, hi, K);
    store_rows<3, 4, 0>(x0, mloc, lds);
    gather_rows<3, 4, 0>(x0, sbuf + C.f34, lds);
    lds_wait<15>(x1);
    fwd_pass8(x1, lo, hi, K);
    tw_load<T + TW4 * 4>(lo, C.a4, lds);
    store_rows<3, 4, 1>(x1, mloc, lds);
    gather_rows<3, 4, 1>(x1, sbuf + C.f34, lds);
    lds_wait<15>(x0, lo);
    fwd_pass1(x0, lo, K);
    lds_wait<0>(x1);
    fwd_pass1(x1, lo, K);
}

// Inverse transform of two polynomials (no N^-1: folded into the BSK), L4 -> L1.
// sloc = buffer of the last forward exchange (wave-local steps), sx = the other buffer.
template <int NB, int BAR = 3>
__device__ __forceinline__ void ntt_inv2(int32_t (&x0)[8], int32_t (&x1)[8], const int32_t* lds, uint32_t sloc,
                                         uint32_t sx, const LaneCtx& C, const FastConst& K) {
    constexpr uint32_t T = T_INV * 4;
    const uint32_t mloc = sloc + C.w * WS * 4;
    const uint32_t m21 = sx + C.w * (uint32_t)(wt(2, 1, 9) * 4);
    v4i lo, hi;
    tw_load<T + TW4 * 4>(lo, C.a4, lds);
    lds_wait<0>(x0, lo);
    inv_pass1(x0, lo, K);
    store_rows<4, 3, 0>(x0, mloc, lds);
    gather_rows<4, 3, 0>(x0, sloc + C.f43, lds);
    inv_pass1(x1, lo, K);
    tw_load<T + TW3 * 4, 64>(lo, hi, C.a3, lds);
    store_rows<4, 3, 1>(x1, mloc, lds);
    gather_rows<4, 3, 1>(x1, sloc + C.f43, lds);
    lds_wait<15>(x0, lo, hi);
    inv_pass8(x0, lo, hi, K);
    store_rows<3, 2, 0>(x0, mloc, lds);
    gather_rows<3, 2, 0>(x0, sloc + C.f32, lds);
    lds_wait<15>(x1);
    inv_pass8(x1, lo, hi, K);
    tw_load<T + TW2 * 4, 8>(lo, hi, C.a2, lds);
    store_rows<3, 2, 1>(x1, mloc, lds);
    gather_rows<3, 2, 1>(x1, sloc + C.f32, lds);
    lds_wait<15>(x0, lo, hi);
    inv_pass8(x0, lo, hi, K);
    if constexpr (NB == 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (BAR & 1) __syncthreads();
    }
    store_rows<2, 1, 0>(x0, m21, lds);
    lds_wait<0>(x1);
    inv_pass8(x1, lo, hi, K);
    store_rows<2, 1, 1>(x1, m21, lds);
    tw_load<T + TW1 * 4, 1>(lo, hi, C.zero, lds);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (BAR & 2) __syncthreads();
    gather_rows<2, 1, 0>(x0, sx + C.f21, lds);
    gather_rows<2, 1, 1>(x1, sx + C.f21, lds);
    lds_wait<8>(x0, lo, hi);
    inv_pass8(x0, lo, hi, K);
    lds_wait<0>(x1);
    inv_pass8(x1, lo, hi, K);
}

// ---------------------------------------------------------------------------
// k_blind_rotate_fast2: the same round with one digit's transforms eliminated.
//
// The signed digits satisfy c = d_0 + 2^7 d_1 + 2^14 d_2 + 2^21 d_3 exactly (rgsw-acc.cpp:83-109
// with thr = 0: the top digit is the remainder, |d_3| <= 33), so in the NTT domain
//     D_3 = 2^-21 (NTT(c) - D_0 - 2^7 D_1 - 2^14 D_2)            (mod Q).
// Substituting into the external product, for key k, column j, polynomial p:
//     sum_l D_{p,l} W[2l+p]  =  sum_{l<3} D_{p,l} (W[2l+p] - 2^(7l-21) W[6+p])  +  C_p 2^-21 N W[6+p]
// with C_p = N^-1 NTT(c_p).  k_pack_fast folds both into the key rows (same BSK size), and
// the kernel keeps C (the accumulator in the NTT domain) next to its coefficient form:
// C <- C + S each round, where S is the round's NTT-domain increment (the BSK carries N^-1).
// Six forward transforms per round instead of eight; the product mod Q is unchanged, so the
// output is bit-identical to the eight-transform round.
//
// C lives in LDS (2 polynomials x 2 halves x 128 lanes x 16 bytes per ciphertext, conflict-
// free ds_read/write_b128) and is reduced every 8 rounds (|C| < 5.2Q, tools/bounds_fast.py).
// The round starts with the C "digit" (no transform), whose key rows were fetched during the
// previous round's inverse transform (PFA groups, when the row sums are dead).
//
// MROT: monomial table stored at f(e) = (e >> 6) | ((e & 63) << 5), so the lanes of a gather
// spread over banks by e's top bits (the plain table is 32-way conflicted when 32 | a').
// With b = e_t a' mod 2N and e = b + 256 c a', f(e)*4 = (((b >> 4) & 0x70) + 16 c a') & 0x70 | F(b).
constexpr uint32_t CW = 2 * FN;  // words of C per ciphertext
constexpr size_t lds_bytes2(int cts, int nb) { return (size_t)(T_WORDS + cts * (nb * XBUF + CW)) * 4; }

// NB = 2: forward transform l uses exchange buffer l & 1, the inverse keeps the last forward
// buffer for its wave-local steps and the other for its cross-wavefront step (no barrier
// before the cross-wavefront stores; 2 x 9 KiB more LDS per ciphertext).
// DEPTH = 1: a digit's non-prefetched key groups are issued one group ahead of their MAC.
// EXP (timing experiments, results invalid): 1 no pre-store barriers, 2 no barriers in the
// transforms, 3 no key loads, 4 = 2 + 3.
template <int MINW, int PF, int PFA, bool MROT, int NB = 1, int DEPTH = 0, int EXP = 0>
__global__ void __launch_bounds__(TPC * 2, MINW)
k_blind_rotate_fast2(FastConst K, uint32_t n, uint32_t loga, const int32_t* __restrict__ tabs,
                     const int32_t* __restrict__ bsk, const uint64_t* __restrict__ a, uint64_t* __restrict__ acc_io,
                     uint32_t B) {
    constexpr int CTS = 2;
    extern __shared__ __align__(16) int32_t lds[];
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < T_WORDS; k += TPC * CTS) lds[k] = tabs[k];
    const uint32_t cl = __builtin_amdgcn_readfirstlane(tid / TPC), t = tid % TPC;
    const uint32_t ct = blockIdx.x * CTS + cl;
    const bool active = ct < B;
    const uint32_t sbuf = (T_WORDS + cl * NB * XBUF) * 4;  // exchange buffer(s) (bytes, uniform)
    constexpr uint32_t XB = NB == 2 ? XBUF * 4 : 0;        // bytes to the second buffer
    v4i* cv = reinterpret_cast<v4i*>(lds + T_WORDS + CTS * NB * XBUF + cl * CW) + t;  // C: cv[(2p + h) * 128]

    LaneCtx C;
    C.w = __builtin_amdgcn_readfirstlane(t >> 6);
    C.f12 = ld_lane<1, 2>(t), C.f23 = ld_lane<2, 3>(t), C.f34 = ld_lane<3, 4>(t);
    C.f43 = ld_lane<4, 3>(t), C.f32 = ld_lane<3, 2>(t), C.f21 = ld_lane<2, 1>(t);
    const uint32_t w6 = t >> 6;
    C.a2 = ((((t >> 3) & 3) | (w6 << 2)) * 16);
    C.a3 = (((t & 31) | (w6 << 5)) * 16);
    const uint32_t nslot = ((t >> 5) & 1) | ((t & 31) << 1) | (w6 << 6);
    C.a4 = t * 16;
    C.zero = 0;

    uint64_t* g = acc_io + (size_t)(active ? ct : 0) * 2 * FN;
    const uint32_t Qh = (uint32_t)K.Q >> 1;
    int32_t acc[2][8];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint64_t v0 = active ? g[p * FN + elem<1>(t, r)] : 0;
            const uint32_t v = (uint32_t)(v0 >= (uint64_t)K.Q ? v0 % (uint64_t)K.Q : v0);
            acc[p][r] = v < Qh ? (int32_t)v : (int32_t)v - K.Q;
        }
    __syncthreads();

    // C = N^-1 NTT(acc), in the MAC layout
    {
        int32_t x0[8], x1[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) x0[r] = acc[0][r], x1[r] = acc[1][r];
        ntt_fwd2<NB>(x0, x1, lds, sbuf + XB, C, K);
#pragma unroll
        for (int r = 0; r < 8; ++r) x0[r] = smul(x0[r], K.ninv, K), x1[r] = smul(x1[r], K.ninv, K);
        cv[0] = v4i{x0[0], x0[1], x0[2], x0[3]};
        cv[128] = v4i{x0[4], x0[5], x0[6], x0[7]};
        cv[256] = v4i{x1[0], x1[1], x1[2], x1[3]};
        cv[384] = v4i{x1[4], x1[5], x1[6], x1[7]};
    }

    constexpr uint32_t ROWB = 2 * FDG2 * 2 * FN * 4;  // key bytes per round
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(bsk), 0, (int)(n * ROWB), 0x00020000);
    const uint32_t voff = nslot * 32;
    const uint32_t et = 2 * (__builtin_bitreverse32(nslot) >> 25) + 1;
    const uint64_t* ap = a + (size_t)(active ? ct : 0) * n;
    const uint32_t amask = (1u << loga) - 1, ashift = 11 - loga;

    // rows 2l (poly 0) and 2l+1 (poly 1) of group g = (key k, column j); l = 3: the C rows
    auto issue = [&](v4i (&pw)[4], uint32_t round_off, int l, int gi) {
        const int k = gi >> 1, j = gi & 1;
        const uint32_t s0 = round_off + ((k * FDG2 + 2 * l) * 2 + j) * FN * 4;
        const uint32_t s1 = round_off + ((k * FDG2 + 2 * l + 1) * 2 + j) * FN * 4;
        if constexpr (EXP >= 3) {
            pw[0] = v4i{(int)s0, (int)s1, 3, 4}, pw[1] = pw[0] + 1, pw[2] = pw[0] + 2, pw[3] = pw[0] + 3;
        } else {
            pw[0] = ld_bsk(rsrc, voff, s0), pw[1] = ld_bsk(rsrc, voff + 16, s0);
            pw[2] = ld_bsk(rsrc, voff, s1), pw[3] = ld_bsk(rsrc, voff + 16, s1);
        }
    };
    constexpr int XBAR = EXP == 1 ? 2 : (EXP == 2 || EXP == 4) ? 0 : 3;
    auto mac = [&](int64_t (&s)[2][2][8], const int32_t (&x0)[8], const int32_t (&x1)[8], const v4i (&pw)[4],
                   int gi) {
        const int k = gi >> 1, j = gi & 1;
        const int32_t w0[8] = {pw[0].x, pw[0].y, pw[0].z, pw[0].w, pw[1].x, pw[1].y, pw[1].z, pw[1].w};
        const int32_t w1[8] = {pw[2].x, pw[2].y, pw[2].z, pw[2].w, pw[3].x, pw[3].y, pw[3].z, pw[3].w};
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            s[k][j][r] = (int64_t)x0[r] * w0[r] + s[k][j][r];
            s[k][j][r] = (int64_t)x1[r] * w1[r] + s[k][j][r];
        }
    };

    v4i pa[4][4];  // C rows of the current round
#pragma unroll
    for (int gi = 0; gi < PFA; ++gi) issue(pa[gi], 0, 3, gi);

    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t ar = active ? (uint32_t)(ap[i] & amask) : 0;
        const uint32_t ai = ((amask + 1 - ar) & amask) << ashift;
        const uint32_t round_off = i * ROWB;

        int64_t s[2][2][8];
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 8; ++r) s[k][j][r] = 0;

        // the C "digit": no transform
        {
            const v4i c00 = cv[0], c01 = cv[128], c10 = cv[256], c11 = cv[384];
            const int32_t x0[8] = {c00.x, c00.y, c00.z, c00.w, c01.x, c01.y, c01.z, c01.w};
            const int32_t x1[8] = {c10.x, c10.y, c10.z, c10.w, c11.x, c11.y, c11.z, c11.w};
            if (DEPTH && PFA == 0) issue(pa[0], round_off, 3, 0);
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                __builtin_amdgcn_sched_barrier(0);
                const int q = gi + DEPTH;
                if (q < 4 && q >= PFA) issue(pa[q], round_off, 3, q);
                mac(s, x0, x1, pa[gi], gi);
            }
        }
#pragma unroll
        for (uint32_t l = 0; l < FDIG - 1; ++l) {
            const int32_t kl = (int32_t)(((1u << (FLOGG * l)) - 1) / ((1u << FLOGG) - 1)) << (FLOGG - 1);
            int32_t x0[8], x1[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                x0[r] = __builtin_amdgcn_sbfe(acc[0][r] + kl, FLOGG * l, FLOGG);
                x1[r] = __builtin_amdgcn_sbfe(acc[1][r] + kl, FLOGG * l, FLOGG);
            }
            v4i pw[4][4];
#pragma unroll
            for (int gi = 0; gi < PF; ++gi) issue(pw[gi], round_off, l, gi);
            __builtin_amdgcn_sched_barrier(0);
            ntt_fwd2<NB, XBAR>(x0, x1, lds, sbuf + (l & 1) * XB, C, K);
            if (DEPTH && PF == 0) issue(pw[0], round_off, l, 0);
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                __builtin_amdgcn_sched_barrier(0);
                const int q = gi + DEPTH;
                if (q < 4 && q >= PF) issue(pw[q], round_off, l, q);
                mac(s, x0, x1, pw[gi], gi);
            }
        }

        // S_j = A_0j * NTT(X^a' - 1) + A_1j * NTT(X^-a' - 1)
        const char* mono = reinterpret_cast<const char*>(lds + T_MONO);
        int32_t S0[8], S1[8];
        uint32_t bp, bn, F4p, F4n;
        if constexpr (MROT) {
            bp = (et * ai) & 2047;
            bn = (0u - bp) & 2047;
            F4p = ((bp >> 4) & 0xC) | ((bp & 63) << 7);
            F4n = ((bn >> 4) & 0xC) | ((bn & 63) << 7);
            bp = (bp >> 4) & 0x70;
            bn = (bn >> 4) & 0x70;
        } else {
            bp = (et * ai) << 2;  // byte offsets into the 2N-entry table
        }
        const uint32_t st4 = (ai << 10) & 8191;  // 256 * ai * 4 mod 8192
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t c = __builtin_bitreverse32((uint32_t)r) >> 29;
            uint32_t op, on;
            if constexpr (MROT) {
                const uint32_t cs = c * 16 * ai;  // uniform
                op = ((bp + cs) & 0x70) | F4p;
                on = ((bn - cs) & 0x70) | F4n;
            } else {
                const uint32_t e4 = bp + c * st4;
                op = e4 & 8188;
                on = (0u - e4) & 8188;
            }
            const int32_t mp = *reinterpret_cast<const int32_t*>(mono + op);
            const int32_t mn = *reinterpret_cast<const int32_t*>(mono + on);
            const int32_t A00 = sredc(s[0][0][r], K), A01 = sredc(s[0][1][r], K);
            const int32_t A10 = sredc(s[1][0][r], K), A11 = sredc(s[1][1][r], K);
            S0[r] = sredc((int64_t)A00 * mp + (int64_t)A10 * mn, K);
            S1[r] = sredc((int64_t)A01 * mp + (int64_t)A11 * mn, K);
        }
        // C <- C + S, reduced every 8 rounds
        __builtin_amdgcn_sched_barrier(0);
        {
            const v4i c00 = cv[0], c01 = cv[128], c10 = cv[256], c11 = cv[384];
            int32_t y0[8] = {c00.x, c00.y, c00.z, c00.w, c01.x, c01.y, c01.z, c01.w};
            int32_t y1[8] = {c10.x, c10.y, c10.z, c10.w, c11.x, c11.y, c11.z, c11.w};
#pragma unroll
            for (int r = 0; r < 8; ++r) y0[r] += S0[r], y1[r] += S1[r];
            if ((i & 7) == 7) {
#pragma unroll
                for (int r = 0; r < 8; ++r) y0[r] = smul(y0[r], K.rM, K), y1[r] = smul(y1[r], K.rM, K);
            }
            cv[0] = v4i{y0[0], y0[1], y0[2], y0[3]};
            cv[128] = v4i{y0[4], y0[5], y0[6], y0[7]};
            cv[256] = v4i{y1[0], y1[1], y1[2], y1[3]};
            cv[384] = v4i{y1[4], y1[5], y1[6], y1[7]};
        }
        // next round's C rows (the last round re-fetches its own: no loads past the key)
        const uint32_t next_off = (i + 1 < n ? i + 1 : i) * ROWB;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int gi = 0; gi < PFA; ++gi) issue(pa[gi], next_off, 3, gi);
        __builtin_amdgcn_sched_barrier(0);
        ntt_inv2<NB, XBAR>(S0, S1, lds, sbuf, sbuf + XB, C, K);  // last forward used buffer 0
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
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t k = elem<1>(t, r);
            const uint32_t v = (uint32_t)(acc[0][r] < 0 ? acc[0][r] + K.Q : acc[0][r]);
            const uint32_t v1 = (uint32_t)(acc[1][r] < 0 ? acc[1][r] + K.Q : acc[1][r]);
            g[(FN - k) & (FN - 1)] = k == 0 ? v : (v == 0 ? 0 : (uint32_t)K.Q - v);
            g[FN + k] = v1;
        }
    }
}

// generic (plain, N^-1-scaled) BSK and tables -> centred Montgomery copies: key rows with the
// top digit folded in when M.fold (hc[l] = G^(l - top), hc[top] = N G^-top mod Q; STD128:
// 2^(7l-21) and N 2^-21, see k_blind_rotate_fast2), else plain; twiddles packed per pass
// (table-block comment above), monomials in the rotated layout.
struct PackMode {
    uint32_t hc[8];
    uint32_t rw;    // key rows per (key, column) = dG2
    uint32_t fold;  // top digit eliminated
};
__global__ void k_pack_fast(uint32_t Q, const uint32_t* __restrict__ bsk, size_t words, const uint32_t* __restrict__ psi,
                            const uint32_t* __restrict__ ipsi, const uint32_t* __restrict__ mono,
                            int32_t* __restrict__ out, PackMode M) {
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto mont = [Q](uint32_t v) {
        const uint32_t m = (uint32_t)(((uint64_t)v << 32) % Q);
        return m > Q / 2 ? (int32_t)m - (int32_t)Q : (int32_t)m;
    };
    if (idx < words) {
        // idx = (((i * 2 + k) * rw + row) * 2 + j) * N + slot; row = 2l + p
        const uint32_t row = (uint32_t)((idx / (2 * FN)) % M.rw), l = row >> 1, p = row & 1, top = M.rw / 2 - 1;
        uint32_t v = bsk[idx] % Q;
        if (M.fold) {
            const size_t it = idx + ((size_t)(2 * top + p) - row) * 2 * FN;  // row 2 top + p, same k, j, slot
            const uint64_t wt = (uint64_t)(bsk[it] % Q) * M.hc[l] % Q;
            v = l < top ? (uint32_t)(((uint64_t)v + Q - wt) % Q) : (uint32_t)wt;
        }
        out[TB_WORDS + idx] = mont(v);
    }
    if (idx < TW_WORDS) {
        // which packed entry is idx?  e = position within the block (0..3 lo, 4..7 hi)
        uint32_t k = 0;
        bool zero = false;
        if (idx < TW4) {
            uint32_t m, nblk, j;
            if (idx < TW2) m = 1, nblk = 1, j = idx;
            else if (idx < TW3) m = 8, nblk = 8, j = idx - TW2;
            else m = 64, nblk = 64, j = idx - TW3;
            const uint32_t hi = j >= 4 * nblk, c = (j % (4 * nblk)) >> 2, e = (hi ? 4 : 0) + (j & 3);
            zero = e == 7;
            k = e == 0 ? m + c : e < 3 ? 2 * m + 2 * c + (e - 1) : 4 * m + 4 * c + (e - 3);
        } else {
            const uint32_t j = idx - TW4, t = j >> 2, q = j & 3;
            const uint32_t nslot = ((t >> 5) & 1) | ((t & 31) << 1) | ((t >> 6) << 6);
            k = 512 + 4 * nslot + q;
        }
        out[T_FWD + idx] = zero ? 0 : mont(psi[k]);
        out[T_INV + idx] = zero ? 0 : mont(ipsi[k]);
    }
    if (idx < 2 * FN) {
        const uint32_t e = (uint32_t)idx;
        out[T_MONO + ((e >> 6) | ((e & 63) << 5))] = mont(mono[idx]);
    }
}

}  // namespace

// The digit shape of P for the 4-wavefront kernel; fold when no digit is thrown and the top
// digit of every centred coefficient c in [-(Q>>1)-1, Q>>1) stays in [-G/2, G/2) (no wrap), so
// that c = sum_l d_l G^l exactly (DESIGN.md 3.1 idea 1).
static Fast4Shape fast_shape(const BRParams& P) {
    Fast4Shape sh{(int)P.digits, (int)P.logG, (int)P.thr, false};
    if (P.thr == 0 && P.digits >= 2 && P.logG >= 1 && P.logG * P.digits <= 40) {
        const int64_t G = (int64_t)1 << P.logG, Qh = (int64_t)(P.Q >> 1);
        const uint32_t top = P.digits - 1;
        int64_t K = 0;
        for (uint32_t z = 0; z < top; ++z) K = K * G + G / 2;  // (G/2)(G^top - 1)/(G - 1)
        const int64_t lo = (-Qh - 1 + K) >> (P.logG * top), hi = (Qh - 1 + K) >> (P.logG * top);
        sh.fold = lo >= -G / 2 && hi < G / 2;
    }
    return sh;
}

bool fast_path_supported(const BRParams& P, int word_bits) {
    return word_bits == 32 && P.N == FN && P.dG2 == 2 * P.digits && P.Q < (1ull << 27) && P.n > 0 &&
           fast4_shape_supported(fast_shape(P));
}

size_t bsk_fast_bytes(const BRParams& P) { return ((size_t)P.n * 2 * P.dG2 * 2 * FN + TB_WORDS) * 4; }

namespace {
// TFHE_FAST_VARIANT selects the kernel build (A/B experiments): 30-58 k_blind_rotate_fast2
// (two wavefronts per ciphertext), >= 59 k_blind_rotate_fast4 (blind_rotate_fast4.hip; 60 =
// default).  The variant table is in DESIGN.md 3.1.  Timing-only builds (no barriers / no key
// loads / no transforms: results invalid) are taken only with TFHE_TIMING_EXPERIMENTS=1.
constexpr int kDefaultVariant = 60;
// builds the launchers know (blind_rotate_fast4.hip's list for >= 59); timing-only ones excluded
bool known_variant(int v) {
    static const int k[] = {34, 39, 40, 59, 60, 70, 76, 81, 83, 84, 85, 86, 87, 88};
    for (int x : k)
        if (x == v) return true;
    return false;
}
std::atomic<int> g_variant{-1};
int fast_variant() {
    int v = g_variant.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = std::getenv("TFHE_FAST_VARIANT");
        v = e && e[0] ? std::atoi(e) : kDefaultVariant;
        // timing-only builds (results invalid) need an explicit opt-in
        const char* x = std::getenv("TFHE_TIMING_EXPERIMENTS");
        if (!known_variant(v) && !(x && x[0] == '1')) v = kDefaultVariant;
        g_variant.store(v, std::memory_order_relaxed);
    }
    return v;
}
uint64_t powmod(uint64_t b, uint64_t e, uint64_t m) {
    uint64_t r = 1 % m;
    for (b %= m; e; e >>= 1, b = (unsigned __int128)b * b % m)
        if (e & 1) r = (unsigned __int128)r * b % m;
    return r;
}
int32_t mont_centred(uint64_t v, uint32_t Q) {
    const uint32_t m = (uint32_t)(((unsigned __int128)(v % Q) << 32) % Q);
    return m > Q / 2 ? (int32_t)m - (int32_t)Q : (int32_t)m;
}
}  // namespace

bool set_fast_variant(int v) {
    if (v == 0) v = kDefaultVariant;
    if (!known_variant(v)) return false;
    g_variant.store(v, std::memory_order_relaxed);
    return true;
}
int get_fast_variant() { return fast_variant(); }

hipError_t launch_pack_bsk_fast(const BRParams& P, const DevTables& T, const void* bsk, void* bsk_fast,
                                hipStream_t s) {
    const size_t words = (size_t)P.n * 2 * P.dG2 * 2 * FN;
    const Fast4Shape sh = fast_shape(P);
    if (P.dG2 > 16 || !fast4_shape_supported(sh)) return hipErrorNotSupported;
    PackMode M{};
    M.rw = P.dG2;
    M.fold = sh.fold;
    const uint32_t top = P.digits - 1;
    const uint64_t Q = P.Q, igt = powmod(2, Q - 1 - (uint64_t)P.logG * top, Q);  // G^-top (Q prime)
    for (uint32_t l = 0; l < top; ++l) M.hc[l] = (uint32_t)((unsigned __int128)powmod(2, (uint64_t)P.logG * l, Q) * igt % Q);
    M.hc[top] = (uint32_t)((unsigned __int128)FN * igt % Q);
    hipLaunchKernelGGL(k_pack_fast, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, (uint32_t)P.Q,
                       (const uint32_t*)bsk, words, (const uint32_t*)T.psi, (const uint32_t*)T.ipsi,
                       (const uint32_t*)T.mono, (int32_t*)bsk_fast, M);
    if (fast4_table_words() != T4W) return hipErrorInvalidValue;
    return launch_pack_tables_fast4((uint32_t)P.Q, T, (int32_t*)bsk_fast + T_WORDS, s);
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
    K.ninv = mont_centred(Q - (Q - 1) / FN, Q);  // N (Q-1)/N = -1 mod Q
    K.bm = (uint32_t)((1ull << 32) / Q);
    const int32_t* tabs = (const int32_t*)bsk_fast;
    const int32_t* bsk = tabs + TB_WORDS;
    const int variant = fast_variant();
    const Fast4Shape sh = fast_shape(P);
    const bool std128 = sh.dig == (int)FDIG && sh.logg == (int)FLOGG && sh.thr == 0 && sh.fold;
    if (variant >= 59 || !std128)  // the two-wavefront builds know only the STD128 shape
        return launch_blind_rotate_fast4(variant, sh, &K, P.n, loga, tabs + T_WORDS, bsk, a, acc, B, s);
    auto launch2 = [&](auto kern, int nb = 1) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes2(2, nb));
        hipLaunchKernelGGL(kern, dim3((unsigned)((B + 1) / 2)), dim3(TPC * 2), lds_bytes2(2, nb), s, K, P.n, loga,
                           tabs, bsk, a, acc, (uint32_t)B);
    };
    switch (variant) {
        // k_blind_rotate_fast2 <MINW, PF, PFA, MROT, NB, DEPTH, EXP>
        case 34: launch2(k_blind_rotate_fast2<3, 1, 4, true>); break;
        case 40: launch2(k_blind_rotate_fast2<2, 4, 4, true, 2>, 2); break;
        case 51: launch2(k_blind_rotate_fast2<3, 1, 2, true, 1, 1, 1>); break;  // timing only: no pre-store barriers
        case 52: launch2(k_blind_rotate_fast2<3, 1, 2, true, 1, 1, 2>); break;  // timing only: no barriers
        case 53: launch2(k_blind_rotate_fast2<3, 1, 2, true, 1, 1, 3>); break;  // timing only: no key loads
        default: launch2(k_blind_rotate_fast2<3, 1, 2, true, 1, 1>); break;     // = 39
    }
    return hipGetLastError();
}

}  // namespace tfhe
