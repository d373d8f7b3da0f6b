// ks_tiled.hip -- batch-tiled key switch (the KeySwitch of MKM, lwe-pke.cpp:299-321;
// reference kernel MKMSwitchKernel bootstrapping.cu:73-118).
//
// out[ct][k] = RoundqQ(-sum_{i<N, j<dKS} A[i][d_j(ct, i)][j][k] mod qKS, fmod, qKS)
// with d_j(ct, i) the j-th base-baseKS digit of RoundqQ(ext[ct][i], qKS, Q), and the
// same for the B column (b - sum).
//
// The gather form (k_mkm, one wavefront per ciphertext) reads N*dKS KSK rows per
// ciphertext: B times the rows, from L2/MALL/HBM.  Here a workgroup owns a tile of
// T = 256*CTS ciphertexts and CT columns, and for every (i, j) stages the baseKS row
// segments A[i][0..baseKS)[j][c0..c0+CT) in LDS once; its T ciphertexts then pick
// their rows from LDS.  The KSK leaves HBM ceil(B/T) times instead of B times
// (C3, qKS = 2^35: 4.8 GB KSK, 150 MB of gathered rows per ciphertext).
//
// Two launches:
//   k_ks_digits  RoundqQ + digits of every coefficient, transposed to
//                dig[(i*dKS + j)][ct] (u8) so a tile's digits for one (i, j) are one
//                contiguous run; bq[ct] = RoundqQ(b).
//   k_ks_tiled   the tiled accumulation; one workgroup barrier per (i, j): the next
//                step's row segments and digits are loaded into registers while this
//                step's are summed, then stored into the other LDS buffer.
#include "device_math.hpp"
#include "kernels.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <vector>

namespace tfhe {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // a native vector: stays in registers
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));  // two packed u16 column sums (v_pk_add_u16)
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));  // a 16-byte piece of u16 key words

constexpr int KT = 256;         // threads per workgroup
constexpr int DIG_TILE = 64;    // ciphertexts x coefficients per k_ks_digits block
constexpr int GMAX = 4;         // (i, j) steps per LDS stage (one barrier each): 2 or 4
constexpr uint32_t KS_MAX_DKS = 16;

// Digit planes: dig[(s / 4) * Bp + ct] holds the digits of steps s = 4g .. 4g+3 of one
// ciphertext (s = i*dKS + j, byte s % 4), so one u32 load gives a stage's digits.
__global__ void __launch_bounds__(256) k_ks_digits(KSParams P, const uint64_t* __restrict__ ext,
                                                   uint32_t* __restrict__ dig, uint64_t* __restrict__ bq, size_t B,
                                                   size_t Bp) {
    extern __shared__ __align__(16) unsigned char tile[];  // [64 coefficients * dKS steps][64 ciphertexts]
    const uint32_t N = P.N, dks = P.dKS, bks = P.baseKS;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t ct0 = (size_t)blockIdx.x * DIG_TILE;
    const uint32_t i0 = blockIdx.y * DIG_TILE;
    const uint32_t i = i0 + lane;
    for (uint32_t r = 0; r < DIG_TILE / 4; ++r) {
        const uint32_t cl = w * (DIG_TILE / 4) + r;
        const size_t ct = ct0 + cl;
        uint64_t x = 0;
        if (ct < B && i <= N) x = round_qQ(ext[ct * (N + 1) + i], P.qKS, P.Q);  // row ct: 64 consecutive words
        if (i == N) {
            if (ct < B) bq[ct] = x;
        } else {
            for (uint32_t j = 0; j < dks; ++j, x /= bks) tile[(lane * dks + j) * DIG_TILE + cl] = (uint8_t)(x % bks);
        }
    }
    __syncthreads();
    // the tile's 64*dKS steps start at step i0*dKS (a multiple of 4): words of 4 steps
    const uint32_t ni = min(DIG_TILE, (int)(N - min(N, i0)));
    const uint32_t groups = ni * dks / 4;
    const size_t g0 = (size_t)i0 * dks / 4;
    for (uint32_t wd = threadIdx.x; wd < groups * DIG_TILE; wd += 256) {
        const uint32_t g = wd / DIG_TILE, cl = wd % DIG_TILE;
        const unsigned char* t = tile + (size_t)g * 4 * DIG_TILE + cl;
        const uint32_t v = t[0] | (t[DIG_TILE] << 8) | (t[2 * DIG_TILE] << 16) | ((uint32_t)t[3 * DIG_TILE] << 24);
        dig[(g0 + g) * Bp + ct0 + cl] = v;
    }
}

// v-th KW word of a 16-byte piece (v a compile-time constant after unrolling)
template <typename KW>
__device__ __forceinline__ KW word_of(const u32x4& u, int v);
template <>
__device__ __forceinline__ uint16_t word_of<uint16_t>(const u32x4& u, int v) {
    const uint32_t w = v < 2 ? u.x : v < 4 ? u.y : v < 6 ? u.z : u.w;
    return (uint16_t)(w >> (16 * (v & 1)));
}
template <>
__device__ __forceinline__ uint32_t word_of<uint32_t>(const u32x4& u, int v) {
    return v == 0 ? u.x : v == 1 ? u.y : v == 2 ? u.z : u.w;
}
template <>
__device__ __forceinline__ uint64_t word_of<uint64_t>(const u32x4& u, int v) {
    return v == 0 ? ((uint64_t)u.y << 32 | u.x) : ((uint64_t)u.w << 32 | u.z);
}

// ACC: exact per-column sum type (u32 when N*dKS*(qKS-1) < 2^32).  Workgroup = T = 256*CTS
// ciphertexts x CT columns; G (i, j) steps per LDS stage; MAXL staged 16-byte pieces per
// thread and stage.  Block mapping: blocks b and b + 8 run on one XCD (round-robin
// dealing), so consecutive blocks of one XCD take the ciphertext tiles of ONE column tile:
// they stream the same KSK segments at about the same time and share them in that XCD's L2.
// Split over the steps (small batches: too few ciphertext x column tiles to fill the chip): the
// blocks of split z sum stages [z S, (z + 1) S) and store their partial sums (u64, column n = the
// B sum) in part[z][ct][n + 1]; k_ks_combine adds the splits and finishes.  nsplit = 1 finishes here.
// PK (u16 keys, qKS a power of two <= 2^16): the column sums are kept mod 2^16 as packed u16 pairs --
// each 16-byte piece of 8 key words is 4 v_pk_add_u16, with no unpacking -- which is exact mod qKS
// because qKS divides 2^16.
template <typename KW, typename ACC, int CT, int CTS, int MAXL, int G, bool PK = false>
__global__ void __launch_bounds__(KT, 2) k_ks_tiled(KSParams P, const KW* __restrict__ kska,
                                                 const KW* __restrict__ kskb, const uint32_t* __restrict__ dig,
                                                 const uint64_t* __restrict__ bq, size_t B, size_t Bp, uint32_t nct,
                                                 uint32_t ncol, uint64_t fmod, uint64_t* __restrict__ out,
                                                 uint32_t nsplit, uint64_t* __restrict__ part) {
    constexpr int VEC = 16 / sizeof(KW);           // KSK words per 16-byte piece
    constexpr int PIECES = CT / VEC;               // pieces per row segment
    constexpr int STRIDE = CT * sizeof(KW) + 16;   // LDS row pitch: consecutive rows start 4 banks apart
    static_assert(CT % VEC == 0, "column tile is whole pieces");
    static_assert(!PK || sizeof(KW) == 2, "packed sums are for u16 keys");
    static_assert(G == 2 || G == 4, "a stage is half or all of a digit word");
    extern __shared__ __align__(16) unsigned char sm[];
    const uint32_t bks = P.baseKS, dks = P.dKS, npad = P.n_pad, n = P.n;
    const uint32_t th = threadIdx.x;
    const uint32_t per_split = gridDim.x / nsplit, split = blockIdx.x / per_split;
    const uint32_t L = blockIdx.x - split * per_split, k = L >> 3;
    const uint32_t col_tile = (k / nct) * 8 + (L & 7), ct_tile = k % nct;
    if (col_tile >= ncol) return;  // whole workgroup
    const uint32_t c0 = col_tile * CT;
    const size_t t0 = (size_t)ct_tile * KT * CTS;
    const bool bcol = col_tile == 0;  // this column tile also sums the B column
    const uint32_t step_bytes = bks * STRIDE;
    const uint32_t stage_bytes = G * step_bytes;
    KW* bb = reinterpret_cast<KW*>(sm + 2 * stage_bytes);  // [2][G][baseKS] B entries
    const uint32_t npieces = bks * PIECES;                  // per step

    // Staging slots: slot l of a thread moves one 16-byte piece of step st_l = l / lps of a stage
    // (lps = slots per step, uniform), piece r = (l % lps) KT + th of that step's baseKS x PIECES.
    // Everything lane-dependent (the piece's offset in its step's KSK block and in LDS) is fixed for
    // the whole launch; per stage only the uniform step bases change (scalar arithmetic: s / dKS by
    // a magic multiply, exact for s < 2^32 / dKS), so a staged load is one global_load with a scalar
    // base and a 32-bit lane offset.  Loads are branch-free (clamped pieces, no exec-masked loads),
    // so the compiler's wait counters stay exact, and written without lambdas, so the staging
    // registers are not demoted to scratch.  Two register sets (X, Y) alternate: the rows of stage
    // g+2 are issued while those of g+1 are in flight.  Pieces past n_pad read in-row words of
    // another column instead of zeros: those columns (>= n_pad >= n) are never written out.
    const uint32_t lps = (npieces + KT - 1) / KT;
    const uint64_t dmagic = ((1ull << 32) + dks - 1) / dks;  // ceil(2^32 / dKS)
    const uint32_t bd = bks * dks;
    uint32_t st_of[MAXL], loff[MAXL], sto[MAXL];  // step (uniform), KSK lane offset (bytes), LDS offset
#pragma unroll
    for (int l = 0; l < MAXL; ++l) {
        const uint32_t st = (uint32_t)l / lps, r = ((uint32_t)l - st * lps) * KT + th;
        const uint32_t rr = min(r, npieces - 1);
        const uint32_t v = rr / PIECES, pc = rr - v * PIECES;
        const uint32_t col = min(c0 + pc * VEC, npad - VEC);
        st_of[l] = min(st, (uint32_t)G - 1);
        loff[l] = (v * dks * npad + col) * (uint32_t)sizeof(KW);
        sto[l] = (st < (uint32_t)G && r < npieces) ? st * step_bytes + v * STRIDE + pc * 16 : ~0u;
    }
    const uint32_t vb = min(th, bks - 1) * dks;  // B column: this lane's row v, in KW words
#define KS_LOAD(STG, BSTG, DGV, gg)                                                                 \
    do {                                                                                            \
        _Pragma("unroll") for (int c = 0; c < CTS; ++c)                                             \
            DGV[c] = dig[(size_t)((gg) * G / 4) * Bp + t0 + th + KT * c] >> (8 * (((gg) * G) % 4)); \
        _Pragma("unroll") for (int l = 0; l < MAXL; ++l) {                                          \
            const uint32_t s_ = (gg) * G + st_of[l];                                                \
            const uint32_t i = (uint32_t)(((uint64_t)s_ * dmagic) >> 32), j = s_ - i * dks;         \
            const char* pb = reinterpret_cast<const char*>(kska) + ((size_t)i * bd + j) * npad * sizeof(KW); \
            STG[l] = *reinterpret_cast<const u32x4*>(pb + loff[l]);                                 \
        }                                                                                           \
        if (bcol) {                                                                                 \
            _Pragma("unroll") for (int st = 0; st < G; ++st) {                                      \
                const uint32_t s_ = (gg) * G + st;                                                  \
                const uint32_t i = (uint32_t)(((uint64_t)s_ * dmagic) >> 32), j = s_ - i * dks;     \
                BSTG[st] = kskb[(size_t)i * bd + j + vb];                                           \
            }                                                                                       \
        }                                                                                           \
    } while (0)
#define KS_STORE(STG, BSTG, gg)                                                                     \
    do {                                                                                            \
        unsigned char* b_ = sm + ((gg) & 1) * stage_bytes;                                          \
        _Pragma("unroll") for (int l = 0; l < MAXL; ++l) {                                          \
            if (sto[l] != ~0u) *reinterpret_cast<u32x4*>(b_ + sto[l]) = STG[l];                     \
        }                                                                                           \
        if (bcol && th < bks) {                                                                     \
            _Pragma("unroll") for (int st = 0; st < G; ++st) bb[(((gg) & 1) * G + st) * bks + th] = BSTG[st]; \
        }                                                                                           \
    } while (0)
#define KS_SUM(DGV, gg)                                                                             \
    do {                                                                                            \
        const unsigned char* b_ = sm + ((gg) & 1) * stage_bytes;                                    \
        _Pragma("unroll 1") for (int st = 0; st < G; ++st) {                                        \
            _Pragma("unroll") for (int c = 0; c < CTS; ++c) {                                       \
                const uint32_t d = (DGV[c] >> (8 * st)) & 0xff;                                     \
                const unsigned char* r = b_ + st * step_bytes + d * STRIDE;                         \
                _Pragma("unroll") for (int p = 0; p < PIECES; ++p) {                                \
                    const u32x4 u = *reinterpret_cast<const u32x4*>(r + p * 16);                    \
                    if constexpr (PK) {                                                             \
                        const u16x8 h = *reinterpret_cast<const u16x8*>(r + p * 16);                \
                        apk[c][4 * p + 0] += __builtin_shufflevector(h, h, 0, 1);                   \
                        apk[c][4 * p + 1] += __builtin_shufflevector(h, h, 2, 3);                   \
                        apk[c][4 * p + 2] += __builtin_shufflevector(h, h, 4, 5);                   \
                        apk[c][4 * p + 3] += __builtin_shufflevector(h, h, 6, 7);                   \
                    } else {                                                                        \
                        _Pragma("unroll") for (int v = 0; v < VEC; ++v)                             \
                            acc[c][p * VEC + v] += (ACC)word_of<KW>(u, v);                          \
                    }                                                                               \
                }                                                                                   \
                if (bcol) bsum[c] += (uint64_t)bb[(((gg) & 1) * G + st) * bks + d];                 \
            }                                                                                       \
        }                                                                                           \
    } while (0)

    using BW = typename std::conditional<sizeof(KW) == 8, uint64_t, uint32_t>::type;  // B entries, widened
    u32x4 stgX[MAXL], stgY[MAXL];
    BW bX[G], bY[G];
    uint32_t dX[CTS], dY[CTS];
    ACC acc[CTS][PK ? 1 : CT];
    u16x2 apk[CTS][PK ? CT / 2 : 1];
    uint64_t bsum[CTS];
#pragma unroll
    for (int c = 0; c < CTS; ++c) {
        bsum[c] = 0;
#pragma unroll
        for (int kk = 0; kk < (PK ? 1 : CT); ++kk) acc[c][kk] = 0;
#pragma unroll
        for (int kk = 0; kk < (PK ? CT / 2 : 1); ++kk) apk[c][kk] = u16x2{0, 0};
    }
    // column kk's sum (PK: mod 2^16)
    auto colsum = [&](int c, int kk) -> uint64_t {
        if constexpr (PK) return (uint64_t)apk[c][kk >> 1][kk & 1];
        else return (uint64_t)acc[c][kk];
    };
#pragma unroll
    for (int st = 0; st < G; ++st) bX[st] = bY[st] = 0;
    const uint32_t stages = P.N * dks / G;  // even (ks_tiled_supported); nsplit divides stages / 2
    const uint32_t s_len = stages / nsplit, s_lo = split * s_len, s_hi = s_lo + s_len;
    KS_LOAD(stgX, bX, dX, s_lo);
    KS_LOAD(stgY, bY, dY, s_lo + 1);
    for (uint32_t g = s_lo; g < s_hi; g += 2) {
        // the last two stages reload their own rows (unconditional loads keep the counts exact)
        KS_STORE(stgX, bX, g);
        uint32_t dXc[CTS];
#pragma unroll
        for (int c = 0; c < CTS; ++c) dXc[c] = dX[c];
        KS_LOAD(stgX, bX, dX, min(g + 2, s_hi - 2));
        __syncthreads();
        KS_SUM(dXc, g);
        KS_STORE(stgY, bY, g + 1);
        uint32_t dYc[CTS];
#pragma unroll
        for (int c = 0; c < CTS; ++c) dYc[c] = dY[c];
        KS_LOAD(stgY, bY, dY, min(g + 3, s_hi - 1));
        __syncthreads();
        KS_SUM(dYc, g + 1);
    }
#undef KS_LOAD
#undef KS_STORE
#undef KS_SUM

    if (nsplit > 1) {  // partial sums for k_ks_combine
#pragma unroll
        for (int c = 0; c < CTS; ++c) {
            const size_t ct = t0 + th + KT * c;
            if (ct >= B) continue;
            uint64_t* o = part + ((size_t)split * B + ct) * (size_t)(n + 1);
#pragma unroll
            for (int kk = 0; kk < CT; ++kk)
                if (c0 + kk < n) o[c0 + kk] = colsum(c, kk);
            if (bcol) o[n] = bsum[c];
        }
        return;
    }
    const uint64_t qks = P.qKS;
#pragma unroll
    for (int c = 0; c < CTS; ++c) {
        const size_t ct = t0 + th + KT * c;
        if (ct >= B) continue;
        uint64_t* o = out + ct * (size_t)(n + 1);
#pragma unroll
        for (int kk = 0; kk < CT; ++kk) {
            const uint32_t col = c0 + kk;
            if (col < n) {
                const uint64_t r = colsum(c, kk) % qks;
                o[col] = round_qQ(r == 0 ? 0 : qks - r, fmod, qks);  // 0 - sum
            }
        }
        if (bcol) {
            const uint64_t r = bsum[c] % qks, x = bq[ct];
            o[n] = round_qQ(x >= r ? x - r : x + (qks - r), fmod, qks);  // b - sum
        }
    }
}

// ---------------------------------------------------------------------------
// Split-word form for the logQ contexts' 8-byte keys (verdict r5 item 5): qKS = 2^(32+b), 1 <= b <= 5
// (2^35 there), so every key word is below 2^(32+b).  k_pack_ks40 derives, once at setup, one 80-byte
// record per (KSK row, 16-column tile): the 16 low words (u32, 64 B), then the 16 high parts (u8, 16 B) --
// 80 B of LDS and L2 traffic per row segment against 128 B of u64 words.  The column sums only matter mod
// qKS: the low words sum exactly in u64 (one v_mad_u64_u32 with a unit factor each, as the u64 form's add;
// K40_SDWA below: two u32 sums of 16-bit halves instead, measured slower);
// the high parts sum as byte fields of u32 words, four columns per add, reduced mod 2^b after every stage
// of four steps (a field stays below 5 * 2^b <= 160, no carry into its neighbour); a column's sum is
// lo + (field mod 2^b) 2^32, congruent to the exact sum mod qKS.  Records are contiguous, so a row
// segment is five 16-byte pieces and the staging of k_ks_tiled carries over unchanged.
constexpr int K40_CT = 16, K40_REC = 80, K40_PIECES = K40_REC / 16;
// steps of a stage unrolled in the sum loop: 2 overlaps a step's LDS reads with the previous step's sums (same box,
// ARB12 at 128 / 1024 / 4096 ciphertexts: 1.32 / 2.75 / 8.74 ms unrolled once, 1.31 / 2.68 / 8.56 twice; round 5's
// u64 form 1.455 / 3.46 / 12.07; profiles/r06h)
#ifndef KS40_UNROLL
#define KS40_UNROLL 2
#endif
#if KS40_UNROLL == 2
#define K40_UNR _Pragma("unroll 2")
#else
#define K40_UNR _Pragma("unroll 1")
#endif

__global__ void k_pack_ks40(const uint64_t* __restrict__ ksk, size_t rows, uint32_t n, uint32_t npad64,
                            uint32_t ntiles, unsigned char* __restrict__ out) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;  // (row, tile, column)
    if (idx >= rows * ntiles * K40_CT) return;
    const uint32_t col = (uint32_t)(idx % K40_CT);
    const size_t rt = idx / K40_CT, row = rt / ntiles;
    const uint32_t cc = (uint32_t)(rt % ntiles) * K40_CT + col;
    const uint64_t w = cc < n ? ksk[row * npad64 + cc] : 0;  // columns past n are never written out
    unsigned char* rec = out + rt * K40_REC;
    reinterpret_cast<uint32_t*>(rec)[col] = (uint32_t)w;
    rec[64 + col] = (unsigned char)(w >> 32);
}

// K40_SDWA (A/B builds): 1 sums the low words as two u32 sums of their 16-bit halves (two SDWA adds per word),
// 0 (default) as u64 sums (one v_mad_u64_u32 with a unit factor per word): the SDWA form measured 4-5 % slower
// unrolled once and 1.7x slower unrolled twice (246 VGPRs; profiles/r06h)
#ifndef K40_SDWA
#define K40_SDWA 0
#endif
__device__ __forceinline__ uint64_t mad_u64_u32_1(uint32_t x, uint64_t acc) {  // acc + x in one VALU
    uint64_t r, junk;  // (the carry-out lane mask is never read)
    asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(r), "=s"(junk) : "v"(x), "v"(acc));
    return r;
}

template <int CTS, int MAXL, int G>
__global__ void __launch_bounds__(KT, 2) k_ks_tiled40(KSParams P, const unsigned char* __restrict__ rec,
                                                   const uint64_t* __restrict__ kskb, const uint32_t* __restrict__ dig,
                                                   const uint64_t* __restrict__ bq, size_t B, size_t Bp, uint32_t nct,
                                                   uint32_t ncol, uint64_t fmod, uint64_t* __restrict__ out,
                                                   uint32_t nsplit, uint64_t* __restrict__ part, uint32_t hbits) {
    static_assert(G == 2 || G == 4, "a stage is half or all of a digit word");
    extern __shared__ __align__(16) unsigned char sm[];
    const uint32_t bks = P.baseKS, dks = P.dKS, n = P.n;
    const uint32_t th = threadIdx.x;
    const uint32_t per_split = gridDim.x / nsplit, split = blockIdx.x / per_split;
    const uint32_t L = blockIdx.x - split * per_split, k = L >> 3;
    const uint32_t col_tile = (k / nct) * 8 + (L & 7), ct_tile = k % nct;  // (k_ks_tiled's XCD-aware mapping)
    if (col_tile >= ncol) return;  // whole workgroup
    const uint32_t c0 = col_tile * K40_CT;
    const size_t t0 = (size_t)ct_tile * KT * CTS;
    const bool bcol = col_tile == 0;
    const uint32_t step_bytes = bks * K40_REC;
    const uint32_t stage_bytes = G * step_bytes;
    uint64_t* bb = reinterpret_cast<uint64_t*>(sm + 2 * stage_bytes);  // [2][G][baseKS] B entries
    const uint32_t npieces = bks * K40_PIECES;                          // per step
    // staging slots as in k_ks_tiled: everything lane-dependent fixed for the launch
    const uint32_t lps = (npieces + KT - 1) / KT;
    const uint64_t dmagic = ((1ull << 32) + dks - 1) / dks;
    const uint32_t bd = bks * dks;
    const size_t rec_step = (size_t)ncol * K40_REC;  // bytes per KSK row (all its tiles)
    uint32_t st_of[MAXL], loff[MAXL], sto[MAXL];
#pragma unroll
    for (int l = 0; l < MAXL; ++l) {
        const uint32_t st = (uint32_t)l / lps, r = ((uint32_t)l - st * lps) * KT + th;
        const uint32_t rr = min(r, npieces - 1);
        const uint32_t v = rr / K40_PIECES, pc = rr - v * K40_PIECES;
        st_of[l] = min(st, (uint32_t)G - 1);
        loff[l] = (uint32_t)(v * dks * rec_step) + col_tile * K40_REC + pc * 16;
        sto[l] = (st < (uint32_t)G && r < npieces) ? st * step_bytes + v * K40_REC + pc * 16 : ~0u;
    }
    const uint32_t vb = min(th, bks - 1) * dks;
    const uint32_t hmask = 0x01010101u * ((1u << hbits) - 1);
    u32x4 stgX[MAXL], stgY[MAXL];
    uint64_t bX[G], bY[G];
    uint32_t dX[CTS], dY[CTS];
    uint32_t a0[CTS][K40_SDWA ? K40_CT : 1], a1[CTS][K40_SDWA ? K40_CT : 1];  // sums of the low words' 16-bit halves
    uint64_t al[CTS][K40_SDWA ? 1 : K40_CT];                                   // (each < 2^30: exact), or u64 sums
    uint32_t hs[CTS][K40_CT / 4];
    uint64_t bsum[CTS];
#pragma unroll
    for (int c = 0; c < CTS; ++c) {
        bsum[c] = 0;
#pragma unroll
        for (int kk = 0; kk < K40_CT; ++kk) {
            if constexpr (K40_SDWA) a0[c][kk] = a1[c][kk] = 0;
            else al[c][kk] = 0;
        }
#pragma unroll
        for (int m = 0; m < K40_CT / 4; ++m) hs[c][m] = 0;
    }
#pragma unroll
    for (int st = 0; st < G; ++st) bX[st] = bY[st] = 0;
#define K40_LOAD(STG, BSTG, DGV, gg)                                                                \
    do {                                                                                            \
        _Pragma("unroll") for (int c = 0; c < CTS; ++c)                                             \
            DGV[c] = dig[(size_t)((gg) * G / 4) * Bp + t0 + th + KT * c] >> (8 * (((gg) * G) % 4)); \
        _Pragma("unroll") for (int l = 0; l < MAXL; ++l) {                                          \
            const uint32_t s_ = (gg) * G + st_of[l];                                                \
            const uint32_t i = (uint32_t)(((uint64_t)s_ * dmagic) >> 32), j = s_ - i * dks;         \
            const unsigned char* pb = rec + ((size_t)i * bd + j) * rec_step;                        \
            STG[l] = *reinterpret_cast<const u32x4*>(pb + loff[l]);                                 \
        }                                                                                           \
        if (bcol) {                                                                                 \
            _Pragma("unroll") for (int st = 0; st < G; ++st) {                                      \
                const uint32_t s_ = (gg) * G + st;                                                  \
                const uint32_t i = (uint32_t)(((uint64_t)s_ * dmagic) >> 32), j = s_ - i * dks;     \
                BSTG[st] = kskb[(size_t)i * bd + j + vb];                                           \
            }                                                                                       \
        }                                                                                           \
    } while (0)
#define K40_STORE(STG, BSTG, gg)                                                                    \
    do {                                                                                            \
        unsigned char* b_ = sm + ((gg) & 1) * stage_bytes;                                          \
        _Pragma("unroll") for (int l = 0; l < MAXL; ++l) {                                          \
            if (sto[l] != ~0u) *reinterpret_cast<u32x4*>(b_ + sto[l]) = STG[l];                     \
        }                                                                                           \
        if (bcol && th < bks) {                                                                     \
            _Pragma("unroll") for (int st = 0; st < G; ++st) bb[(((gg) & 1) * G + st) * bks + th] = BSTG[st]; \
        }                                                                                           \
    } while (0)
#define K40_SUM(DGV, gg)                                                                            \
    do {                                                                                            \
        const unsigned char* b_ = sm + ((gg) & 1) * stage_bytes;                                    \
        K40_UNR for (int st = 0; st < G; ++st) {                                                       \
            /* every row piece of the step for all CTS ciphertexts in flight before the first sum  \
               (two waves per SIMD hide little LDS latency) */                                      \
            u32x4 U[CTS][K40_PIECES];                                                               \
            uint32_t dd[CTS];                                                                       \
            _Pragma("unroll") for (int c = 0; c < CTS; ++c) {                                       \
                dd[c] = (DGV[c] >> (8 * st)) & 0xff;                                                \
                const unsigned char* r = b_ + st * step_bytes + dd[c] * K40_REC;                    \
                _Pragma("unroll") for (int p = 0; p < K40_PIECES; ++p)                              \
                    U[c][p] = *reinterpret_cast<const u32x4*>(r + p * 16);                          \
            }                                                                                       \
            _Pragma("unroll") for (int c = 0; c < CTS; ++c) {                                       \
                _Pragma("unroll") for (int p = 0; p < 4; ++p)                                       \
                    _Pragma("unroll") for (int v = 0; v < 4; ++v) {                                 \
                        const uint32_t w = v == 0 ? U[c][p].x : v == 1 ? U[c][p].y : v == 2 ? U[c][p].z : U[c][p].w; \
                        if constexpr (K40_SDWA) {                                                   \
                            a0[c][4 * p + v] += w & 0xffff;  /* two SDWA adds */                    \
                            a1[c][4 * p + v] += w >> 16;                                            \
                        } else {                                                                    \
                            al[c][4 * p + v] = mad_u64_u32_1(w, al[c][4 * p + v]);                  \
                        }                                                                           \
                    }                                                                               \
                hs[c][0] += U[c][4].x, hs[c][1] += U[c][4].y, hs[c][2] += U[c][4].z, hs[c][3] += U[c][4].w; \
                if (bcol) bsum[c] += bb[(((gg) & 1) * G + st) * bks + dd[c]];                       \
            }                                                                                       \
        }                                                                                           \
        _Pragma("unroll") for (int c = 0; c < CTS; ++c)                                             \
            _Pragma("unroll") for (int m = 0; m < 4; ++m) hs[c][m] &= hmask;                        \
    } while (0)
    const uint32_t stages = P.N * dks / G;
    const uint32_t s_len = stages / nsplit, s_lo = split * s_len, s_hi = s_lo + s_len;
    K40_LOAD(stgX, bX, dX, s_lo);
    K40_LOAD(stgY, bY, dY, s_lo + 1);
    for (uint32_t g = s_lo; g < s_hi; g += 2) {
        K40_STORE(stgX, bX, g);
        uint32_t dXc[CTS];
#pragma unroll
        for (int c = 0; c < CTS; ++c) dXc[c] = dX[c];
        K40_LOAD(stgX, bX, dX, min(g + 2, s_hi - 2));
        __syncthreads();
        K40_SUM(dXc, g);
        K40_STORE(stgY, bY, g + 1);
        uint32_t dYc[CTS];
#pragma unroll
        for (int c = 0; c < CTS; ++c) dYc[c] = dY[c];
        K40_LOAD(stgY, bY, dY, min(g + 3, s_hi - 1));
        __syncthreads();
        K40_SUM(dYc, g + 1);
    }
#undef K40_LOAD
#undef K40_STORE
#undef K40_SUM
    // column kk's sum, congruent mod qKS = 2^(32 + hbits)
    auto colsum = [&](int c, int kk) -> uint64_t {
        const uint64_t lo = K40_SDWA ? (uint64_t)a0[c][kk] + ((uint64_t)a1[c][kk] << 16) : al[c][K40_SDWA ? 0 : kk];
        return lo + ((uint64_t)((hs[c][kk >> 2] >> (8 * (kk & 3))) & ((1u << hbits) - 1)) << 32);
    };
    if (nsplit > 1) {
#pragma unroll
        for (int c = 0; c < CTS; ++c) {
            const size_t ct = t0 + th + KT * c;
            if (ct >= B) continue;
            uint64_t* o = part + ((size_t)split * B + ct) * (size_t)(n + 1);
#pragma unroll
            for (int kk = 0; kk < K40_CT; ++kk)
                if (c0 + kk < n) o[c0 + kk] = colsum(c, kk);
            if (bcol) o[n] = bsum[c];
        }
        return;
    }
    const uint64_t qks = P.qKS;
#pragma unroll
    for (int c = 0; c < CTS; ++c) {
        const size_t ct = t0 + th + KT * c;
        if (ct >= B) continue;
        uint64_t* o = out + ct * (size_t)(n + 1);
#pragma unroll
        for (int kk = 0; kk < K40_CT; ++kk) {
            const uint32_t col = c0 + kk;
            if (col < n) {
                const uint64_t r = colsum(c, kk) % qks;
                o[col] = round_qQ(r == 0 ? 0 : qks - r, fmod, qks);  // 0 - sum
            }
        }
        if (bcol) {
            const uint64_t r = bsum[c] % qks, x = bq[ct];
            o[n] = round_qQ(x >= r ? x - r : x + (qks - r), fmod, qks);  // b - sum
        }
    }
}

// sum of the splits' partial sums (u64; u32 partials that wrapped mod 2^32 only when qKS divides
// 2^32, launch_ks_tiled), then the key switch's finish as in k_ks_tiled
__global__ void __launch_bounds__(256) k_ks_combine(KSParams P, const uint64_t* __restrict__ part, uint32_t nsplit,
                                                    const uint64_t* __restrict__ bq, size_t B, uint64_t fmod,
                                                    uint64_t* __restrict__ out) {
    const uint32_t n = P.n;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= B * (n + 1)) return;
    const size_t ct = i / (n + 1);
    const uint32_t col = (uint32_t)(i - ct * (n + 1));
    uint64_t sum = 0;
    for (uint32_t z = 0; z < nsplit; ++z) sum += part[(size_t)z * B * (n + 1) + i];
    const uint64_t qks = P.qKS, r = sum % qks;
    if (col < n) {
        out[i] = round_qQ(r == 0 ? 0 : qks - r, fmod, qks);  // 0 - sum
    } else {
        const uint64_t x = bq[ct];
        out[i] = round_qQ(x >= r ? x - r : x + (qks - r), fmod, qks);  // b - sum
    }
}

// Splits for a batch: enough blocks for two per CU (512), dividing the stage pairs; at most 4 up to
// kSplitMaxB ciphertexts, at most kMaxSplit up to kWideSplitMaxB (round 4: a 128- or 256-ciphertext
// batch has one ciphertext tile, 32 blocks for STD128Q -- the C5 shard of 1024 over 8 GPUs)
// Round 5 (profiles/r05y2, tools/ks_bench.py at 128 ciphertexts): the u64-key form there reads the whole
// 4.8 GB KSK once per launch, at 2.96 TB/s with 704 blocks; more blocks in flight (target 2048, up to 32
// splits) take LOGQ23's key switch 1.715 -> 1.412 ms.  The u16 / u32 forms keep at most 16 splits (32 cost
// STD128Q's 0.324 ms 12 %).
#ifndef KS_BLOCK_TARGET
#define KS_BLOCK_TARGET 2048
#endif
constexpr uint32_t kMaxSplit = 32, kMaxSplitNarrow = 16, kSplitMaxB = 2048, kWideSplitMaxB = 512;
// Round 6: the last wave's tail.  Every block of a launch sums the same number of steps, so a launch of `blocks`
// blocks with `slots` resident at once takes ceil(blocks z / slots) / z block-lengths when the steps split z ways
// (C3: 704 blocks at two per CU = 1.375 waves, i.e. two block-lengths with the second wave 37 % full).  Among
// z, 2z, 4z, ... (within the knob's cap, kTailSplitMax, the stage pairs and the partial-sum buffer) the shortest
// is taken; a candidate must beat the current one by 3 % (the partial sums and k_ks_combine cost a little).
constexpr uint32_t kTailSplitMax = 8, kTailSplitMaxCts = 8 * 8192;  // partial-sum rows: z B <= kTailSplitMaxCts
uint32_t ks_nsplit(const KSParams& P, size_t blocks, size_t B, const Knobs& kn, bool wide_keys, size_t slots) {
    const uint32_t knob = (uint32_t)std::max(1, kn.ks_split);  // knob (TFHE_KS_SPLIT): 1 = no split
    const uint32_t cap = std::min<uint32_t>(knob, B <= kWideSplitMaxB ? (wide_keys ? kMaxSplit : kMaxSplitNarrow) : 4);
    const uint32_t pairs = P.N * P.dKS / (2 * GMAX);
    uint32_t z = 1;
    while (2 * z <= cap && B <= kSplitMaxB && blocks * z < KS_BLOCK_TARGET && pairs % (2 * z) == 0) z *= 2;
    if (slots == 0) return z;
    auto cost = [&](uint32_t x) { return (double)((blocks * x + slots - 1) / slots) / x; };
    uint32_t best = z;
    for (uint32_t x = 2 * z; x <= std::min(knob, std::max(z, kTailSplitMax)) && pairs % (2 * x) == 0 &&
                             (size_t)x * B <= kTailSplitMaxCts;
         x *= 2)
        if (cost(x) < 0.97 * cost(best)) best = x;
    return best;
}

// resident blocks of kernel k at `lds` bytes of LDS per block, chip-wide (occupancy x CUs of the current device),
// cached per (kernel, lds)
size_t resident_blocks(const void* k, size_t lds) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<const void*, size_t>, size_t>> cache;
    std::lock_guard<std::mutex> lock(mu);
    for (auto& e : cache)
        if (e.first.first == k && e.first.second == lds) return e.second;
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, KT, lds) != hipSuccess || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;  // unknown: the round-5 rule alone
    const size_t r = (size_t)std::max(0, per_cu) * (size_t)std::max(0, cus);
    cache.push_back({{k, lds}, r});
    return r;
}

template <typename KW, typename ACC, int CT, int CTS, int G = 4, bool PK = false>
hipError_t launch_tiled(const KSParams& P, const void* kska, const void* kskb, const uint32_t* dig,
                        const uint64_t* bq, size_t B, size_t Bp, uint64_t fmod, uint64_t* out, uint64_t* part,
                        hipStream_t s, const Knobs& kn) {
    constexpr int STRIDE = CT * sizeof(KW) + 16;
    const size_t lds = 2 * (size_t)G * P.baseKS * STRIDE + 2 * (size_t)G * P.baseKS * sizeof(KW);
    // staging slots per thread and stage: G steps, ceil(pieces per step / KT) slots each (k_ks_tiled)
    const size_t lpt = (size_t)G * ((P.baseKS * (CT * sizeof(KW) / 16) + KT - 1) / KT);
    if (lds > 80 * 1024 || lpt > 8) return hipErrorNotSupported;
    // staging depth MAXL: only the depths some parameter set reaches are built (round 4; each is in a parity
    // test, tests/test_gpu_keyswitch.py): u16 keys 2 (baseKS 32: the *_OPT / STD256Q sets) or 4 (baseKS
    // 128), u32 keys with u32 sums 4 or 8 (baseKS 28 / 32 / 64: STD192, STD128Q / STD192Q), the others 4.
    // Any other shape takes the gather form.
    constexpr bool D2 = sizeof(KW) == 2, D8 = sizeof(KW) == 4 && sizeof(ACC) == 4;
    void (*k)(KSParams, const KW*, const KW*, const uint32_t*, const uint64_t*, size_t, size_t, uint32_t, uint32_t,
              uint64_t, uint64_t*, uint32_t, uint64_t*) = nullptr;
    if (lpt <= 2) {
        if constexpr (D2) k = k_ks_tiled<KW, ACC, CT, CTS, 2, G, PK>;
        else k = k_ks_tiled<KW, ACC, CT, CTS, 4, G, PK>;  // (a shallower need fits the depth-4 build)
    } else if (lpt <= 4) {
        k = k_ks_tiled<KW, ACC, CT, CTS, 4, G, PK>;
    } else {
        if constexpr (D8) k = k_ks_tiled<KW, ACC, CT, CTS, 8, G, PK>;
    }
    if (!k) return hipErrorNotSupported;
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    const uint32_t nct = (uint32_t)((B + KT * CTS - 1) / (KT * CTS));
    const uint32_t ncol = (P.n_pad + CT - 1) / CT;
    const uint32_t blocks = nct * ((ncol + 7) / 8) * 8;
    const uint32_t nsplit = ks_nsplit(P, blocks, B, kn, sizeof(KW) == 8, resident_blocks((const void*)k, lds));
    if (kn.trace)
        std::fprintf(stderr, "[ks] B=%zu key bytes=%d blocks=%u resident=%zu nsplit=%u\n", B, (int)sizeof(KW), blocks,
                     resident_blocks((const void*)k, lds), nsplit);
    hipLaunchKernelGGL(k, dim3(blocks * nsplit), dim3(KT), lds, s, P, (const KW*)kska, (const KW*)kskb, dig, bq, B, Bp,
                       nct, ncol, fmod, out, nsplit, part);
    if (nsplit > 1) {
        const size_t words = B * (P.n + 1);
        hipLaunchKernelGGL(k_ks_combine, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, P, part, nsplit, bq,
                           B, fmod, out);
    }
    return hipGetLastError();
}

uint32_t ks40_tiles(const KSParams& P) { return (P.n + K40_CT - 1) / K40_CT; }

// the split-word form's width: qKS = 2^(32 + b) with 1 <= b <= 5 (0: not applicable)
uint32_t ks40_hbits(const KSParams& P) {
    if ((P.qKS & (P.qKS - 1)) != 0 || P.qKS <= (1ull << 32) || P.qKS > (1ull << 37)) return 0;
    return (uint32_t)__builtin_ctzll(P.qKS) - 32;
}

template <int CTS, int G = 4>
hipError_t launch_tiled40(const KSParams& P, const void* rec, const void* kskb, const uint32_t* dig, const uint64_t* bq,
                          size_t B, size_t Bp, uint64_t fmod, uint64_t* out, uint64_t* part, hipStream_t s,
                          const Knobs& kn, uint32_t hbits) {
    const size_t lds = 2 * (size_t)G * P.baseKS * K40_REC + 2 * (size_t)G * P.baseKS * sizeof(uint64_t);
    const size_t lpt = (size_t)G * ((P.baseKS * K40_PIECES + KT - 1) / KT);
    if (lds > 80 * 1024 || lpt > 4) return hipErrorNotSupported;
    auto k = k_ks_tiled40<CTS, 4, G>;
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    const uint32_t nct = (uint32_t)((B + KT * CTS - 1) / (KT * CTS));
    const uint32_t ncol = ks40_tiles(P);
    const uint32_t blocks = nct * ((ncol + 7) / 8) * 8;
    const uint32_t nsplit = ks_nsplit(P, blocks, B, kn, true, resident_blocks((const void*)k, lds));
    if (kn.trace)
        std::fprintf(stderr, "[ks] B=%zu key bytes=%d blocks=%u resident=%zu nsplit=%u\n", B, 5, blocks,
                     resident_blocks((const void*)k, lds), nsplit);
    hipLaunchKernelGGL(k, dim3(blocks * nsplit), dim3(KT), lds, s, P, (const unsigned char*)rec, (const uint64_t*)kskb,
                       dig, bq, B, Bp, nct, ncol, fmod, out, nsplit, part, hbits);
    if (nsplit > 1) {
        const size_t words = B * (P.n + 1);
        hipLaunchKernelGGL(k_ks_combine, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, P, part, nsplit, bq,
                           B, fmod, out);
    }
    return hipGetLastError();
}

constexpr size_t kTileMax = 4 * KT;  // the largest ciphertext tile of the builds below
// (the packed-u16 form's column tile: 16 columns 1.51 ms, 64 columns / four steps per stage exceed the staging
// builds, against 0.93 ms for 32 columns and two steps at 8192; profiles/r06ks)

size_t ks_tiled_bp(size_t B) { return (B + kTileMax - 1) / kTileMax * kTileMax; }

}  // namespace

size_t ks_tiled_part_words(const KSParams& P, size_t B) {  // split partial sums (ks_nsplit)
    return std::max({(size_t)kMaxSplit * std::min(B, (size_t)kWideSplitMaxB), (size_t)4 * std::min(B, (size_t)kSplitMaxB),
                     std::min((size_t)kTailSplitMax * B, (size_t)kTailSplitMaxCts)}) *
           (P.n + 1);
}

size_t ks_tiled_scratch_bytes(const KSParams& P, size_t B) {
    const size_t Bp = ks_tiled_bp(B);
    return (size_t)P.N * P.dKS * Bp + Bp * sizeof(uint64_t) + ks_tiled_part_words(P, B) * sizeof(uint64_t);
}

size_t ks40_bytes(const KSParams& P) {
    return ks40_hbits(P) ? (size_t)P.N * P.baseKS * P.dKS * ks40_tiles(P) * K40_REC : 0;
}

hipError_t launch_pack_ks40(const KSParams& P, const void* kska, void* out, hipStream_t s) {
    if (!ks40_hbits(P)) return hipErrorNotSupported;
    const size_t rows = (size_t)P.N * P.baseKS * P.dKS, threads = rows * ks40_tiles(P) * K40_CT;
    hipLaunchKernelGGL(k_pack_ks40, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, (const uint64_t*)kska,
                       rows, P.n, P.n_pad, ks40_tiles(P), (unsigned char*)out);
    return hipGetLastError();
}

bool ks_tiled_supported(const KSParams& P) {
    // even stage count; step indices s < N dKS far below 2^32 / dKS (k_ks_tiled's magic-multiply s / dKS)
    return P.dKS >= 1 && P.dKS <= KS_MAX_DKS && P.baseKS <= 256 && (P.N * P.dKS) % (8 * GMAX) == 0 &&
           (uint64_t)P.N * P.dKS < (1ull << 24);
}

hipError_t launch_ks_tiled(const KSParams& P, int ksk_bits, const void* kska, const void* kskb, const uint64_t* ext,
                           uint64_t fmod, uint64_t* out, size_t B, void* scratch, hipStream_t s, const Knobs& kn,
                           const void* ksk40) {
    if (B == 0) return hipSuccess;
    if (!ks_tiled_supported(P)) return hipErrorNotSupported;
    const bool acc32 = (unsigned __int128)P.N * P.dKS * (P.qKS - 1) < ((unsigned __int128)1 << 32);
    // u16 keys sum in 32 bits: exact below 2^32, and wrapping mod 2^32 is harmless when qKS divides
    // it; otherwise the gather form (k_mkm, 64-bit sums) serves the call
    if (ksk_bits == 16 && !acc32 && (P.qKS & (P.qKS - 1)) != 0) return hipErrorNotSupported;
    const size_t Bp = ks_tiled_bp(B);
    uint32_t* dig = static_cast<uint32_t*>(scratch);
    uint64_t* bq = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(scratch) + (size_t)P.N * P.dKS * Bp);
    uint64_t* part = bq + Bp;
    const size_t lds_dig = (size_t)P.dKS * DIG_TILE * DIG_TILE;
    hipError_t e = hipFuncSetAttribute((const void*)k_ks_digits, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_dig);
    if (e != hipSuccess) return e;
    // every ciphertext tile of Bp gets digits (zeros past B), so k_ks_tiled reads no garbage
    const dim3 g1((unsigned)(Bp / DIG_TILE), (P.N + 1 + DIG_TILE - 1) / DIG_TILE);
    hipLaunchKernelGGL(k_ks_digits, g1, dim3(256), lds_dig, s, P, ext, dig, bq, B, Bp);
    // ciphertexts per thread: two halve the KSK segments streamed per ciphertext; they pay for u64 keys
    // (ARB12 B = 4096 13.8 -> 12.5 ms, logQ = 23 B = 1024 4.06 -> 3.66) and for u32 keys at large
    // batches (STD192 8192 5.81 -> 5.24), not for STD128Q at 1024 (1.26 -> 1.40) or the packed u16
    // form (profiles/r03ks, r03ks2, r03z).  The ks_cts knob (TFHE_KS_CTS) overrides (A/B runs and tests).
    // (ks_cts 4 builds only for the packed u16 form; the other widths take 2 for it)
    const int cts = kn.ks_cts ? std::min(kn.ks_cts, 2) : (ksk_bits == 64 || (ksk_bits == 32 && B >= 4096)) ? 2 : 1;
    // the packed u16 form (STD128): four ciphertexts per thread from 2048 ciphertexts -- the KSK (256.5 MiB, at the
    // Infinity Cache's size) is streamed once per ciphertext tile, so 8192 / 1024 tiles instead of 8192 / 256
    // (same box, two alternations: 8192 0.927 -> 0.641-0.646 ms, 4096 0.552-0.556 -> 0.372-0.375, 2048 0.33 ->
    // 0.265-0.276; two per thread 0.79 / 0.47 / 0.28; at 1024 two per thread were slower, 0.217 -> 0.234:
    // profiles/r06ks2, r06ks3)
    const int cts16 = kn.ks_cts ? kn.ks_cts : B >= 2048 ? 4 : 1;
    switch (ksk_bits) {
        case 16:  // baseKS = 128 rows per step: two steps per stage keep the LDS at 40 KiB
            // qKS a power of two <= 2^16 (STD128: 2^14): packed u16 sums (ks_pk knob 0: u32 sums, A/B runs)
            if ((P.qKS & (P.qKS - 1)) == 0 && P.qKS <= (1u << 16) && kn.ks_pk)
                return cts16 == 4   ? launch_tiled<uint16_t, uint32_t, 32, 4, 2, true>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn)
                       : cts16 == 2 ? launch_tiled<uint16_t, uint32_t, 32, 2, 2, true>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn)
                                    : launch_tiled<uint16_t, uint32_t, 32, 1, 2, true>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn);
            return launch_tiled<uint16_t, uint32_t, 32, 1, 2>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn);
        case 32:
            // u32 sums also when they wrap mod 2^32 harmlessly: qKS a power of two (STD128Q: 2^25)
            if (acc32 || (P.qKS & (P.qKS - 1)) == 0)
                return cts == 2 ? launch_tiled<uint32_t, uint32_t, 32, 2>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn)
                                : launch_tiled<uint32_t, uint32_t, 32, 1>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn);
            return cts == 2 ? launch_tiled<uint32_t, uint64_t, 16, 2>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn)
                            : launch_tiled<uint32_t, uint64_t, 32, 1>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn);
        default:
            // the split-word records (ks40 knob, default on; 0: the u64 form, A/B runs and tests)
            if (ksk40 && kn.ks40 && ks40_hbits(P)) {
                const hipError_t e40 = cts == 2 ? launch_tiled40<2>(P, ksk40, kskb, dig, bq, B, Bp, fmod, out, part, s, kn, ks40_hbits(P))
                                                : launch_tiled40<1>(P, ksk40, kskb, dig, bq, B, Bp, fmod, out, part, s, kn, ks40_hbits(P));
                if (e40 != hipErrorNotSupported) return e40;
            }
            return cts == 2 ? launch_tiled<uint64_t, uint64_t, 16, 2>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn)
                            : launch_tiled<uint64_t, uint64_t, 16, 1>(P, kska, kskb, dig, bq, B, Bp, fmod, out, part, s, kn);
    }
}

}  // namespace tfhe
