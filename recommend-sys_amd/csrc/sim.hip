// sim.hip -- K4 / K5: all-pairs similarity of KNN.Fit (reference core/knn.go:143-217 with
// core/sim.go:10-81 as the pair function), gfx950.
//
// K4 (Cosine, MSD; bit-exact): when every rating is r = x / s with integer x, s in {1, 2} and
// 1 <= x <= 11 (ML-100K/1M integer stars: s = 1; ML-20M half stars: s = 2), the co-rated sums of
// sim.go are exact integers times 1/s^2.  They are computed as int8 x int8 -> int32 MFMA
// contractions over the dense (left x right) matrices X (x), X2 (x^2) and M (1 where rated):
//     l = X X^T,   m = X2 M^T,   n = M X2^T,   count = M M^T  (MSD only)
// and the float64 epilogue evaluates exactly the reference expressions
//     Cosine  l / (sqrt(m) * sqrt(n))            (sim.go:24)
//     MSD     1 / (sum / count + 1), sum = m + n - 2 l  (sim.go:43)
// on the exactly-representable sums, so every similarity (and the NaN pattern: 0/0 where nothing
// is co-rated, knn.go:205) is bitwise equal to the reference's sorted-merge result.
// Only tiles of the upper triangle are computed; each writes S[a][b] and S[b][a] (knn.go:206-207)
// and the diagonal stays NaN (knn.go:202).
//
// K5 (Pearson, and Cosine/MSD when ratings are not of that form): one workgroup per left row a,
// row a scattered densely into LDS (or a global scratch row), one thread per partner b > a walking
// b's ID-sorted list; the co-rated IDs are therefore visited in ascending order exactly like the
// sorted merge of sim.go, with the same float64 operations in the same order -> bitwise equal.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

#include "common.hpp"

namespace rs {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 128;   // block tile (a x b)
constexpr int kKBlock = 64;  // bytes of the contraction dimension per iteration

// ---------------------------------------------------------------------------------------------
// dense operand X[a][k] = x in [1, 11], 0 = not rated (rows padded to kTile, k padded to kKBlock)

__global__ void knn_scatter_kernel(int32_t L, const int64_t* __restrict__ rowptr,
                                   const int32_t* __restrict__ ids, const int8_t* __restrict__ x,
                                   int64_t ldk, int8_t* __restrict__ X) {
    const int32_t a = blockIdx.x;
    if (a >= L) return;
    for (int64_t t = rowptr[a] + threadIdx.x; t < rowptr[a + 1]; t += blockDim.x)
        X[static_cast<int64_t>(a) * ldk + ids[t]] = x[t];
}

// KIND 0 = Cosine (3 contractions), 1 = MSD (4 contractions), 2 = SlopeOne deviations
// (3 contractions: X M^T, M X^T, M M^T; slope_one.go:64-92, see the epilogue).
//
// One 128 x 128 tile (ta <= tb) of the upper triangle per workgroup, tiles taken from a host-built
// list in 16 x 16 super-tile groups so the workgroups resident together share row blocks.  Four
// waves, each a 64 x 64 sub-tile of 2 x 2 v_mfma_i32_32x32x32_i8 tiles.  Only X is read from HBM:
// every rating is x = r s with x in [1, 11] and 0 marks "not rated", so the loader derives
// X2 = x^2 (two v_pk_mul_lo_u16 per dword) and M = [x > 0] (SWAR add/and) itself -- a third of
// the global traffic of loading all three.  Per 64-byte K step the workgroup stages the A rows (ta)
// and B rows (tb) of X, X2 and M into a double-buffered LDS tile; the next step's X loads are in
// flight during the MFMAs, and the steps are separated by a raw s_barrier after an lgkmcnt-only
// wait, so the loads stay in flight across it.  LDS rows are
// 64 bytes with the 16-byte chunk c of row r stored at chunk c ^ ((r >> 2) & 3): the staging
// writes and the fragment reads are both bank-conflict free.
constexpr int kRowPad = 64;                             // bytes per staged row
constexpr int kStageMat = kTile * kRowPad;              // one matrix, one side
constexpr int kStageBytes = 3 * 2 * kStageMat;          // X, X2, M for A and B
constexpr int kXChunks = 2 * kTile * (kKBlock / 16);    // 16-byte X chunks per step (A and B)

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t sq_bytes(uint32_t w) {  // per byte x^2 (x <= 11)
    const uint32_t e = w & 0x00FF00FFu, o = (w >> 8) & 0x00FF00FFu;
    const u16x2 e2 = __builtin_bit_cast(u16x2, e) * __builtin_bit_cast(u16x2, e);
    const u16x2 o2 = __builtin_bit_cast(u16x2, o) * __builtin_bit_cast(u16x2, o);
    return __builtin_bit_cast(uint32_t, e2) | (__builtin_bit_cast(uint32_t, o2) << 8);
}
__device__ __forceinline__ uint32_t sq_bytes_perm(uint32_t w) {  // sq_bytes in five operations
    const uint32_t e = w & 0x00FF00FFu;                         // bytes 0, 2 as u16 lanes
    const uint32_t o = __builtin_amdgcn_perm(0u, w, 0x0C030C01u);  // bytes 1, 3 as u16 lanes
    const u16x2 e2 = __builtin_bit_cast(u16x2, e) * __builtin_bit_cast(u16x2, e);
    const u16x2 o2 = __builtin_bit_cast(u16x2, o) * __builtin_bit_cast(u16x2, o);
    // bytes [e2.lo, o2.lo, e2.hi, o2.hi]: selector picks byte 0 of e2 (4), byte 0 of o2 (0), ...
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, e2), __builtin_bit_cast(uint32_t, o2), 0x02060004u);
}
__device__ __forceinline__ uint32_t mask128_bytes(uint32_t w) {  // per byte 0x80 (= -128) where x > 0
    return (w + 0x7F7F7F7Fu) & 0x80808080u;
}
__device__ __forceinline__ uint32_t mask_bytes(uint32_t w) {  // per byte [x > 0] (x <= 127)
    return ((w + 0x7F7F7F7Fu) & 0x80808080u) >> 7;
}

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: global loads stay in flight
    __builtin_amdgcn_s_barrier();
}

// NWJ = 32-column MFMA tiles per wave along b: 2 -> four waves of 64 x 64 (one wave per SIMD,
// 192 accumulator AGPRs); 1 -> eight waves of 64 x 32 (two waves per SIMD, 96 AGPRs each, so the
// SIMD interleaves two waves' phases; PIPE 2 only).
template <int KIND, int PIPE, int NWJ = 2, int ROT = 0, bool LEAN = false>
__global__ __launch_bounds__(NWJ == 2 ? 256 : 512) void knn_sims_mfma_kernel(const int8_t* __restrict__ X,
                                                            int64_t ldk, int32_t L,
                                                            const int2* __restrict__ tiles,
                                                            double inv_s2, double* __restrict__ S) {
    constexpr int NC = KIND == 1 ? 4 : 3;
    static_assert(NWJ == 2 || PIPE >= 1, "the eight-wave tiling exists for the pipelined loops only");
    constexpr int NT = NWJ == 2 ? 256 : 512;      // threads
    constexpr int kXPerThread = kXChunks / NT;    // 16-byte X chunks staged per thread and step
    constexpr int FPM = 2 + NWJ;                  // fragments per matrix and half: 2 a-tiles, NWJ b-tiles
    extern __shared__ __attribute__((aligned(16))) int8_t smem[];
    const int2 tile = tiles[blockIdx.x];
    const int32_t ta = tile.x, tb = tile.y;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wa = NWJ == 2 ? wave >> 1 : wave >> 2, wb = NWJ == 2 ? wave & 1 : wave & 3;
    // strictly below the diagonal (a rows start at or after the b columns end): the mirror covers it
    const bool live = !(ta == tb && 64 * wa >= 32 * NWJ * (wb + 1));
    const int row = lane & 31, half = lane >> 5;

    i32x16 acc[NC][2][NWJ];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < NWJ; ++j) acc[c][i][j] = i32x16{};

    // staging map: chunk j of thread tid = side j >> 1, row (tid >> 2) + 64 (j & 1), 16-byte
    // column tid & 3 -- a wave-uniform base per (side, j) plus one 32-bit lane offset (eight
    // waves: chunk j = side j, row tid >> 2)
    const int8_t* baseA = X + static_cast<int64_t>(ta) * kTile * ldk;
    const int8_t* baseB = X + static_cast<int64_t>(tb) * kTile * ldk;
    const uint32_t loff = static_cast<uint32_t>((tid >> 2) * ldk + 16 * (tid & 3));
    const int64_t half_rows = 64 * ldk;
    const int r_lo = tid >> 2;
    int32_t dst[kXPerThread];
#pragma unroll
    for (int j = 0; j < kXPerThread; ++j) {
        const int side = NWJ == 2 ? j >> 1 : j, r = r_lo + (NWJ == 2 ? 64 * (j & 1) : 0), c = tid & 3;
        dst[j] = side * kStageMat + r * kRowPad + 16 * (c ^ ((r >> 2) & 3));
    }
    auto gload = [&](i32x4 (&st)[kXPerThread], int64_t k0) {
#pragma unroll
        for (int j = 0; j < kXPerThread; ++j) {
            const int8_t* base = NWJ == 2 ? ((j >> 1) ? baseB : baseA) + (j & 1) * half_rows + k0
                                          : (j ? baseB : baseA) + k0;
            st[j] = *reinterpret_cast<const i32x4*>(base + loff);
        }
    };
    auto lstore = [&](const i32x4 (&st)[kXPerThread], int buf) {
        int8_t* b = smem + buf * kStageBytes;
#pragma unroll
        for (int j = 0; j < kXPerThread; ++j) {
            *reinterpret_cast<i32x4*>(b + 0 * 2 * kStageMat + dst[j]) = st[j];
            i32x4 v;
            if constexpr (KIND != 2) {  // SlopeOne never reads X2
#pragma unroll
                for (int d = 0; d < 4; ++d) v[d] = static_cast<int>(sq_bytes(static_cast<uint32_t>(st[j][d])));
                *reinterpret_cast<i32x4*>(b + 1 * 2 * kStageMat + dst[j]) = v;
            }
#pragma unroll
            for (int d = 0; d < 4; ++d) v[d] = static_cast<int>(mask_bytes(static_cast<uint32_t>(st[j][d])));
            *reinterpret_cast<i32x4*>(b + 2 * 2 * kStageMat + dst[j]) = v;
        }
    };
    // fragment of (matrix m, side, 32-row tile i, k sub-step s): lane (row, half) reads the 16
    // bytes [32 s + 16 half, +16) of its row -- the same k bijection for both operands, so
    // sum_k A[a][k] B[b][k] is exact whatever the MFMA's internal k order.
    auto frag = [&](const int8_t* b, int m, int side, int i, int s) {
        const int r = (side ? 32 * NWJ * wb : 64 * wa) + 32 * i + row;
        const int c = (2 * s + half) ^ ((r >> 2) & 3);
        return *reinterpret_cast<const i32x4*>(b + (m * 2 + side) * kStageMat + r * kRowPad + 16 * c);
    };
    auto compute = [&](int buf) {
        if constexpr (NWJ != 2) return;
        const int8_t* b = smem + buf * kStageBytes;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (PIPE) {
                if (s == 1) break;
            }
            i32x4 fa[3][2], fb[3][2];
#pragma unroll
            for (int m = 0; m < 3; ++m)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    fa[m][i] = frag(b, m, 0, i, s);
                    fb[m][i] = frag(b, m, 1, i, s);
                }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (KIND == 2) {  // s1 = X_a M_b, s2 = M_a X_b, count = M_a M_b
                        acc[0][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[0][i], fb[2][j], acc[0][i][j], 0, 0, 0);
                        acc[1][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[2][i], fb[0][j], acc[1][i][j], 0, 0, 0);
                        acc[2][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[2][i], fb[2][j], acc[2][i][j], 0, 0, 0);
                        continue;
                    }
                    acc[0][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[0][i], fb[0][j], acc[0][i][j], 0, 0, 0);
                    acc[1][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[1][i], fb[2][j], acc[1][i][j], 0, 0, 0);
                    acc[2][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[2][i], fb[1][j], acc[2][i][j], 0, 0, 0);
                    if constexpr (NC == 4)
                        acc[3][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[2][i], fb[2][j], acc[3][i][j], 0, 0, 0);
                }
        }
    };

    // One K step of the software pipeline (PIPE): all 24 fragment reads up front, then the MFMAs
    // of both 32-deep halves with the next step's X2 / M derivation and staging writes woven
    // between them.  One wave per SIMD (192 accumulator AGPRs) cannot hide the VALU, LDS and MFMA
    // phases behind other waves, so the wave has to overlap them itself: an MFMA occupies the
    // matrix pipe for 32 cycles while the wave issues the independent VALU / LDS work behind it.
    // The body is one basic block (the last step reloads its own chunk and stages it into the
    // buffer nobody reads again), so the scheduler can apply the group pattern.
    auto pipe_step = [&](int buf, i32x4 (&st)[kXPerThread]) {
        const int8_t* b = smem + buf * kStageBytes;
        int8_t* nb = smem + (buf ^ 1) * kStageBytes;  // last read in the previous step (barrier between)
        i32x4 fa[2][3][2], fb[2][3][NWJ];
        auto read = [&](int s, int x) {  // fragment x of 3 FPM: matrix x / FPM, then a-tiles 0-1, b-tiles
            const int m = x / FPM, r = x % FPM, side = r >= 2, i = side ? r - 2 : r;
            if (PIPE == 2 && m == 2) {  // M = [x > 0] of the X fragment read at the same place
                i32x4& d = side ? fb[s][2][i] : fa[s][2][i];
                const i32x4& src = side ? fb[s][0][i] : fa[s][0][i];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    d[e] = static_cast<int>(LEAN ? mask128_bytes(static_cast<uint32_t>(src[e])) : mask_bytes(static_cast<uint32_t>(src[e])));
            } else if (side) {
                fb[s][m][i] = frag(b, m, 1, i, s);
            } else {
                fa[s][m][i] = frag(b, m, 0, i, s);
            }
        };
        constexpr int NM = 2 * NWJ * NC;  // MFMAs per half
        auto mfma = [&](int s, int x) {  // x = (c * 2 + i) * NWJ + j
            const int c = x / (2 * NWJ), i = (x / NWJ) & 1, j = x % NWJ;
            // operands per contraction c: Cosine/MSD (X,X) (X2,M) (M,X2) (M,M); SlopeOne (X,M) (M,X) (M,M)
            const int ma = KIND == 2 ? (c == 0 ? 0 : 2) : (c == 0 ? 0 : c == 1 ? 1 : 2);
            const int mb = KIND == 2 ? (c == 1 ? 0 : 2) : (c == 0 ? 0 : c == 1 ? 2 : c == 2 ? 1 : 2);
            acc[c][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[s][ma][i], fb[s][mb][j], acc[c][i][j], 0, 0, 0);
        };
        i32x4 sq[kXPerThread], mk[kXPerThread];
        auto stage = [&](int x) {  // slice x of the next step's staging (x in [0, NM))
            constexpr int per = (3 * kXPerThread + NM - 1) / NM;  // (chunk, part) units per slice
#pragma unroll
            for (int u = 0; u < per; ++u) {
                const int w = x * per + u;
                if (w >= 3 * kXPerThread) break;
                const int j = w / 3, part = w % 3;
                if (part == 0) {
                    *reinterpret_cast<i32x4*>(nb + dst[j]) = st[j];
                } else if (part == 1) {
                    if constexpr (KIND != 2) {
#pragma unroll
                        for (int d = 0; d < 4; ++d)
                            sq[j][d] = static_cast<int>(LEAN ? sq_bytes_perm(static_cast<uint32_t>(st[j][d])) : sq_bytes(static_cast<uint32_t>(st[j][d])));
                        *reinterpret_cast<i32x4*>(nb + 1 * 2 * kStageMat + dst[j]) = sq[j];
                    }
                } else if (PIPE != 2) {  // PIPE 2 derives M from the X fragments instead
#pragma unroll
                    for (int d = 0; d < 4; ++d) mk[j][d] = static_cast<int>(mask_bytes(static_cast<uint32_t>(st[j][d])));
                    *reinterpret_cast<i32x4*>(nb + 2 * 2 * kStageMat + dst[j]) = mk[j];
                }
            }
        };
        // half 0's fragments; then its MFMAs, each followed by one of half 1's fragment reads;
        // then half 1's MFMAs, each followed by a slice of the next step's X2 / M derivation and
        // staging writes.  sched_barrier(0) keeps this order: an MFMA holds the matrix pipe for 32
        // cycles while the wave issues the independent LDS / VALU work behind it.
        // (PIPE 2: half 0's M fragments are derived behind its first four MFMAs, the X X^T ones;
        // SlopeOne never reads X2 and its first contraction, X M^T, needs M at once)
        // The late M fragments go b-side first: the second contraction (X2_a, M_b) needs them.
        constexpr bool m_late = PIPE == 2 && KIND != 2;
        constexpr int NF = 3 * FPM;
        auto needed = [](int x) { return !(KIND == 2 && x / FPM == 1); };
        auto late = [](int k) { return k < NWJ ? 2 * FPM + 2 + k : 2 * FPM + k - NWJ; };
#pragma unroll
        for (int x = 0; x < NF; ++x)
            if (needed(x) && !(m_late && x >= 2 * FPM)) read(0, x);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int x = 0; x < NM; ++x) {
            mfma(0, x);
            if (m_late && x < FPM) read(0, late(x));
            if (x < NF && needed(x)) read(1, x);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int x = NM; x < NF; ++x)
            if (needed(x)) read(1, x);
#pragma unroll
        for (int x = 0; x < NM; ++x) {
            mfma(1, x);
            stage(x);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // the next step's X loads are in flight during this step's MFMAs (a second set in flight
    // spills: 153 VGPRs, 3x slower -- measured)
    const int64_t nsteps = ldk / kKBlock;
    i32x4 st[kXPerThread];
    gload(st, 0);
    lstore(st, 0);
    lds_barrier();
    if constexpr (ROT == 1) {
        // loads one step further ahead through a rotation: st (step t + 1, loaded during step
        // t - 1) is staged while st2 loads step t + 2; st = st2 at the end of the step, so a load
        // has a whole step to land before anything waits on it
        i32x4 st2[kXPerThread];
        gload(st, std::min<int64_t>(1, nsteps - 1) * kKBlock);
        for (int64_t step = 0; step < nsteps; ++step) {
            const int buf = static_cast<int>(step & 1);
            gload(st2, std::min<int64_t>(step + 2, nsteps - 1) * kKBlock);
            pipe_step(buf, st);
#pragma unroll
            for (int j = 0; j < kXPerThread; ++j) st[j] = st2[j];
            lds_barrier();
        }
    } else if constexpr (PIPE) {
        for (int64_t step = 0; step < nsteps; ++step) {
            const int buf = static_cast<int>(step & 1);
            gload(st, std::min<int64_t>(step + 1, nsteps - 1) * kKBlock);
            pipe_step(buf, st);
            lds_barrier();
        }
    } else {
        for (int64_t step = 0; step < nsteps; ++step) {
            const int buf = static_cast<int>(step & 1);
            if (step + 1 < nsteps) gload(st, (step + 1) * kKBlock);
            compute(buf);
            if (step + 1 < nsteps) lstore(st, buf ^ 1);  // buf ^ 1 was last read in step - 1
            lds_barrier();
        }
    }
    if (!live) return;
    const int32_t r0 = ta * kTile + 64 * wa;  // left rows (a)
    const int32_t c0 = tb * kTile + 32 * NWJ * wb;  // partner rows (b)
    // epilogue: C/D layout of 32x32 MFMA: col = lane & 31, row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5)
    const double nan = __builtin_nan("");
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NWJ; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int32_t a = r0 + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * half;
                const int32_t bb = c0 + 32 * j + row;
                if (a >= L || bb >= L) continue;
                if (a == bb) {
                    S[static_cast<int64_t>(a) * L + bb] = KIND == 2 ? 0.0 : nan;  // dev: zero matrix
                    continue;
                }
                if (ta == tb && a > bb) continue;
                // LEAN: the M operand is -128 where rated, so its contractions carry a factor -128 (count:
                // 16384); exact while a co-rated count stays below 2^17 (the host checks the row degrees)
                constexpr bool m128 = LEAN && PIPE == 2;
                const int64_t li = m128 && KIND == 2 ? -(acc[0][i][j][q] >> 7) : acc[0][i][j][q];
                const int64_t mi = m128 ? -(acc[1][i][j][q] >> 7) : acc[1][i][j][q];
                const int64_t ni = m128 ? (KIND == 2 ? acc[2][i][j][q] >> 14 : -(acc[2][i][j][q] >> 7)) : acc[2][i][j][q];
                double v;
                if constexpr (KIND == 2) {
                    // slope_one.go:68-88 for the pair i = bb > j = a: sum of (r_bb - r_a) over the
                    // co-rated users, exact in float64 whatever the order (half-integers) and equal
                    // to (sum x_bb - sum x_a) / s; dev[i][j] = sum / count, dev[j][i] = -dev[i][j];
                    // nothing co-rated: both stay 0 (newZeroMatrix).  inv_s2 carries 1 / s here.
                    double d = 0.0, md = 0.0;
                    if (ni > 0) {
                        d = static_cast<double>(mi - li) * inv_s2 / static_cast<double>(ni);
                        md = -d;
                    }
                    S[static_cast<int64_t>(bb) * L + a] = d;
                    S[static_cast<int64_t>(a) * L + bb] = md;
                    continue;
                } else if constexpr (KIND == 0) {
                    const double l = static_cast<double>(li) * inv_s2;
                    const double m = static_cast<double>(mi) * inv_s2;
                    const double n = static_cast<double>(ni) * inv_s2;
                    v = l / (sqrt(m) * sqrt(n));
                } else {
                    const double sum = static_cast<double>(mi + ni - 2 * li) * inv_s2;
                    const double count = static_cast<double>(m128 ? (acc[3][i][j][q] >> 14) : acc[3][i][j][q]);
                    v = 1.0 / (sum / count + 1.0);
                }
                S[static_cast<int64_t>(a) * L + bb] = v;
                S[static_cast<int64_t>(bb) * L + a] = v;
            }
}

// Upper-triangle tiles (ta <= tb < T) in 16 x 16 super-tile groups, super-tiles column-major
// (measured on the ML-20M shape: 10 % less time than plain column-major order; an XCD-striped
// variant of the groups was slower).  The super-tile columns run from the last to the first:
// once every column group >= g is done, the rows of group g are complete (their entries right of
// the diagonal come from tiles (r, tb >= r), those left of it from the mirrored tiles (ta, r) of
// group g itself), which is what the streamed download (sims_streamed) relies on.  group_off[j]
// is the first tile of column group NS - 1 - j; group_off[NS] = the tile count.
constexpr int32_t kGroup = 16;
static std::vector<int2> tile_order(int32_t T, std::vector<size_t>* group_off = nullptr) {
    std::vector<int2> t;
    t.reserve(static_cast<size_t>(T) * (T + 1) / 2);
    const int32_t NS = (T + kGroup - 1) / kGroup;
    if (group_off) group_off->clear();
    for (int32_t sj = NS - 1; sj >= 0; --sj) {
        if (group_off) group_off->push_back(t.size());
        for (int32_t si = 0; si <= sj; ++si)
            for (int32_t b = sj * kGroup; b < std::min(T, (sj + 1) * kGroup); ++b)
                for (int32_t a = si * kGroup; a < std::min(T, (si + 1) * kGroup); ++a)
                    if (a <= b) t.push_back(make_int2(a, b));
    }
    if (group_off) group_off->push_back(t.size());
    return t;
}

// Multi-GPU sharding: the L rows are cut into 128-row blocks and part p of n owns the
// blocks t with t mod 2n in {p, 2n - 1 - p} (zig-zag: block t carries T - t tiles of the upper
// triangle, so every part gets near-equal work).  A part computes every pair (a, b), b >= a, whose
// row a lies in its blocks and writes both S[a][b] and S[b][a]: parts write disjoint entries, no
// collective is needed, and the union of all parts is the full matrix.
static bool part_owns(int32_t t, int32_t part, int32_t n_parts) {
    const int32_t m = t % (2 * n_parts);
    return m == part || m == 2 * n_parts - 1 - part;
}

// ---------------------------------------------------------------------------------------------
// K5: merge-order float64 kernel (any ratings; Pearson always)

// Per-row mean over ALL of the row's ratings in ID order (sim.go:49-62).
__global__ void row_mean_kernel(int32_t L, const int64_t* __restrict__ rowptr,
                                const double* __restrict__ r, double* __restrict__ mean) {
    const int32_t a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= L) return;
    double count = 0.0, sum = 0.0;
    for (int64_t t = rowptr[a]; t < rowptr[a + 1]; ++t) {
        sum += r[t];
        count += 1;
    }
    mean[a] = sum / count;
}

template <int KIND>  // 0 Cosine, 1 MSD, 2 Pearson, 3 SlopeOne dev[b][a] (NaN: nothing co-rated)
__device__ __forceinline__ double pair_sim(const double* __restrict__ dense_a, const uint8_t* __restrict__ has_a,
                                           double mean_a, int64_t bb, int64_t be,
                                           const int32_t* __restrict__ ids, const double* __restrict__ r,
                                           double mean_b) {
    if constexpr (KIND == 0) {
        double m = 0.0, n = 0.0, l = 0.0;
        for (int64_t t = bb; t < be; ++t) {
            const int32_t id = ids[t];
            if (has_a[id]) {
                const double ra = dense_a[id], rb = r[t];
                m += ra * ra;
                n += rb * rb;
                l += ra * rb;
            }
        }
        return l / (sqrt(m) * sqrt(n));
    } else if constexpr (KIND == 1) {
        double count = 0.0, sum = 0.0;
        for (int64_t t = bb; t < be; ++t) {
            const int32_t id = ids[t];
            if (has_a[id]) {
                const double d = dense_a[id] - r[t];
                sum += d * d;
                count++;
            }
        }
        return 1.0 / (sum / count + 1.0);
    } else if constexpr (KIND == 3) {  // slope_one.go:72-87 with i = b (walked), j = a (dense)
        double count = 0.0, sum = 0.0;
        for (int64_t t = bb; t < be; ++t) {
            const int32_t id = ids[t];
            if (has_a[id]) {
                count++;
                sum += r[t] - dense_a[id];
            }
        }
        return count > 0 ? sum / count : __builtin_nan("");
    } else {
        double m = 0.0, n = 0.0, l = 0.0;
        for (int64_t t = bb; t < be; ++t) {
            const int32_t id = ids[t];
            if (has_a[id]) {
                const double ra = dense_a[id] - mean_a;
                const double rb = r[t] - mean_b;
                m += ra * ra;
                n += rb * rb;
                l += ra * rb;
            }
        }
        return l / (sqrt(m) * sqrt(n));
    }
}

// Persistent workgroups walk the left rows a = blockIdx.x, blockIdx.x + gridDim.x, ...; row a lives
// densely in the workgroup's own global scratch row (R doubles + R flags), written and read only by
// that workgroup between barriers, then cleared.  One thread per partner b > a.
template <int KIND>
__global__ __launch_bounds__(256) void sims_merge_kernel(
    int32_t L, int32_t R, const int64_t* __restrict__ rowptr, const int32_t* __restrict__ ids,
    const double* __restrict__ r, const double* __restrict__ mean, double* __restrict__ scratch,
    uint8_t* __restrict__ scratch_has, double* __restrict__ S, const int32_t* __restrict__ rows,
    int32_t n_rows) {
    double* dense = scratch + static_cast<int64_t>(blockIdx.x) * R;
    uint8_t* has = scratch_has + static_cast<int64_t>(blockIdx.x) * R;
    for (int32_t x = blockIdx.x; x < n_rows; x += gridDim.x) {
        const int32_t a = rows[x];
        for (int64_t t = rowptr[a] + threadIdx.x; t < rowptr[a + 1]; t += blockDim.x) {
            dense[ids[t]] = r[t];
            has[ids[t]] = 1;
        }
        __syncthreads();
        const double ma = KIND == 2 ? mean[a] : 0.0;
        if (threadIdx.x == 0) S[static_cast<int64_t>(a) * L + a] = KIND == 3 ? 0.0 : __builtin_nan("");
        for (int32_t b = a + 1 + threadIdx.x; b < L; b += blockDim.x) {
            const double v = pair_sim<KIND>(dense, has, ma, rowptr[b], rowptr[b + 1], ids, r,
                                            KIND == 2 ? mean[b] : 0.0);
            if constexpr (KIND == 3) {  // dev[b][a] = v, dev[a][b] = -v; not co-rated: both 0
                const bool none = isnan(v);
                S[static_cast<int64_t>(b) * L + a] = none ? 0.0 : v;
                S[static_cast<int64_t>(a) * L + b] = none ? 0.0 : -v;
            } else {
                S[static_cast<int64_t>(a) * L + b] = v;  // NaN stays NaN (knn.go:205)
                S[static_cast<int64_t>(b) * L + a] = v;
            }
        }
        __syncthreads();
        for (int64_t t = rowptr[a] + threadIdx.x; t < rowptr[a + 1]; t += blockDim.x) has[ids[t]] = 0;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// host side

// RSGPU_KNN_TRACE=1: host-side phase times of rs_knn_sims on stderr (end-to-end study)
struct PhaseTrace {
    bool on = std::getenv("RSGPU_KNN_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "knn-trace %-12s %9.3f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t).count());
        t = t1;
    }
};
static thread_local PhaseTrace* g_trace = nullptr;  // set for the duration of one traced rs_knn_sims_part call
static void trace_mark(const char* what) {
    if (g_trace) g_trace->mark(what);
}

// The left rows handed to the kernels: rowptr rebased to 0, and the ids / ratings either the
// caller's own arrays (the MFMA path scatters them densely, so row order does not matter) or the
// ID-sorted copies of sort_rows (the merge path walks them in order).  scale: the int8 path's s
// (0 = not applicable), -1 = not decided yet.
struct SortedRows {
    std::vector<int64_t> rowptr;
    std::vector<int32_t> ids;
    std::vector<double> r;
    const int32_t* pid = nullptr;
    const double* pr = nullptr;
    int64_t nnz = 0;
    int scale = -1;
    void own() { pid = ids.data(); pr = r.data(); nnz = static_cast<int64_t>(ids.size()); }
};

// data.go:236-243 sorts(): each row ID-ascending (stable, so duplicates keep data order).  Rows
// already in order are copied as they are; the others sort 64-bit keys (id, position in the row),
// which are unique, so the order is the stable one.  Host threads take row ranges of near-equal
// rating counts.
static void sort_rows(int32_t L, const int64_t* rowptr, const int32_t* ids, const double* r,
                      SortedRows& out) {
    out.rowptr.assign(rowptr, rowptr + L + 1);
    const int64_t nnz = rowptr[L] - rowptr[0];
    out.ids.resize(nnz);
    out.r.resize(nnz);
    const int64_t o = rowptr[0];
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nt = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({16, hw, nnz / 65536 + 1})));
    std::vector<int32_t> cut(nt + 1, L);
    cut[0] = 0;
    for (int t = 1; t < nt; ++t)
        cut[t] = static_cast<int32_t>(std::lower_bound(rowptr, rowptr + L + 1, o + nnz * t / nt) - rowptr);
    auto work = [&](int t) {
        std::vector<uint64_t> key;
        for (int64_t a = cut[t]; a < cut[t + 1]; ++a) {
            const int64_t b = rowptr[a], e = rowptr[a + 1];
            if (std::is_sorted(ids + b, ids + e)) {
                std::copy(ids + b, ids + e, out.ids.begin() + (b - o));
                std::copy(r + b, r + e, out.r.begin() + (b - o));
                continue;
            }
            key.resize(e - b);
            for (int64_t x = b; x < e; ++x)  // ids are >= 0 (check_knn_csr)
                key[x - b] = (static_cast<uint64_t>(static_cast<uint32_t>(ids[x])) << 32) | static_cast<uint64_t>(x - b);
            std::sort(key.begin(), key.end());
            for (int64_t x = b; x < e; ++x) {
                const int64_t src = b + static_cast<int64_t>(key[x - b] & 0xFFFFFFFFu);
                out.ids[x - o] = ids[src];
                out.r[x - o] = r[src];
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (std::thread& x : th) x.join();
    for (auto& p : out.rowptr) p -= o;
    out.own();
}

// ratings exactly x / s, s in {1, 2}, |x| <= 11, and no repeated id inside a row -> MFMA path
static bool scale_ok(const SortedRows& sr, int s) {
    const int64_t n = sr.nnz;
    std::atomic<bool> any{false};
    parallel_ranges(n, 16, [&](int64_t t0, int64_t t1) {
        for (int64_t t = t0; t < t1 && !any.load(std::memory_order_relaxed); ++t) {
            const double x = sr.pr[t] * s;
            if (!(x == std::floor(x)) || x < 1.0 || x > 11.0) {  // 0 marks "not rated"
                any.store(true, std::memory_order_relaxed);
                return;
            }
        }
    });
    return !any.load();
}
static int int8_scale(const SortedRows& sr) {
    for (int s = 1; s <= 2; ++s)
        if (scale_ok(sr, s)) return s;
    return 0;
}

// A repeated id inside a row (any row order): one bitmap of the right ids per host thread, marked
// and cleared row by row.
static bool has_repeats(int32_t L, int32_t R, const SortedRows& sr) {
    std::atomic<bool> any{false};
    parallel_ranges(L, 16, [&](int64_t a0, int64_t a1) {
        std::vector<uint64_t> seen((static_cast<size_t>(R) + 63) / 64, 0);
        for (int64_t a = a0; a < a1 && !any.load(std::memory_order_relaxed); ++a) {
            const int64_t b = sr.rowptr[a], e = sr.rowptr[a + 1];
            int64_t t = b;
            for (; t < e; ++t) {
                const uint32_t id = static_cast<uint32_t>(sr.pid[t]);
                const uint64_t bit = uint64_t{1} << (id & 63);
                if (seen[id >> 6] & bit) break;
                seen[id >> 6] |= bit;
            }
            for (int64_t x = b; x < t; ++x) seen[static_cast<uint32_t>(sr.pid[x]) >> 6] = 0;
            if (t < e) {
                any.store(true, std::memory_order_relaxed);
                return;
            }
        }
    });
    return any.load();
}

// The rows for sims_device: the caller's arrays as they are when the int8 MFMA path applies
// (Cosine / MSD / SlopeOne on x / s ratings without repeated ids), the ID-sorted copy otherwise.
static void prepare_rows(int32_t kind, bool allow_mfma, int32_t L, int32_t R, const int64_t* rowptr,
                         const int32_t* ids, const double* r, SortedRows& out) {
    out.rowptr.assign(rowptr, rowptr + L + 1);
    for (auto& p : out.rowptr) p -= rowptr[0];
    out.pid = ids + rowptr[0];
    out.pr = r + rowptr[0];
    out.nnz = rowptr[L] - rowptr[0];
    out.scale = 0;
    if (kind != RS_SIM_PEARSON && allow_mfma) {
        const int sc = int8_scale(out);
        if (sc && !has_repeats(L, R, out)) {
            out.scale = sc;
            trace_mark("scale-check");
            return;
        }
    }
    trace_mark("scale-check");
    sort_rows(L, rowptr, ids, r, out);
    out.scale = 0;
    trace_mark("sort");
}

// ---------------------------------------------------------------------------------------------
// Streamed download of the MFMA path's Sims (rs_knn_sims, one part).  The tiles run as one launch
// per super-tile column group, last group first, round robin over two streams (the groups write
// disjoint entries, so consecutive launches overlap at their tails); after groups >= g are done,
// the rows of group g are complete (tile_order) and the copy engine moves them, in chunks of whole
// rows, into a pinned ring held by the ctx while the next groups compute.  Host threads copy each
// chunk from the ring into the caller's buffer as its DMA completes.  Only the first group's rows
// (the last to finish) are exposed after the kernels.
constexpr int kDlSlots = 16;
constexpr size_t kDlSlotBytes = size_t(16) << 20;
constexpr int kDlWorkers = 8;
// compute streams of the group launches: 3 measured 166 ms of kernels but 0.29 s of Fit wall
// against 170 ms / 0.26 s for 2 (rows complete later when more groups run at once)
constexpr int kDlCompute = 2;

static uint8_t* ctx_staging(rs_ctx* ctx) {
    if (!ctx->staging) {
        void* p = nullptr;
        RS_HIP(hipHostMalloc(&p, kDlSlots * kDlSlotBytes, hipHostMallocDefault));
        ctx->staging = std::shared_ptr<void>(p, [](void* q) { (void)hipHostFree(q); });
    }
    return static_cast<uint8_t*>(ctx->staging.get());
}

struct StreamSet {  // per-call streams and events, released on every path
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;
    ~StreamSet() {
        for (hipStream_t s : st) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
    hipStream_t stream() {
        hipStream_t s;
        RS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        st.push_back(s);
        return s;
    }
    hipEvent_t event() {
        hipEvent_t e;
        RS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ev.push_back(e);
        return e;
    }
};

template <typename Launch>
static void sims_streamed(rs_ctx* ctx, int32_t L, const std::vector<size_t>& group_off, Launch launch,
                          const double* dS, double* host) {
    const int32_t NG = static_cast<int32_t>(group_off.size()) - 1;
    const int64_t group_rows = static_cast<int64_t>(kGroup) * kTile;
    StreamSet ss;
    // kDlCompute compute streams (the ctx stream first) take the launches round robin
    const int NS = std::max(1, std::min(kDlCompute, NG));
    std::vector<hipStream_t> sk(NS, ctx->stream);
    for (int i = 1; i < NS; ++i) sk[i] = ss.stream();
    hipStream_t sC = ss.stream();
    std::vector<hipEvent_t> ev_g(NG);
    for (auto& e : ev_g) e = ss.event();
    kernel_span_begin(ctx);
    for (int i = 1; i < NS; ++i) RS_HIP(hipStreamWaitEvent(sk[i], ctx->k0, 0));
    for (int32_t j = 0; j < NG; ++j) {  // launch j = column group NG - 1 - j
        hipStream_t s = sk[j % NS];
        launch(group_off[j], group_off[j + 1] - group_off[j], s);
        RS_HIP(hipEventRecord(ev_g[NG - 1 - j], s));
    }
    for (int i = 1; i < NS; ++i) {
        hipEvent_t e = ss.event();
        RS_HIP(hipEventRecord(e, sk[i]));
        RS_HIP(hipStreamWaitEvent(sk[0], e, 0));
    }
    (void)hipEventRecord(ctx->k1, sk[0]);

    // chunks of whole rows, never crossing a group: groups NG-1 .. 0, rows ascending within
    struct Chunk { int64_t row0, rows; int32_t group; };
    std::vector<Chunk> chunks;
    const int64_t row_bytes = static_cast<int64_t>(L) * sizeof(double);
    const int64_t per = std::max<int64_t>(1, static_cast<int64_t>(kDlSlotBytes) / row_bytes);
    for (int32_t g = NG - 1; g >= 0; --g) {
        const int64_t r1 = std::min<int64_t>(L, (g + 1) * group_rows);
        for (int64_t r = g * group_rows; r < r1; r += per) chunks.push_back({r, std::min(per, r1 - r), g});
    }
    uint8_t* ring = ctx_staging(ctx);
    std::vector<hipEvent_t> ev_slot(kDlSlots);
    for (auto& e : ev_slot) e = ss.event();
    const int64_t NC = static_cast<int64_t>(chunks.size());
    std::atomic<int64_t> issued{0};                       // chunks whose DMA is enqueued
    std::vector<std::atomic<int64_t>> freed(kDlSlots);    // per slot: chunks copied out of it
    for (auto& f : freed) f.store(0);
    std::atomic<bool> failed{false};
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int W = static_cast<int>(std::min<unsigned>(kDlWorkers, hw));
    auto worker = [&](int w) {
        for (int64_t c = w; c < NC; c += W) {
            while (issued.load(std::memory_order_acquire) <= c) {
                if (failed.load()) return;
                std::this_thread::yield();
            }
            const int slot = static_cast<int>(c % kDlSlots);
            if (hipEventSynchronize(ev_slot[slot]) != hipSuccess) {
                failed.store(true);
                return;
            }
            std::memcpy(host + chunks[c].row0 * L, ring + slot * kDlSlotBytes,
                        static_cast<size_t>(chunks[c].rows * row_bytes));
            freed[slot].store(c / kDlSlots + 1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (int w = 0; w < W; ++w) th.emplace_back(worker, w);
    std::string err;
    try {
        int32_t waited = NG;
        for (int64_t c = 0; c < NC; ++c) {
            const int slot = static_cast<int>(c % kDlSlots);
            while (freed[slot].load(std::memory_order_acquire) < c / kDlSlots) {
                if (failed.load()) throw HipError{hipErrorUnknown, "streamed download: event wait failed"};
                std::this_thread::yield();
            }
            const int32_t g = chunks[c].group;
            if (g < waited) {  // every group >= g is done: the last one on each compute stream
                for (int32_t h = g; h < std::min(NG, g + NS); ++h) RS_HIP(hipStreamWaitEvent(sC, ev_g[h], 0));
                waited = g;
            }
            RS_HIP(hipMemcpyAsync(ring + slot * kDlSlotBytes, dS + chunks[c].row0 * L,
                                  static_cast<size_t>(chunks[c].rows * row_bytes), hipMemcpyDeviceToHost, sC));
            RS_HIP(hipEventRecord(ev_slot[slot], sC));
            issued.store(c + 1, std::memory_order_release);
        }
    } catch (const HipError& e) {
        failed.store(true);
        err = e.what;
    }
    for (std::thread& x : th) x.join();
    if (!err.empty() || failed.load()) throw HipError{hipErrorUnknown, err.empty() ? "streamed download failed" : err};
    float ms = 0.f;
    if (hipEventSynchronize(ctx->k1) == hipSuccess && hipEventElapsedTime(&ms, ctx->k0, ctx->k1) == hipSuccess)
        ctx->last_kernel_ms = ms;
}

// Returns true when the Sims already reached `host` (the streamed MFMA path, one part only);
// otherwise they are in dS for the caller to copy.
static bool sims_device(rs_ctx* ctx, int32_t kind, int32_t L, int32_t R, const SortedRows& sr,
                        bool allow_mfma, DevBuf<double>& dS, int32_t part = 0, int32_t n_parts = 1,
                        double* host = nullptr) {
    hipStream_t s = ctx->stream;
    const int64_t nnz = sr.nnz;
    dS.alloc(std::max<int64_t>(1, static_cast<int64_t>(L) * L));
    if (L == 0) return false;
    const int scale = sr.scale >= 0 ? sr.scale
                    : (kind != RS_SIM_PEARSON && allow_mfma && !has_repeats(L, R, sr)) ? int8_scale(sr) : 0;
    DevBuf<int64_t> drow(sr.rowptr.size());
    DevBuf<int32_t> dids(std::max<int64_t>(1, nnz));
    drow.upload(sr.rowptr.data(), sr.rowptr.size(), s);
    dids.upload(sr.pid, nnz, s);
    if (scale) {
        const int64_t ldk = ((static_cast<int64_t>(R) + kKBlock - 1) / kKBlock) * kKBlock;
        const int64_t Lp = ((static_cast<int64_t>(L) + kTile - 1) / kTile) * kTile;
        std::vector<int8_t> hx(nnz);
        parallel_ranges(nnz, 16, [&](int64_t t0, int64_t t1) {
            for (int64_t t = t0; t < t1; ++t) hx[t] = static_cast<int8_t>(sr.pr[t] * scale);
        });
        DevBuf<int8_t> dx(std::max<int64_t>(1, nnz));
        dx.upload(hx.data(), nnz, s);
        DevBuf<int8_t> X(Lp * ldk);
        RS_HIP(hipMemsetAsync(X.p, 0, X.n, s));
        hipLaunchKernelGGL(knn_scatter_kernel, dim3(L), dim3(256), 0, s, L, drow.p, dids.p, dx.p,
                           ldk, X.p);
        RS_HIP(hipGetLastError());
        RS_HIP(hipStreamSynchronize(s));
        trace_mark("dense-X");
        const int32_t T = static_cast<int32_t>(Lp / kTile);
        std::vector<size_t> group_off;
        std::vector<int2> order = tile_order(T, &group_off);
        if (n_parts > 1) {
            std::vector<int2> mine;
            for (const int2& t : order)
                if (part_owns(t.x, part, n_parts)) mine.push_back(t);
            order.swap(mine);
            if (order.empty()) return false;
        }
        DevBuf<int2> dtiles(order.size());
        dtiles.upload(order.data(), order.size(), s);
        // Cosine / MSD scale the sums by 1 / s^2; SlopeOne's differences by 1 / s
        const double inv_s2 = kind == RS_DEV_SLOPE_ONE ? 1.0 / scale : 1.0 / static_cast<double>(scale * scale);
        const size_t lds = 2 * kStageBytes;
        // K loop (RSGPU_KNN_PIPE, the variants the tests cross-check against each other):
        // 5 = default: software pipeline on eight waves (two per SIMD, 64 x 32 each), M derived from the X
        // fragments in registers, X loads rotated one step further ahead, and the LEAN operand forms
        // (M = -128 where rated: two VALU operations per dword instead of three; x^2 by two byte
        // permutes around the packed multiplies: five instead of six) -- 107 VALU per 12 MFMAs instead of
        // 139, 155 -> 148 ms on the ML-20M shape; 6 = the same without LEAN (also the default when a row
        // has 2^17 or more ratings: a co-rated count times 16384 must fit int32); 3 = without the
        // rotation; 4 = M staged in LDS; 0 = round 1 (four waves, phases in sequence).  Measured and
        // dropped in round 3 (profiles/r03_experiments/knn_k4.log): a third register set (loads two
        // whole steps ahead: no change), s_setprio for the second half of the waves (no change), x^2
        // stored in HBM beside X (196 ms: the doubled operand traffic costs more than the VALU it saves).
        int64_t max_deg = 0;
        for (int32_t a = 0; a < L; ++a) max_deg = std::max(max_deg, sr.rowptr[a + 1] - sr.rowptr[a]);
        const bool lean_ok = max_deg < (int64_t{1} << 17);
        const char* pipe_env = std::getenv("RSGPU_KNN_PIPE");
        int pipe = (pipe_env && (pipe_env[0] == '0' || pipe_env[0] == '3' || pipe_env[0] == '4' || pipe_env[0] == '6'))
                       ? pipe_env[0] - '0' : 5;
        if (pipe == 5 && !lean_ok) pipe = 6;
        for (const void* f : {reinterpret_cast<const void*>(&knn_sims_mfma_kernel<0, 0>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<1, 0>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<2, 0>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<0, 2, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<1, 2, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<2, 2, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<0, 1, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<1, 1, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<2, 1, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<0, 2, 1, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<1, 2, 1, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<2, 2, 1, 1>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<0, 2, 1, 1, true>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<1, 2, 1, 1, true>),
                              reinterpret_cast<const void*>(&knn_sims_mfma_kernel<2, 2, 1, 1, true>)})
            RS_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
        auto launch = [&](size_t first, size_t count, hipStream_t st) {
            if (!count) return;
            const dim3 grid(static_cast<uint32_t>(count));
            auto go = [&](auto kern, int threads) {
                hipLaunchKernelGGL(kern, grid, dim3(threads), lds, st, X.p, ldk, L, dtiles.p + first, inv_s2, dS.p);
            };
            auto by_pipe = [&](auto k0, auto k3, auto k4, auto k5, auto k6) {
                pipe == 0 ? go(k0, 256) : pipe == 3 ? go(k3, 512) : pipe == 4 ? go(k4, 512) : pipe == 6 ? go(k6, 512)
                          : go(k5, 512);
            };
            if (kind == RS_SIM_COSINE)
                by_pipe(knn_sims_mfma_kernel<0, 0>, knn_sims_mfma_kernel<0, 2, 1>, knn_sims_mfma_kernel<0, 1, 1>,
                        knn_sims_mfma_kernel<0, 2, 1, 1, true>, knn_sims_mfma_kernel<0, 2, 1, 1>);
            else if (kind == RS_SIM_MSD)
                by_pipe(knn_sims_mfma_kernel<1, 0>, knn_sims_mfma_kernel<1, 2, 1>, knn_sims_mfma_kernel<1, 1, 1>,
                        knn_sims_mfma_kernel<1, 2, 1, 1, true>, knn_sims_mfma_kernel<1, 2, 1, 1>);
            else
                by_pipe(knn_sims_mfma_kernel<2, 0>, knn_sims_mfma_kernel<2, 2, 1>, knn_sims_mfma_kernel<2, 1, 1>,
                        knn_sims_mfma_kernel<2, 2, 1, 1, true>, knn_sims_mfma_kernel<2, 2, 1, 1>);
            RS_HIP(hipGetLastError());
        };
        if (host && n_parts == 1) {
            trace_mark("tiles");
            sims_streamed(ctx, L, group_off, launch, dS.p, host);
            trace_mark("streamed");
            return true;
        }
        kernel_span_begin(ctx);
        launch(0, order.size(), s);
        kernel_span_end(ctx);
        return false;
    }
    DevBuf<double> dr(std::max<int64_t>(1, nnz)), dmean(L);
    dr.upload(sr.pr, nnz, s);
    hipLaunchKernelGGL(row_mean_kernel, dim3((L + 255) / 256), dim3(256), 0, s, L, drow.p, dr.p,
                       dmean.p);
    std::vector<int32_t> rows;
    for (int32_t a = 0; a < L; ++a)
        if (n_parts == 1 || part_owns(a / kTile, part, n_parts)) rows.push_back(a);
    if (rows.empty()) return false;
    DevBuf<int32_t> drows(rows.size());
    drows.upload(rows.data(), rows.size(), s);
    const int32_t n_rows = static_cast<int32_t>(rows.size());
    const int32_t grid = std::min<int32_t>(n_rows, 2048);
    DevBuf<double> scratch(static_cast<int64_t>(std::max(1, R)) * grid);
    DevBuf<uint8_t> scratch_has(static_cast<int64_t>(std::max(1, R)) * grid);
    RS_HIP(hipMemsetAsync(scratch_has.p, 0, scratch_has.n, s));
    RS_HIP(hipStreamSynchronize(s));
    kernel_span_begin(ctx);
    if (kind == RS_SIM_COSINE)
        hipLaunchKernelGGL(sims_merge_kernel<0>, dim3(grid), dim3(256), 0, s, L, R, drow.p, dids.p, dr.p, dmean.p, scratch.p, scratch_has.p, dS.p, drows.p, n_rows);
    else if (kind == RS_SIM_MSD)
        hipLaunchKernelGGL(sims_merge_kernel<1>, dim3(grid), dim3(256), 0, s, L, R, drow.p, dids.p, dr.p, dmean.p, scratch.p, scratch_has.p, dS.p, drows.p, n_rows);
    else if (kind == RS_SIM_PEARSON)
        hipLaunchKernelGGL(sims_merge_kernel<2>, dim3(grid), dim3(256), 0, s, L, R, drow.p, dids.p, dr.p, dmean.p, scratch.p, scratch_has.p, dS.p, drows.p, n_rows);
    else
        hipLaunchKernelGGL(sims_merge_kernel<3>, dim3(grid), dim3(256), 0, s, L, R, drow.p, dids.p, dr.p, dmean.p, scratch.p, scratch_has.p, dS.p, drows.p, n_rows);
    RS_HIP(hipGetLastError());
    kernel_span_end(ctx);
    return false;
}

// ---------------------------------------------------------------------------------------------
// KNN.Predict on the device (core/knn.go:75-141).  One wave per (left, right)
// query: candidates are RightRatings[right] (data order) with a non-NaN similarity (knn.go:93-99);
// at most min_k of them -> GlobalMean (knn.go:102-104); otherwise the top min(k, count) by
// (similarity desc, position asc) -- the documented tie rule for the reference's unstable
// sort.Sort (knn.go:107-108) -- are taken one per round by a wave arg-max below the previous pick,
// and lane 0 accumulates weightSum / weightRating in exactly that order with the type-specific
// centring (knn.go:116-140), so every output is bitwise equal to the restatement.
constexpr int kPredCache = 4096;  // candidate similarities cached in LDS per query

__global__ __launch_bounds__(64) void knn_predict_kernel(
    const double* __restrict__ S, int32_t L, int32_t n_right, const int64_t* __restrict__ rrp,
    const int32_t* __restrict__ rids, const double* __restrict__ rr, const double* __restrict__ means,
    const double* __restrict__ stddevs, const double* __restrict__ bias, double gmean, int32_t type,
    int32_t k, int32_t min_k, int64_t n, const int32_t* __restrict__ left,
    const int32_t* __restrict__ right, double* __restrict__ out) {
    __shared__ double cache[kPredCache];
    const int64_t qi = blockIdx.x;
    if (qi >= n) return;
    const int lane = threadIdx.x;
    const int32_t li = left[qi], ri = right[qi];
    if (li < 0 || li >= L || ri < 0 || ri >= n_right) {  // knn.go:89-91
        if (lane == 0) out[qi] = gmean;
        return;
    }
    const double* srow = S + static_cast<int64_t>(li) * L;
    const int64_t b = rrp[ri];
    const int32_t m = static_cast<int32_t>(rrp[ri + 1] - b);
    auto sim_at = [&](int32_t t) { return t < kPredCache ? cache[t] : srow[rids[b + t]]; };
    int32_t cnt = 0;
    for (int32_t t = lane; t < m; t += 64) {
        const double v = srow[rids[b + t]];
        if (t < kPredCache) cache[t] = v;
        cnt += !isnan(v);
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    __syncthreads();
    if (cnt <= min_k) {
        if (lane == 0) out[qi] = gmean;
        return;
    }
    const int32_t nn = min(k, cnt);
    double ps = 0.0;
    int32_t pp = -1;  // previous pick; -1: none yet
    double weightSum = 0.0, weightRating = 0.0;
    for (int32_t j = 0; j < nn; ++j) {
        bool found = false;
        double bs = 0.0;
        int32_t bp = 0;
        for (int32_t t = lane; t < m; t += 64) {
            const double v = sim_at(t);
            if (isnan(v)) continue;
            const bool below = pp < 0 || v < ps || (v == ps && t > pp);
            if (below && (!found || v > bs)) {  // strided t ascending: ties keep the first
                found = true;
                bs = v;
                bp = t;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            const int of = __shfl_xor(static_cast<int>(found), off);
            const double os = __shfl_xor(bs, off);
            const int32_t op = __shfl_xor(bp, off);
            if (of && (!found || os > bs || (os == bs && op < bp))) {
                found = true;
                bs = os;
                bp = op;
            }
        }
        ps = bs;
        pp = bp;
        if (lane == 0) {  // knn.go:118-130 in pick order
            const int32_t id = rids[b + bp];
            weightSum += bs;
            double rating = rr[b + bp];
            if (type == 1) rating -= means[id];
            else if (type == 2) rating = (rating - means[id]) / stddevs[id];
            else if (type == 3) rating -= bias[id];
            weightRating += bs * rating;
        }
    }
    if (lane == 0) {
        double prediction = weightRating / weightSum;  // knn.go:131-139
        if (type == 1) prediction += means[li];
        else if (type == 3) prediction += bias[li];
        else if (type == 2) {
            prediction *= stddevs[li];
            prediction += means[li];
        }
        out[qi] = prediction;
    }
}

// ---- KNN.Predict with the reference's tie order (RS_TIE_GO_SORT, the default) --------------------------------
// knn.go:107-108 orders the candidates with Go 1.24's sort.Sort -- pdqsort, not stable -- so among equal
// similarities (ML-100K has ~293k pairs tied at exactly 1.0) the order, the top-k boundary and the
// summation order of knn.go:118-130 are whatever its exact Less / Swap sequence leaves.  GoSort restates that
// sequence (sort/zsortinterface.go) call for call on one lane; the recursion on the smaller part becomes an
// explicit stack (depth <= log2 n).  Less(i, j) = sims_i > sims_j (knn.go:43-45); Swap moves a candidate's
// similarity and position together.  oracle/oracle.c and host/gosort.hpp restate the same algorithm.
struct GoSort {
    double* s;
    int32_t* p;
    __device__ bool less(int32_t i, int32_t j) const { return s[i] > s[j]; }
    __device__ void swap(int32_t i, int32_t j) const {
        const double a = s[i];
        s[i] = s[j];
        s[j] = a;
        const int32_t b = p[i];
        p[i] = p[j];
        p[j] = b;
    }
    __device__ static int bits_len(uint32_t x) { return x ? 32 - __clz(static_cast<int>(x)) : 0; }
    __device__ void insertion(int32_t a, int32_t b) const {
        for (int32_t i = a + 1; i < b; ++i)
            for (int32_t j = i; j > a && less(j, j - 1); --j) swap(j, j - 1);
    }
    __device__ void sift_down(int32_t lo, int32_t hi, int32_t first) const {
        int32_t root = lo;
        for (;;) {
            int32_t child = 2 * root + 1;
            if (child >= hi) return;
            if (child + 1 < hi && less(first + child, first + child + 1)) ++child;
            if (!less(first + root, first + child)) return;
            swap(first + root, first + child);
            root = child;
        }
    }
    __device__ void heap_sort(int32_t a, int32_t b) const {
        const int32_t first = a, lo = 0, hi = b - a;
        for (int32_t i = (hi - 1) / 2; i >= 0; --i) sift_down(i, hi, first);
        for (int32_t i = hi - 1; i >= 0; --i) {
            swap(first, first + i);
            sift_down(lo, i, first);
        }
    }
    __device__ void order2(int32_t& a, int32_t& b, int& swaps) const {
        if (less(b, a)) {
            const int32_t t = a;
            a = b;
            b = t;
            ++swaps;
        }
    }
    __device__ int32_t median(int32_t a, int32_t b, int32_t c, int& swaps) const {
        order2(a, b, swaps);
        order2(b, c, swaps);
        order2(a, b, swaps);
        return b;
    }
    __device__ int32_t choose_pivot(int32_t a, int32_t b, int& hint) const {  // hint: 0 unknown, 1 inc, 2 dec
        const int32_t l = b - a;
        int swaps = 0;
        int32_t i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
        if (l >= 8) {
            if (l >= 50) {  // Tukey ninther
                i = median(i - 1, i, i + 1, swaps);
                j = median(j - 1, j, j + 1, swaps);
                k = median(k - 1, k, k + 1, swaps);
            }
            j = median(i, j, k, swaps);
        }
        hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
        return j;
    }
    __device__ bool partial_insertion(int32_t a, int32_t b) const {
        int32_t i = a + 1;
        for (int step = 0; step < 5; ++step) {
            while (i < b && !less(i, i - 1)) ++i;
            if (i == b) return true;
            if (b - a < 50) return false;
            swap(i, i - 1);
            if (i - a >= 2)
                for (int32_t j = i - 1; j >= 1; --j) {
                    if (!less(j, j - 1)) break;
                    swap(j, j - 1);
                }
            if (b - i >= 2)
                for (int32_t j = i + 1; j < b; ++j) {
                    if (!less(j, j - 1)) break;
                    swap(j, j - 1);
                }
        }
        return false;
    }
    __device__ void break_patterns(int32_t a, int32_t b) const {
        const int32_t length = b - a;
        if (length < 8) return;
        uint64_t r = static_cast<uint64_t>(length);  // xorshift seeded with the length
        const uint64_t modulus = uint64_t{1} << bits_len(static_cast<uint32_t>(length));
        const int32_t idx = a + (length / 4) * 2 - 1;
        for (int t = 0; t < 3; ++t) {
            r ^= r << 13;
            r ^= r >> 7;
            r ^= r << 17;
            int32_t other = static_cast<int32_t>(r & (modulus - 1));
            if (other >= length) other -= length;
            swap(idx - 1 + t, a + other);
        }
    }
    __device__ int32_t partition_equal(int32_t a, int32_t b, int32_t pivot) const {
        swap(a, pivot);
        int32_t i = a + 1, j = b - 1;
        for (;;) {
            while (i <= j && !less(a, i)) ++i;
            while (i <= j && less(a, j)) --j;
            if (i > j) break;
            swap(i, j);
            ++i;
            --j;
        }
        return i;
    }
    __device__ int32_t partition(int32_t a, int32_t b, int32_t pivot, bool& already) const {
        swap(a, pivot);
        int32_t i = a + 1, j = b - 1;
        while (i <= j && less(i, a)) ++i;
        while (i <= j && !less(j, a)) --j;
        if (i > j) {
            swap(j, a);
            already = true;
            return j;
        }
        swap(i, j);
        ++i;
        --j;
        for (;;) {
            while (i <= j && less(i, a)) ++i;
            while (i <= j && !less(j, a)) --j;
            if (i > j) break;
            swap(i, j);
            ++i;
            --j;
        }
        swap(j, a);
        already = false;
        return j;
    }
    // sort.Sort over [0, n): pdqsort's loop, its recursive call on the smaller part as a pushed frame
    __device__ void sort(int32_t n) const {
        if (n <= 1) return;
        struct Frame { int32_t a, b, limit; bool wb, wp; };
        Frame st[40];
        int sp = 0;
        Frame f{0, n, bits_len(static_cast<uint32_t>(n)), true, true};
        for (;;) {
            bool done = false;
            for (;;) {  // one pdqsort(data, a, b, limit) activation
                const int32_t length = f.b - f.a;
                if (length <= 12) {
                    insertion(f.a, f.b);
                    done = true;
                    break;
                }
                if (f.limit == 0) {
                    heap_sort(f.a, f.b);
                    done = true;
                    break;
                }
                if (!f.wb) {
                    break_patterns(f.a, f.b);
                    --f.limit;
                }
                int hint = 0;
                int32_t pivot = choose_pivot(f.a, f.b, hint);
                if (hint == 2) {
                    for (int32_t i = f.a, j = f.b - 1; i < j; ++i, --j) swap(i, j);
                    pivot = (f.b - 1) - (pivot - f.a);
                    hint = 1;
                }
                if (f.wb && f.wp && hint == 1 && partial_insertion(f.a, f.b)) {
                    done = true;
                    break;
                }
                if (f.a > 0 && !less(f.a - 1, pivot)) {
                    f.a = partition_equal(f.a, f.b, pivot);
                    continue;
                }
                bool already = false;
                const int32_t mid = partition(f.a, f.b, pivot, already);
                f.wp = already;
                const int32_t left_len = mid - f.a, right_len = f.b - mid, threshold = length / 8;
                Frame child;
                if (left_len < right_len) {
                    f.wb = left_len >= threshold;
                    child = Frame{f.a, mid, f.limit, true, true};
                    f.a = mid + 1;
                } else {
                    f.wb = right_len >= threshold;
                    child = Frame{mid + 1, f.b, f.limit, true, true};
                    f.b = mid;
                }
                st[sp++] = f;  // the caller continues after the child returns
                f = child;
            }
            if (done) {
                if (sp == 0) return;
                f = st[--sp];
            }
        }
    }
};

constexpr int kGoSortLds = 4096;  // candidates sorted in LDS; more go to the per-block global scratch

// One wave per query (grid-stride): the non-NaN candidates in RightRatings order (knn.go:95-99) are
// compacted by ballot into (similarity, position) arrays, lane 0 runs GoSort on them, and the first
// min(k, n) are accumulated in that order (knn.go:111-130), so the result is bitwise the reference's.
__global__ __launch_bounds__(64) void knn_predict_gosort_kernel(
    const double* __restrict__ S, int32_t L, int32_t n_right, const int64_t* __restrict__ rrp,
    const int32_t* __restrict__ rids, const double* __restrict__ rr, const double* __restrict__ means,
    const double* __restrict__ stddevs, const double* __restrict__ bias, double gmean, int32_t type,
    int32_t k, int32_t min_k, int64_t n, const int32_t* __restrict__ left,
    const int32_t* __restrict__ right, double* __restrict__ out, double* __restrict__ gs,
    int32_t* __restrict__ gp, int64_t scratch) {
    __shared__ double ls[kGoSortLds];
    __shared__ int32_t lp[kGoSortLds];
    const int lane = threadIdx.x;
    for (int64_t qi = blockIdx.x; qi < n; qi += gridDim.x) {
        const int32_t li = left[qi], ri = right[qi];
        if (li < 0 || li >= L || ri < 0 || ri >= n_right) {  // knn.go:89-91
            if (lane == 0) out[qi] = gmean;
            continue;
        }
        const double* srow = S + static_cast<int64_t>(li) * L;
        const int64_t b = rrp[ri];
        const int32_t m = static_cast<int32_t>(rrp[ri + 1] - b);
        const bool in_lds = m <= kGoSortLds;
        double* sv = in_lds ? ls : gs + blockIdx.x * scratch;
        int32_t* pv = in_lds ? lp : gp + blockIdx.x * scratch;
        int32_t cnt = 0;  // wave-uniform
        for (int32_t t0 = 0; t0 < m; t0 += 64) {
            const int32_t t = t0 + lane;
            const double v = t < m ? srow[rids[b + t]] : 0.0;
            const bool ok = t < m && !isnan(v);
            const uint64_t mask = __ballot(ok);
            if (ok) {
                const int32_t at = cnt + __popcll(mask & ((uint64_t{1} << lane) - 1));
                sv[at] = v;
                pv[at] = t;
            }
            cnt += __popcll(mask);
        }
        __syncthreads();
        if (cnt <= min_k) {  // knn.go:102-104
            if (lane == 0) out[qi] = gmean;
            __syncthreads();
            continue;
        }
        if (lane == 0) {
            GoSort{sv, pv}.sort(cnt);  // knn.go:107-108
            const int32_t nn = min(k, cnt);
            double weightSum = 0.0, weightRating = 0.0;
            for (int32_t j = 0; j < nn; ++j) {  // knn.go:118-130
                const int32_t t = pv[j], id = rids[b + t];
                weightSum += sv[j];
                double rating = rr[b + t];
                if (type == 1) rating -= means[id];
                else if (type == 2) rating = (rating - means[id]) / stddevs[id];
                else if (type == 3) rating -= bias[id];
                weightRating += sv[j] * rating;
            }
            double prediction = weightRating / weightSum;  // knn.go:131-139
            if (type == 1) prediction += means[li];
            else if (type == 3) prediction += bias[li];
            else if (type == 2) {
                prediction *= stddevs[li];
                prediction += means[li];
            }
            out[qi] = prediction;
        }
        __syncthreads();  // the next query overwrites the arrays
    }
}

// SlopeOne.Predict (core/slope_one.go:21-45), one thread per query, bitwise: prediction = the user's
// mean rating (means(), data.go:222-235, precomputed by row_mean_kernel in the same order) or the
// global mean for an unknown user; for a known (user, item) the user's ratings are walked in data
// order (TrainSet.UserRatings) adding dev[item][j], and sum / count is added.
__global__ __launch_bounds__(256) void slope_one_predict_kernel(
    const double* __restrict__ dev, int32_t L, int32_t n_users, const int64_t* __restrict__ urp,
    const int32_t* __restrict__ uitems, const double* __restrict__ umean, double gmean, int64_t n,
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, double* __restrict__ out) {
    const int64_t q = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (q >= n) return;
    const int32_t u = users[q], i = items[q];
    const bool ku = u >= 0 && u < n_users, ki = i >= 0 && i < L;
    double prediction = ku ? umean[u] : gmean;
    if (ku && ki) {
        const double* row = dev + static_cast<int64_t>(i) * L;
        double sum = 0.0, count = 0.0;
        for (int64_t t = urp[u]; t < urp[u + 1]; ++t) {
            sum += row[uitems[t]];
            count++;
        }
        if (count > 0) prediction += sum / count;
    }
    out[q] = prediction;
}

// Validates a left CSR (rowptr monotone, ids in [0, n_right)) for rs_knn_sims / plan creation.
static int check_knn_csr(rs_ctx* ctx, int32_t n_left, int32_t n_right, const int64_t* rowptr,
                         const int32_t* ids, const double* ratings) {
    if (n_left < 0 || n_right < 0 || !rowptr) return set_error(ctx, RS_ERR_INVALID, "bad knn arguments");
    const int64_t nnz = rowptr[n_left] - rowptr[0];
    if (nnz > 0 && (!ids || !ratings)) return set_error(ctx, RS_ERR_INVALID, "ids/ratings NULL");
    for (int32_t a = 0; a < n_left; ++a)
        if (rowptr[a + 1] < rowptr[a]) return set_error(ctx, RS_ERR_INVALID, "rowptr not monotone");
    for (int64_t t = rowptr[0]; t < rowptr[n_left]; ++t)
        if (ids[t] < 0 || ids[t] >= n_right) return set_error(ctx, RS_ERR_INVALID, "id out of range");
    return RS_OK;
}

}  // namespace rs

extern "C" int rs_knn_sims_part(rs_ctx* ctx, int32_t kind, int32_t n_left, int32_t n_right,
                                const int64_t* rowptr, const int32_t* ids, const double* ratings,
                                int32_t part, int32_t n_parts, double* sims) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        rs::drop_fit_cache(ctx);
        if (kind < RS_SIM_COSINE || kind > RS_DEV_SLOPE_ONE)
            return rs::set_error(ctx, RS_ERR_INVALID, "unknown similarity kind");
        if (n_parts < 1 || part < 0 || part >= n_parts)
            return rs::set_error(ctx, RS_ERR_INVALID, "part must be in [0, n_parts)");
        if (n_left > 0 && !sims) return rs::set_error(ctx, RS_ERR_INVALID, "sims is NULL");
        rs::PhaseTrace tr;
        rs::g_trace = tr.on ? &tr : nullptr;
        struct Reset { ~Reset() { rs::g_trace = nullptr; } } reset_trace;
        const int st = rs::check_knn_csr(ctx, n_left, n_right, rowptr, ids, ratings);
        if (st != RS_OK) return st;
        rs::SortedRows sr;
        tr.mark("check");
        const char* env = std::getenv("RSGPU_KNN_NO_MFMA");
        rs::prepare_rows(kind, !(env && env[0] == '1'), n_left, n_right, rowptr, ids, ratings, sr);
        rs::DevBuf<double> dS;
        const char* nostream = std::getenv("RSGPU_KNN_NO_STREAM");  // A/B switch: one launch, one copy
        const bool done = rs::sims_device(ctx, kind, n_left, n_right, sr, !(env && env[0] == '1'), dS, part,
                                          n_parts, (nostream && nostream[0] == '1') ? nullptr : sims);
        hipStream_t s = ctx->stream;
        if (done) {
        } else if (n_parts == 1) {
            dS.download(sims, static_cast<int64_t>(n_left) * n_left, s);
        } else {  // the part's rows from their diagonal block rightwards, and the mirrored columns
            const size_t pitch = static_cast<size_t>(n_left) * sizeof(double);
            for (int32_t t = 0; t * rs::kTile < n_left; ++t) {
                if (!rs::part_owns(t, part, n_parts)) continue;
                const int32_t a0 = t * rs::kTile, na = std::min(rs::kTile, n_left - a0);
                const size_t off = static_cast<size_t>(a0) * n_left + a0;
                RS_HIP(hipMemcpy2DAsync(sims + off, pitch, dS.p + off, pitch, (n_left - a0) * sizeof(double),
                                        na, hipMemcpyDeviceToHost, s));
                RS_HIP(hipMemcpy2DAsync(sims + off, pitch, dS.p + off, pitch, na * sizeof(double),
                                        n_left - a0, hipMemcpyDeviceToHost, s));
            }
        }
        RS_HIP(hipStreamSynchronize(s));
        tr.mark("download");
        dS.release();
        tr.mark("free");
        return RS_OK;
    });
}

extern "C" int rs_knn_sims(rs_ctx* ctx, int32_t kind, int32_t n_left, int32_t n_right,
                           const int64_t* rowptr, const int32_t* ids, const double* ratings,
                           double* sims) {
    return rs_knn_sims_part(ctx, kind, n_left, n_right, rowptr, ids, ratings, 0, 1, sims);
}

extern "C" int rs_knn_part_blocks(int32_t n_left, int32_t part, int32_t n_parts, int32_t* owned) {
    if (n_left < 0 || n_parts < 1 || part < 0 || part >= n_parts || !owned) return RS_ERR_INVALID;
    const int32_t T = (n_left + rs::kTile - 1) / rs::kTile;
    for (int32_t t = 0; t < T; ++t) owned[t] = rs::part_owns(t, part, n_parts) ? 1 : 0;
    return RS_OK;
}

extern "C" int rs_sim_pair(rs_ctx* ctx, int32_t kind, int64_t na, const int32_t* a_ids,
                           const double* a_r, int64_t nb, const int32_t* b_ids, const double* b_r,
                           double* out) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        if (!out || na < 0 || nb < 0 || (na && (!a_ids || !a_r)) || (nb && (!b_ids || !b_r)))
            return rs::set_error(ctx, RS_ERR_INVALID, "bad sim_pair arguments");
        if (kind < RS_SIM_COSINE || kind > RS_SIM_PEARSON)
            return rs::set_error(ctx, RS_ERR_INVALID, "unknown similarity kind");
        // a two-row KNN problem on the merge kernel: S[0][1] = sim(a, b)
        int32_t R = 1;
        for (int64_t t = 0; t < na; ++t) R = std::max(R, a_ids[t] + 1);
        for (int64_t t = 0; t < nb; ++t) R = std::max(R, b_ids[t] + 1);
        std::vector<int64_t> rowptr = {0, na, na + nb};
        std::vector<int32_t> ids(a_ids, a_ids + na);
        ids.insert(ids.end(), b_ids, b_ids + nb);
        std::vector<double> r(a_r, a_r + na);
        r.insert(r.end(), b_r, b_r + nb);
        for (int32_t t : ids)
            if (t < 0) return rs::set_error(ctx, RS_ERR_INVALID, "negative id");
        rs::SortedRows sr;
        sr.rowptr = rowptr;
        sr.ids = ids;
        sr.r = r;  // inputs are ID-ascending already (SortedIdRatings)
        sr.own();
        rs::DevBuf<double> dS;
        rs::sims_device(ctx, kind, 2, R, sr, false, dS);
        double S[4];
        dS.download(S, 4, ctx->stream);
        RS_HIP(hipStreamSynchronize(ctx->stream));
        *out = S[1];
        return RS_OK;
    });
}

// ------------------------------------------------------------------------------------------------
// Device-resident KNN (similarities stay in HBM; Predict runs on them)

struct rs_knn_plan {
    rs_ctx* ctx = nullptr;
    int32_t L = 0;
    int32_t kind = 0;
    int32_t tie = RS_TIE_GO_SORT;  // rs_knn_plan_set_tie_order
    rs::DevBuf<double> S;
};

extern "C" int rs_knn_plan_set_tie_order(rs_knn_plan* pl, int32_t tie) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (tie != RS_TIE_GO_SORT && tie != RS_TIE_STABLE) return rs::set_error(pl->ctx, RS_ERR_INVALID, "unknown tie order");
    pl->tie = tie;
    return RS_OK;
}

extern "C" int rs_knn_plan_create(rs_ctx* ctx, int32_t kind, int32_t n_left, int32_t n_right,
                                  const int64_t* rowptr, const int32_t* ids, const double* ratings,
                                  rs_knn_plan** out) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        rs::drop_fit_cache(ctx);
        if (!out) return rs::set_error(ctx, RS_ERR_INVALID, "out is NULL");
        *out = nullptr;
        if (kind < RS_SIM_COSINE || kind > RS_DEV_SLOPE_ONE)
            return rs::set_error(ctx, RS_ERR_INVALID, "unknown similarity kind");
        const int st = rs::check_knn_csr(ctx, n_left, n_right, rowptr, ids, ratings);
        if (st != RS_OK) return st;
        auto* pl = new rs_knn_plan();
        try {
            pl->ctx = ctx;
            pl->L = n_left;
            pl->kind = kind;
            rs::SortedRows sr;
            const char* env = std::getenv("RSGPU_KNN_NO_MFMA");
            rs::prepare_rows(kind, !(env && env[0] == '1'), n_left, n_right, rowptr, ids, ratings, sr);
            rs::sims_device(ctx, kind, n_left, n_right, sr, !(env && env[0] == '1'), pl->S);
            RS_HIP(hipStreamSynchronize(ctx->stream));
        } catch (...) {
            delete pl;
            throw;
        }
        *out = pl;
        return RS_OK;
    });
}

extern "C" void rs_knn_plan_destroy(rs_knn_plan* pl) {
    if (!pl) return;
    (void)hipSetDevice(pl->ctx->device);
    delete pl;
}

extern "C" int rs_knn_plan_sims(rs_knn_plan* pl, double* sims) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (pl->L > 0 && !sims) return rs::set_error(pl->ctx, RS_ERR_INVALID, "sims is NULL");
        pl->S.download(sims, static_cast<int64_t>(pl->L) * pl->L, pl->ctx->stream);
        RS_HIP(hipStreamSynchronize(pl->ctx->stream));
        return RS_OK;
    });
}

extern "C" int rs_knn_plan_predict(rs_knn_plan* pl, int32_t type, int32_t n_right,
                                   const int64_t* right_rowptr, const int32_t* right_ids,
                                   const double* right_r, const double* means,
                                   const double* stddevs, const double* bias, double global_mean,
                                   int32_t k, int32_t min_k, int64_t n, const int32_t* left,
                                   const int32_t* right, double* out) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    rs_ctx* ctx = pl->ctx;
    return rs_guard(ctx, [&]() -> int {
        if (type < 0 || type > 3) return rs::set_error(ctx, RS_ERR_INVALID, "unknown KNN type");
        if (n < 0 || n > INT32_MAX || (n > 0 && (!left || !right || !out)) || k < 0)
            return rs::set_error(ctx, RS_ERR_INVALID, "bad predict arguments");
        if ((type == 1 || type == 2) && !means) return rs::set_error(ctx, RS_ERR_INVALID, "means NULL");
        if (type == 2 && !stddevs) return rs::set_error(ctx, RS_ERR_INVALID, "stddevs NULL");
        if (type == 3 && !bias) return rs::set_error(ctx, RS_ERR_INVALID, "bias NULL");
        const int st = rs::check_knn_csr(ctx, n_right, pl->L, right_rowptr, right_ids, right_r);
        if (st != RS_OK) return st;
        if (n == 0) return RS_OK;
        hipStream_t s = ctx->stream;
        const int64_t base = right_rowptr[0], nnz = right_rowptr[n_right] - base;
        std::vector<int64_t> rp(right_rowptr, right_rowptr + n_right + 1);
        for (auto& x : rp) x -= base;
        rs::DevBuf<int64_t> drp(rp.size());
        rs::DevBuf<int32_t> dids(std::max<int64_t>(1, nnz)), dl(n), dr(n);
        rs::DevBuf<double> drr(std::max<int64_t>(1, nnz)), dout(n);
        rs::DevBuf<double> dm(means ? pl->L : 0), dsd(stddevs ? pl->L : 0), db(bias ? pl->L : 0);
        drp.upload(rp.data(), rp.size(), s);
        dids.upload(right_ids + base, nnz, s);
        drr.upload(right_r + base, nnz, s);
        dl.upload(left, n, s);
        dr.upload(right, n, s);
        if (means) dm.upload(means, pl->L, s);
        if (stddevs) dsd.upload(stddevs, pl->L, s);
        if (bias) db.upload(bias, pl->L, s);
        rs::kernel_span_begin(ctx);
        if (pl->tie == RS_TIE_GO_SORT) {
            int64_t mmax = 0;  // rows past the LDS arrays sort in a per-block global scratch
            for (int32_t x = 0; x < n_right; ++x) mmax = std::max(mmax, rp[x + 1] - rp[x]);
            const int32_t grid = static_cast<int32_t>(std::min<int64_t>(n, 4096));
            const int64_t scratch = mmax > rs::kGoSortLds ? mmax : 0;
            rs::DevBuf<double> gs(std::max<int64_t>(1, scratch * grid));
            rs::DevBuf<int32_t> gp(std::max<int64_t>(1, scratch * grid));
            hipLaunchKernelGGL(rs::knn_predict_gosort_kernel, dim3(grid), dim3(64), 0, s, pl->S.p, pl->L, n_right,
                               drp.p, dids.p, drr.p, dm.p, dsd.p, db.p, global_mean, type, k, min_k, n, dl.p, dr.p,
                               dout.p, gs.p, gp.p, scratch);
            RS_HIP(hipGetLastError());
            RS_HIP(hipStreamSynchronize(s));  // the scratch dies with this scope
        } else {
            hipLaunchKernelGGL(rs::knn_predict_kernel, dim3(static_cast<uint32_t>(n)), dim3(64), 0, s,
                               pl->S.p, pl->L, n_right, drp.p, dids.p, drr.p, dm.p, dsd.p, db.p,
                               global_mean, type, k, min_k, n, dl.p, dr.p, dout.p);
        }
        RS_HIP(hipGetLastError());
        rs::kernel_span_end(ctx);
        dout.download(out, n, s);
        RS_HIP(hipStreamSynchronize(s));
        return RS_OK;
    });
}

extern "C" int rs_slope_one_predict(rs_knn_plan* pl, int32_t n_users, const int64_t* user_rowptr,
                                    const int32_t* user_items, const double* user_ratings,
                                    double global_mean, int64_t n, const int32_t* users,
                                    const int32_t* items, double* out) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    rs_ctx* ctx = pl->ctx;
    return rs_guard(ctx, [&]() -> int {
        if (pl->kind != RS_DEV_SLOPE_ONE)
            return rs::set_error(ctx, RS_ERR_INVALID, "plan does not hold a SlopeOne deviation matrix");
        if (n < 0 || (n > 0 && (!users || !items || !out)))
            return rs::set_error(ctx, RS_ERR_INVALID, "bad predict arguments");
        const int st = rs::check_knn_csr(ctx, n_users, pl->L, user_rowptr, user_items, user_ratings);
        if (st != RS_OK) return st;
        if (n == 0) return RS_OK;
        hipStream_t s = ctx->stream;
        const int64_t base = user_rowptr[0], nnz = user_rowptr[n_users] - base;
        std::vector<int64_t> rp(user_rowptr, user_rowptr + n_users + 1);
        for (auto& x : rp) x -= base;
        rs::DevBuf<int64_t> drp(rp.size());
        rs::DevBuf<int32_t> dit(std::max<int64_t>(1, nnz)), du(n), di(n);
        rs::DevBuf<double> dr(std::max<int64_t>(1, nnz)), dmean(std::max(1, n_users)), dout(n);
        drp.upload(rp.data(), rp.size(), s);
        dit.upload(user_items + base, nnz, s);
        dr.upload(user_ratings + base, nnz, s);
        du.upload(users, n, s);
        di.upload(items, n, s);
        rs::kernel_span_begin(ctx);
        if (n_users > 0)
            hipLaunchKernelGGL(rs::row_mean_kernel, dim3((n_users + 255) / 256), dim3(256), 0, s, n_users,
                               drp.p, dr.p, dmean.p);
        hipLaunchKernelGGL(rs::slope_one_predict_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256),
                           0, s, pl->S.p, pl->L, n_users, drp.p, dit.p, dmean.p, global_mean, n, du.p, di.p, dout.p);
        RS_HIP(hipGetLastError());
        rs::kernel_span_end(ctx);
        dout.download(out, n, s);
        RS_HIP(hipStreamSynchronize(s));
        return RS_OK;
    });
}
