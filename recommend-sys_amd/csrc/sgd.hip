// sgd.hip -- K1: SGD epoch of the Funk-SVD model (reference core/svd.go:63-132), gfx950.
//
// Two schedules (SURVEY §8a parity contract):
//   FAST    user-CSR, one wave per work item (heaviest first, LPT); p_u in VGPRs for the whole
//           item; q_i rows gathered D ratings ahead into a register ring; q_i updates written back
//           as float-atomic deltas (RS_SGD_WB_ATOMIC, default: no lost updates) or as write-through
//           stores (RS_SGD_WB_STORE: Hogwild, loses concurrent updates of hot items).  GlobalBias
//           (Q2) is a per-wave local SGD copy folded at epoch end as gb += sum_w n_w (gb_w - gb)/nnz
//           (fixed-order, deterministic).  RMSE parity with the reference (P2).
//           A work item is a whole user row, or -- for users with more than split_cap ratings -- one
//           of ceil(deg / split_cap) near-equal pieces of it: the pieces run as separate waves from
//           the same p_u and the row becomes the count-weighted average of their end states
//           (P += sum len/deg (p_end - p_start), merged after the epoch).  This cuts the per-user
//           serial chain (ML-1M's heaviest user: 2,314 ratings) but costs accuracy on ML-1M-shaped
//           data (measured), so it is off unless the caller asks (rs_svd_plan_set_split).
//           Likewise items with more than item_cap ratings are dealt (in user-CSR order) over
//           ceil(deg / item_cap) row copies, merged by count-weighted average after the epoch and
//           re-broadcast: the float atomics of a hot row are spread over several rows, which the
//           memory-side atomic unit otherwise serialises.  Off by default for the same reason.
//   ORDERED the ratings in train-set order with the exact update order of svd.go:93-129 (aliasing Q1:
//           q_i is updated with the NEW p_u) -- factor parity (P1): conflict-free batches on one
//           workgroup, sgd_ordered.hip.
//   TILE    the FAST default since round 2: user tiles in LDS, per-(item, tile) runs, sgd_tile.hip.
//
// Device layout of the FAST plan (HBM, fp32): P is n_users x ld, Q is n_items x ld with
// ld = 64 * ceil((k + 1) / 64); columns [0, k) hold the factors, column k holds the bias
// (b_u in P, b_i in Q), the rest is zero padding.  Lane l of the wave owns columns l + 64 x, so one
// row is E = ld / 64 coalesced wave instructions; the bias is lane 63 of the last one (last_col), and
// the padding lanes of the last one issue nothing.
//
// Cross-XCD visibility (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement & inter-workgroup
// visibility"): per-CU L1s and per-XCD L2s are not coherent inside a launch.  q_i loads carry sc1
// (bypass L1) and updates go to the memory side (atomics) or write through (sc1 stores); with plain
// accesses every XCD trains its own stale copy of the hot rows (measured: ML-100K RMSE 0.972 vs
// 0.937 for the reference order).
//
// Algorithmic bytes per epoch: nnz*(16 + 8k) + U*(16 + 8k)  (fp32 factors).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <cstring>
#include <memory>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <numeric>
#include <thread>
#include <stdexcept>
#include <type_traits>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "wave.hpp"
#include "sgd_plan.hpp"

namespace rs {

constexpr int kVolatileAux = static_cast<int>(0x80000000u);  // buffer intrinsic aux bit 31: volatile

// wave_sum, fx_to_f, fx_delta, last_col, roff, lane63: sgd_plan.hpp

// One FAST work item (a user row or a piece of one): the SGD chain over its ratings with p_u in
// VGPRs.  Every q_i update is handed to emit(row byte offset, q_new, q_old); the kernels below
// differ only in how that update reaches memory.  Returns n * (gb_end - gb_start) for the fold.
//
// LA (one-rating lookahead; kept for experiments, not instantiated by the launches):
// p_{t+1} = a p_t - c_t q_t, so p_{t+1}.q_{t+1} = a (p_t.q_{t+1}) - c_t (q_t.q_{t+1}).  Both dots
// depend only on p_t and the prefetched rows, so their reductions run beside rating t's chain and
// the chain from c_t to c_{t+1} is one FMA plus the diff.  Parity-tested on the heavy producers,
// but measured slower there (ML-1M epoch 585 -> 610 us, heavy chains still ~250 ns/rating): under
// the atomic load the heavy chain is not gated by its reduction.
template <int E, int D, bool FX = false, bool LA = false, class Emit>
__device__ __forceinline__ double sgd_work_item(
    int32_t w, const int32_t* __restrict__ wk_user, const int64_t* __restrict__ wk_rng,
    const float* __restrict__ wk_frac, const int32_t* __restrict__ items,
    const float* __restrict__ ratings, float* __restrict__ P, __amdgpu_buffer_rsrc_t rq, float gb0,
    float lr, float reg, float* __restrict__ dP, const float* __restrict__ uw, int32_t whole_direct,
    int32_t lc, float fx, Emit&& emit) {
#pragma clang fp contract(fast)
    constexpr int LD = 64 * E, B = 32;  // ratings per chunk (one unrolled loop body)
    static_assert(B % D == 0 && D <= B, "ring depth must divide the 32-rating chunk");
    const int lane = threadIdx.x & 63;
    const int32_t lane4 = lane * 4;
    const bool bias_lane = lane == 63;
    const float a = 1.f - lr * reg, fx_inv = 1.f / fx;
    const int32_t u = wk_user[w];
    const int64_t b = wk_rng[2 * w], e = wk_rng[2 * w + 1];
    const float frac = wk_frac[w];
    float p[E];
    float* prow = P + static_cast<int64_t>(u) * LD;
#pragma unroll
    for (int x = 0; x < E; ++x) p[x] = x < E - 1 ? prow[lane + 64 * x] : (lc >= 0 ? prow[lc] : 0.f);
    float ub = lane63(p[E - 1]);
    float gb = gb0;

    auto load_row = [&](float (&q)[E], int32_t valid, int32_t item) {
        const int32_t row = valid ? item * (LD * 4) : kOutOfRange;  // SGPR arithmetic
#pragma unroll
        for (int x = 0; x < E; ++x) {
            const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rq, roff<E>(row, x, lane4, lc), 0, kSgdAux);
            q[x] = FX ? fx_to_f(v, fx_inv) : __uint_as_float(v);
        }
    };

    // Item ids and ratings come in 32-entry chunks, one vector load per chunk (lane l holds entry
    // l & 31), issued a chunk ahead and read out with v_readlane: no scalar-memory wait sits in the
    // chain (a per-batch s_load round trip, several microseconds while the memory side is
    // saturated with atomics, was measured to set the heavy users' pace).  The loop body is two
    // whole chunks with fixed register sets A and B, so every ring slot and readlane index is a
    // compile-time constant and no register holding an in-flight load is ever copied (a rotating
    // copy made the compiler drain the ring at every chunk).
    const int32_t deg = static_cast<int32_t>(e - b);
    const int32_t l32 = lane & 31;
    // through buffer loads marked volatile (aux bit 31): LLVM would otherwise sink the chunk loads
    // to the end of the next chunk, next to their first use, and every chunk would wait for them
    const int32_t nrec = (deg + 128) * 4;  // arrays padded by 128 entries
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(items + b), 0, nrec, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ratings + b), 0, nrec, 0x00020000);
    auto ld_item = [&](int32_t pos) {
        return static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(ri, (pos + l32) * 4, 0, kVolatileAux));
    };
    auto ld_rating = [&](int32_t pos) {
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, (pos + l32) * 4, 0, kVolatileAux));
    };
    int32_t viA = ld_item(0), viB = ld_item(B);
    float vrA = ld_rating(0), vrB = ld_rating(B);
    // the first two chunks land before the ring loads (an asm that reads them forces the wait
    // here), so the loop header never inherits a just-issued load from the preheader
    asm volatile("" ::"v"(viA), "v"(viB), "v"(vrA), "v"(vrB));
    float ring[D][E];
#pragma unroll
    for (int s = 0; s < D; ++s) {  // in slot order (the loop's waits assume it)
        load_row(ring[s], s < deg, __builtin_amdgcn_readlane(viA, s));
        __builtin_amdgcn_sched_barrier(0);
    }
    float s_next = 0.f;  // LA: p_t.q_t of the next rating, precomputed
    if constexpr (LA) {
        float s0 = 0.f;
#pragma unroll
        for (int x = 0; x < E - 1; ++x) s0 += p[x] * ring[0][x];
        s0 += p[E - 1] * (bias_lane ? 0.f : ring[0][E - 1]);
        s_next = wave_sum(s0);
    }

    // the ratings [base, base + B) of the chunk held in (vi, vr); vn holds the next chunk's items
    auto chunk = [&](int64_t base, int32_t vi, float vr, int32_t vn) {
        const int32_t rem = static_cast<int32_t>(e - base);  // wave-uniform, SALU compares
#pragma unroll
        for (int j = 0; j < B; ++j) {
            constexpr int kD = D;
            const int slot = j % kD;
            if (j < rem) {
                float(&q)[E] = ring[slot];
                const float bq = lane63(q[E - 1]);
                const float rt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vr), j));
                float s = 0.f, la_a = 0.f, la_b = 0.f;
                if constexpr (LA) {
                    s = s_next;
                    static_assert(D >= 2, "lookahead reads the next ring slot");
                    const float(&q1)[E] = ring[(j + 1) % kD];  // the next rating's row (unused past the end)
#pragma unroll
                    for (int x = 0; x < E - 1; ++x) {
                        la_a += p[x] * q1[x];
                        la_b += q[x] * q1[x];
                    }
                    const float q1l = bias_lane ? 0.f : q1[E - 1];
                    la_a += p[E - 1] * q1l;
                    la_b += q[E - 1] * q1l;
                    la_a = wave_sum(la_a);
                    la_b = wave_sum(la_b);
                } else {
#pragma unroll
                    for (int x = 0; x < E - 1; ++x) s += p[x] * q[x];
                    s += p[E - 1] * (bias_lane ? 0.f : q[E - 1]);
                    s = wave_sum(s);
                }
                // svd.go:102-128 in FMA form: a = 1 - lr*reg, c = lr*diff:
                // p <- a p - c q ; q <- a q - c p_new ; b <- a b - c ; gb <- gb - c
                const float diff = ((gb + ub) + bq) + s - rt;
                const float c = lr * diff;
                if constexpr (LA) s_next = __builtin_fmaf(a, la_a, -c * la_b);
                gb -= c;
                ub = __builtin_fmaf(ub, a, -c);
                const float bq_new = __builtin_fmaf(bq, a, -c);
                float qn[E];
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    p[x] = __builtin_fmaf(-c, q[x], p[x] * a);
                    qn[x] = __builtin_fmaf(-c, p[x], q[x] * a);
                }
                p[E - 1] = bias_lane ? ub : p[E - 1];
                qn[E - 1] = bias_lane ? bq_new : qn[E - 1];
                emit(__builtin_amdgcn_readlane(vi, j) * (LD * 4), qn, q);
            }
            // refill this slot with the rating D ahead
            const int jn = j + D;
            load_row(ring[slot], jn < rem, jn < B ? __builtin_amdgcn_readlane(vi, jn % B)
                                                  : __builtin_amdgcn_readlane(vn, jn % B));
        }
    };
    // chunk loads two ahead stay inside the padding: base + 4B - 1 < e + 127
    for (int32_t o = 0; o < deg; o += 2 * B) {
        chunk(b + o, viA, vrA, viB);
        viA = ld_item(o + 2 * B);
        vrA = ld_rating(o + 2 * B);
        if (o + B >= deg) break;
        chunk(b + o + B, viB, vrB, viA);
        viB = ld_item(o + 3 * B);
        vrB = ld_rating(o + 3 * B);
    }
    if (dP && !(whole_direct && frac == 1.f)) {  // weighted delta, P stays at the epoch start
        const float sc = uw ? frac * uw[u] : frac;
        float* drow = dP + static_cast<int64_t>(u) * LD;
#pragma unroll
        for (int x = 0; x < E; ++x) {
            const int32_t c = x < E - 1 ? lane + 64 * x : lc;
            if (c >= 0) atomicAdd(drow + c, sc * (p[x] - prow[c]));
        }
    } else {
#pragma unroll
        for (int x = 0; x < E; ++x) {
            const int32_t c = x < E - 1 ? lane + 64 * x : lc;
            if (c >= 0) prow[c] = p[x];
        }
    }
    return static_cast<double>(deg) * (static_cast<double>(gb) - static_cast<double>(gb0));
}

// FAST epoch kernel (K1), direct write-back: each wave issues its own q_i updates -- float-atomic
// deltas (WB 1) or write-through stores (WB 0).  Four waves per block, one work item per wave.
//
// Write-back of p: direct store when dP is NULL; otherwise the weighted delta
// scale * (p_end - p_start) is float-atomically added to dP (scale = piece fraction, times the
// user's shard weight uw[u] in multi-GPU delta mode) -- except whole rows when whole_direct is set
// (single-GPU: only split users need the merge).
template <int E, int D, int WB>
__global__ __launch_bounds__(256) void svd_epoch_fast_kernel(
    const int32_t* __restrict__ wk_user, const int64_t* __restrict__ wk_rng,
    const float* __restrict__ wk_frac, int32_t n_work, const int32_t* __restrict__ items,
    const float* __restrict__ ratings, float* __restrict__ P, float* Q, int32_t q_bytes,
    const double* __restrict__ gb_in, double* __restrict__ gb_partial, float lr, float reg,
    float* __restrict__ dP, const float* __restrict__ uw, int32_t whole_direct, int32_t kf) {
    __shared__ double s_contrib[4];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + wib);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    const int32_t lane4 = lane * 4;
    const int32_t lc = last_col<E>(lane, kf);
    double contrib = 0.0;
    if (w < n_work) {
        contrib = sgd_work_item<E, D>(
            w, wk_user, wk_rng, wk_frac, items, ratings, P, rq, static_cast<float>(gb_in[0]), lr, reg,
            dP, uw, whole_direct, lc, 1.f, [&](int32_t row, const float (&qn)[E], const float (&q)[E]) {
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    if constexpr (WB == 1)
                        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(qn[x] - q[x], rq, roff<E>(row, x, lane4, lc), 0, 0);
                    else if constexpr (WB == 4)
                        __builtin_amdgcn_sched_barrier(0);
                    else
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(qn[x]), rq, roff<E>(row, x, lane4, lc), 0, kSgdAux);
                }
            });
    }
    if (lane == 0) s_contrib[wib] = contrib;
    __syncthreads();
    if (threadIdx.x == 0)
        gb_partial[blockIdx.x] = ((s_contrib[0] + s_contrib[1]) + s_contrib[2]) + s_contrib[3];
}

// FAST epoch kernel (K1), hybrid write-back (RS_SGD_WB_ATOMIC, the default).
//
// Why (measured): with direct atomics a wave's next q_i load waits, through the
// in-order vmcnt, for the atomics it issued D ratings earlier.  While the chip is saturating the
// memory-side atomic unit those take many microseconds, so a user's chain advances at
// (atomic latency / D) per rating.  Light users do not care (there are thousands of them and the
// epoch is throughput-bound while they run), but the heaviest users' chains set the epoch's tail.
//
// So the first n_heavy work items (the heaviest, LPT order) get a block each: wave 0 runs the SGD
// chain and writes each q_i delta into an LDS ring (E ds_write_b32 per lane, a row word and the
// tail word -- never waited on), and waves 1..3 drain it, writer w taking entries w, w + 3, ...,
// and issue the float atomics: the producer's vmcnt then holds only its loads, and three writers
// keep up to 3 x 63 atomics in flight.  A consumer that sees the tail sees the entry: a wave's DS
// instructions execute in issue order.  Every other block is four light work items with direct
// atomics.  The arithmetic and the memory-side deltas are those of RS_SGD_WB_ATOMIC_DIRECT.
template <int E>
struct HeavyRing {
    static constexpr int kRing = E <= 2 ? 32 : (E <= 4 ? 16 : 8);  // <= 16 KB of LDS per block
    static constexpr int kBatch = E <= 2 ? 8 : (E <= 4 ? 4 : 2);   // entries per writer LDS wait
    static_assert((kRing & (kRing - 1)) == 0, "ring size is a power of two");
};

__device__ __forceinline__ int32_t lds_load_relaxed(const int32_t* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_store_relaxed(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

//
// MERGE (hot replicas, rs_svd_plan_set_hot_replicas): the n_live most-rated items have R row copies
// (their ratings dealt over the copies), so the memory-side float atomics of one hot item are spread
// over R rows at different addresses instead of queueing on one.  The copies are kept one row in
// Hogwild terms by a merger -- the grid's last block -- that, until every other block has counted
// itself done in *done, repeatedly takes each live item's copies c_r and its last merged value L
// (qlast) and sets every copy to N = L + sum_r (c_r - L) by adding N - c_r(read) with float atomics
// (adds that land between the read and the add are kept, and counted in the next round), then
// L = N.  Every update is applied to every copy exactly once (delta sum, not an average); a copy
// misses the other copies' updates for at most one merge round.  svd_live_merge_kernel repeats the
// round once after the epoch so the item row and its copies leave the epoch equal.
constexpr int kMaxLiveCopies = 8;

template <int E, int D, bool DROP = false, bool MERGE = false, bool FX = false>
__global__ __launch_bounds__(256) void svd_epoch_hybrid_kernel(
    const int32_t* __restrict__ wk_user, const int64_t* __restrict__ wk_rng,
    const float* __restrict__ wk_frac, int32_t n_work, int32_t n_heavy,
    const int32_t* __restrict__ items, const float* __restrict__ ratings, float* __restrict__ P,
    float* Q, int32_t q_bytes, const double* __restrict__ gb_in, double* __restrict__ gb_partial,
    float lr, float reg, float* __restrict__ dP, const float* __restrict__ uw, int32_t whole_direct,
    int64_t* __restrict__ trace, const int4* __restrict__ live_meta, int32_t n_live,
    float* __restrict__ qlast, int32_t* __restrict__ done, int32_t kf, float fx) {
    constexpr int R = HeavyRing<E>::kRing, NB = HeavyRing<E>::kBatch, LD = 64 * E, NW = 3;
    // the producer's vmcnt holds only its q_i loads: prefetch as deep as the 63-op counter allows
    constexpr int DH = E == 1 ? 32 : (E == 2 ? 32 : (E <= 4 ? 16 : 8));
    __shared__ float s_q[R][LD];
    __shared__ int32_t s_row[R];
    __shared__ int32_t s_tail, s_done, s_head[NW];
    __shared__ double s_contrib[4];
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    const int32_t lane4 = lane * 4;
    const int32_t lc = last_col<E>(lane, kf);
    const float gb0 = static_cast<float>(gb_in[0]);
    const int blk = static_cast<int>(blockIdx.x);
    const int n_merge_blocks = MERGE ? (n_live + 3) / 4 : 0;
    const int n_sgd_blocks = static_cast<int>(gridDim.x) - n_merge_blocks;
    double contrib = 0.0;
    if (MERGE && blk >= n_sgd_blocks) {  // mergers: one wave per live item (block-uniform branch)
        const int h = (blk - n_sgd_blocks) * 4 + wib;
        if (threadIdx.x == 0) gb_partial[blk] = 0.0;
        if (h >= n_live) return;
        const int4 m = live_meta[h];
        const int R = m.z;
        float last[E];
#pragma unroll
        for (int x = 0; x < E; ++x) {
            const int32_t c = x < E - 1 ? lane + 64 * x : lc;
            last[x] = c >= 0 ? qlast[static_cast<int64_t>(h) * LD + c] : 0.f;
        }
        for (;;) {
            const int32_t d = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if constexpr (FX) {  // the same round on the int32 rows: exact, wrap-around arithmetic
                uint32_t c[kMaxLiveCopies][E];
#pragma unroll
                for (int r = 0; r < kMaxLiveCopies; ++r) {
                    const int32_t row = (r < R ? (r == 0 ? m.x : m.y + r - 1) * (LD * 4) : kOutOfRange);
#pragma unroll
                    for (int x = 0; x < E; ++x)
                        c[r][x] = __builtin_amdgcn_raw_buffer_load_b32(rq, roff<E>(row, x, lane4, lc), 0, kSgdAux);
                }
                uint32_t nv[E];
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    const uint32_t l = __float_as_uint(last[x]);
                    uint32_t acc = l;
#pragma unroll
                    for (int r = 0; r < kMaxLiveCopies; ++r)
                        if (r < R) acc += c[r][x] - l;
                    nv[x] = acc;
                }
#pragma unroll
                for (int r = 0; r < kMaxLiveCopies; ++r) {
                    if (r < R) {
                        const int32_t row = (r == 0 ? m.x : m.y + r - 1) * (LD * 4);
#pragma unroll
                        for (int x = 0; x < E; ++x)
                            __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(static_cast<int32_t>(nv[x] - c[r][x]), rq,
                                                                           roff<E>(row, x, lane4, lc), 0, 0);
                    }
                }
#pragma unroll
                for (int x = 0; x < E; ++x) last[x] = __uint_as_float(nv[x]);
            } else {
                float c[kMaxLiveCopies][E];
#pragma unroll
                for (int r = 0; r < kMaxLiveCopies; ++r) {
                    const int32_t row = (r < R ? (r == 0 ? m.x : m.y + r - 1) * (LD * 4) : kOutOfRange);
#pragma unroll
                    for (int x = 0; x < E; ++x)
                        c[r][x] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rq, roff<E>(row, x, lane4, lc), 0, kSgdAux));
                }
                float nv[E];
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    float acc = last[x];
#pragma unroll
                    for (int r = 0; r < kMaxLiveCopies; ++r)
                        if (r < R) acc += c[r][x] - last[x];
                    nv[x] = acc;
                }
#pragma unroll
                for (int r = 0; r < kMaxLiveCopies; ++r) {
                    if (r < R) {
                        const int32_t row = (r == 0 ? m.x : m.y + r - 1) * (LD * 4);
#pragma unroll
                        for (int x = 0; x < E; ++x)
                            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(nv[x] - c[r][x], rq, roff<E>(row, x, lane4, lc), 0, 0);
                    }
                }
#pragma unroll
                for (int x = 0; x < E; ++x) last[x] = nv[x];
            }
            if (d >= n_sgd_blocks) break;  // one last round after everyone finished
        }
#pragma unroll
        for (int x = 0; x < E; ++x) {
            const int32_t c = x < E - 1 ? lane + 64 * x : lc;
            if (c >= 0) qlast[static_cast<int64_t>(h) * LD + c] = last[x];
        }
        return;
    }
    if (blk >= n_heavy) {  // light blocks: four waves, each striding over the light work items
        const int stride = (n_sgd_blocks - n_heavy) * 4;
        for (int w = n_heavy + (blk - n_heavy) * 4 + wib; w < n_work; w += stride) {
            const int64_t t0 = trace ? static_cast<int64_t>(__builtin_amdgcn_s_memrealtime()) : 0;
            contrib += sgd_work_item<E, D, FX>(
                w, wk_user, wk_rng, wk_frac, items, ratings, P, rq, gb0, lr, reg, dP, uw, whole_direct, lc, fx,
                [&](int32_t row, const float (&qn)[E], const float (&q)[E]) {
#pragma unroll
                    for (int x = 0; x < E; ++x) {
                        if constexpr (DROP) {
                        } else if constexpr (FX) {
                            __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(fx_delta(qn[x], q[x], fx), rq, roff<E>(row, x, lane4, lc), 0, 0);
                        } else {
                            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(qn[x] - q[x], rq, roff<E>(row, x, lane4, lc), 0, 0);
                        }
                    }
                });
            if (trace && lane == 0) {  // diagnostic timeline (100 MHz clock)
                const int64_t t1 = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
                trace[3 * w] = t0;
                trace[3 * w + 1] = t1;
                trace[3 * w + 2] = t1;
            }
        }
        if (lane == 0) s_contrib[wib] = contrib;
        __syncthreads();
        if (threadIdx.x == 0) {
            gb_partial[blk] = ((s_contrib[0] + s_contrib[1]) + s_contrib[2]) + s_contrib[3];
            if (MERGE) __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // heavy block (block-uniform branch): work item blk, wave 0 produces, waves 1..3 write
    if (threadIdx.x == 0) {
        s_tail = 0;
        s_done = 0;
    }
    if (threadIdx.x < NW) s_head[threadIdx.x] = static_cast<int32_t>(threadIdx.x);
    __syncthreads();
    const int64_t t0 = trace ? static_cast<int64_t>(__builtin_amdgcn_s_memrealtime()) : 0;
    if (wib == 0) {
        int32_t tail = 0, free_end = R;  // entries [tail, free_end) may be written
        contrib = sgd_work_item<E, DH, FX, false>(
            blk, wk_user, wk_rng, wk_frac, items, ratings, P, rq, gb0, lr, reg, dP, uw, whole_direct, lc, fx,
            [&](int32_t row, const float (&qn)[E], const float (&q)[E]) {
                if (tail >= free_end) {  // ring full: every entry below min(head) has been drained
                    for (;;) {
                        const int32_t h = min(min(lds_load_relaxed(&s_head[0]), lds_load_relaxed(&s_head[1])),
                                              lds_load_relaxed(&s_head[2]));
                        free_end = h + R;
                        if (tail < free_end) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                const int slot = tail & (R - 1);
#pragma unroll
                for (int x = 0; x < E; ++x)
                    s_q[slot][lane + 64 * x] = FX ? __int_as_float(fx_delta(qn[x], q[x], fx)) : qn[x] - q[x];
                if (lane == 0) s_row[slot] = row;
                __atomic_signal_fence(__ATOMIC_SEQ_CST);  // entry before tail, in issue order
                ++tail;
                if (lane == 0) lds_store_relaxed(&s_tail, tail);
            });
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (lane == 0) lds_store_relaxed(&s_done, 1);
        if (trace && lane == 0) trace[3 * blk + 1] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
    } else {
        const int wr = wib - 1;
        int32_t next = wr;  // next entry index of this writer: wr, wr + 3, ...
        for (;;) {
            const int32_t done = lds_load_relaxed(&s_done);  // done before tail: the final tail
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            const int32_t tail = lds_load_relaxed(&s_tail);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            if (next < tail) {
                while (next < tail) {  // up to NB of this writer's entries per LDS wait
                    const int32_t n = min((tail - next + NW - 1) / NW, NB);
                    const int32_t myrow = s_row[(next + NW * (lane & (NB - 1))) & (R - 1)];
                    float v[NB][E];
#pragma unroll
                    for (int j = 0; j < NB; ++j)
#pragma unroll
                        for (int x = 0; x < E; ++x) v[j][x] = s_q[(next + NW * j) & (R - 1)][lane + 64 * x];
#pragma unroll
                    for (int j = 0; j < NB; ++j) {
                        if (j < n) {
                            const int32_t row = __builtin_amdgcn_readlane(myrow, j);
#pragma unroll
                            for (int x = 0; x < E; ++x) {
                                if constexpr (DROP) {
                                } else if constexpr (FX) {
                                    __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(__float_as_int(v[j][x]), rq, roff<E>(row, x, lane4, lc), 0, 0);
                                } else {
                                    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v[j][x], rq, roff<E>(row, x, lane4, lc), 0, 0);
                                }
                            }
                        }
                    }
                    next += NW * n;
                }
                __atomic_signal_fence(__ATOMIC_SEQ_CST);  // entries read before their slots are freed
                if (lane == 0) lds_store_relaxed(&s_head[wr], next);
            } else if (done) {
                break;
            } else {
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        gb_partial[blk] = contrib;
        if (MERGE) __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (trace) {
            trace[3 * blk] = t0;
            trace[3 * blk + 2] = static_cast<int64_t>(__builtin_amdgcn_s_memrealtime());
        }
    }
}

// gb += (sum of block partials in fixed order) / nnz  -- one block, deterministic tree.
__global__ __launch_bounds__(256) void gb_fold_kernel(const double* __restrict__ partial, int64_t n,
                                                      double* __restrict__ gb, double inv_nnz) {
    __shared__ double s[256];
    double t = 0.0;
    for (int64_t x = threadIdx.x; x < n; x += 256) t += partial[x];
    s[threadIdx.x] = t;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (static_cast<int>(threadIdx.x) < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) gb[0] += s[0] * inv_nnz;
}

// Split users (single GPU): P[u] += dP[u], dP[u] = 0 for the listed rows (one wave per row).
__global__ __launch_bounds__(64) void svd_merge_rows_kernel(float* __restrict__ P, float* __restrict__ dP,
                                                           const int32_t* __restrict__ rows, int32_t ld) {
    const int64_t r = static_cast<int64_t>(rows[blockIdx.x]) * ld;
    for (int32_t c = threadIdx.x; c < ld; c += 64) {
        P[r + c] += dP[r + c];
        dP[r + c] = 0.f;
    }
}

// Split items: meta = {item row, first extra row, copies R, offset into frac}.  mode 0: the item row
// and its R - 1 copies become the count-weighted average of the copies (fixed order); mode 1: the
// copies are set to the item row (after an upload).  One wave per split item.
__global__ __launch_bounds__(64) void svd_item_merge_kernel(float* __restrict__ Q,
                                                           const int4* __restrict__ meta,
                                                           const float* __restrict__ frac, int32_t ld,
                                                           int32_t mode) {
    const int4 m = meta[blockIdx.x];
    auto row = [&](int32_t c) { return static_cast<int64_t>(c == 0 ? m.x : m.y + c - 1) * ld; };
    for (int32_t col = threadIdx.x; col < ld; col += 64) {
        float v = 0.f;
        if (mode == 0) {
            for (int32_t c = 0; c < m.z; ++c) v = __builtin_fmaf(frac[m.w + c], Q[row(c) + col], v);
        } else {
            v = Q[row(0) + col];
        }
        for (int32_t c = 0; c < m.z; ++c) Q[row(c) + col] = v;
    }
}

// Live (hot-replica) items around an epoch, one wave per item: meta = {item row, first extra row,
// copies R, unused}.  mode 0 (before): L = the item row (all copies are equal here).  mode 1 (after):
// the merge round of the hybrid kernel's merger, N = L + sum_r (c_r - L), written to every copy.
__global__ __launch_bounds__(64) void svd_live_merge_kernel(float* __restrict__ Q, const int4* __restrict__ meta,
                                                           float* __restrict__ qlast, int32_t ld, int32_t mode) {
    const int4 m = meta[blockIdx.x];
    auto row = [&](int32_t c) { return static_cast<int64_t>(c == 0 ? m.x : m.y + c - 1) * ld; };
    float* L = qlast + static_cast<int64_t>(blockIdx.x) * ld;
    for (int32_t col = threadIdx.x; col < ld; col += 64) {
        if (mode == 0) {
            L[col] = Q[row(0) + col];
        } else {
            const float l = L[col];
            float v = l;
            for (int32_t c = 0; c < m.z; ++c) v += Q[row(c) + col] - l;
            for (int32_t c = 0; c < m.z; ++c) Q[row(c) + col] = v;
        }
    }
}

// Fixed-point item rows around a call (tile schedule; hybrid with rs_svd_plan_set_fixed_q), in place
// over Q's n words: to == 1: q -> round(q * 2^shift) (saturating), to == 0: back to fp32.  A value that
// is non-finite or |q| >= 2^(31 - shift) going in (128 at the star-scale shift 24), or within 1/2 of the
// int32 range coming back (integer atomics wrap), raises *flag (plan_download reports RS_ERR_NUMERIC).
__global__ __launch_bounds__(256) void svd_q_fixed_kernel(float* __restrict__ Q, int64_t n, int32_t to,
                                                          int32_t* __restrict__ flag, int32_t shift) {
    const float fx = static_cast<float>(1u << shift), range = static_cast<float>(1u << (31 - shift));
    const int32_t lim = static_cast<int32_t>(0x80000000u - (1u << (shift - 1)));  // within 1/2 of the int32 range
    bool bad = false;
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; t < n;
         t += static_cast<int64_t>(gridDim.x) * 256) {
        if (to) {
            const float v = Q[t];
            bad |= !(fabsf(v) < range);
            Q[t] = __int_as_float(__float2int_rn(v * fx));
        } else {
            const int32_t v = __float_as_int(Q[t]);
            bad |= v >= lim || v <= -lim;
            Q[t] = fx_to_f(static_cast<uint32_t>(v), 1.f / fx);
        }
    }
    if (bad) flag[0] = 1;
}

// The live items' final merge round on the int32 rows (fixed-point epochs): exact integer
// N = L + sum_r (c_r - L), written to every copy; L := N.
__global__ __launch_bounds__(64) void svd_live_merge_fx_kernel(int32_t* __restrict__ Q, const int4* __restrict__ meta,
                                                              int32_t* __restrict__ qlast, int32_t ld) {
    const int4 m = meta[blockIdx.x];
    auto row = [&](int32_t c) { return static_cast<int64_t>(c == 0 ? m.x : m.y + c - 1) * ld; };
    int32_t* L = qlast + static_cast<int64_t>(blockIdx.x) * ld;
    for (int32_t col = threadIdx.x; col < ld; col += 64) {
        const uint32_t l = static_cast<uint32_t>(L[col]);
        uint32_t v = l;
        for (int32_t c = 0; c < m.z; ++c) v += static_cast<uint32_t>(Q[row(c) + col]) - l;
        for (int32_t c = 0; c < m.z; ++c) Q[row(c) + col] = static_cast<int32_t>(v);
        L[col] = static_cast<int32_t>(v);
    }
}

// After each epoch of a fixed-point run (plan_epochs keeps Q in int32 across its epochs), one launch
// does what three did: blocks [0, n_live) the live items' final integer merge round (as
// svd_live_merge_fx_kernel: N = L + sum_r (c_r - L) to every copy, L := N), blocks
// [n_live, n_live + n_split) the split users' row merges (as svd_merge_rows_kernel), and the last
// block the GlobalBias fold (as gb_fold_kernel, the same 256-thread tree) plus re-arming the
// merger's done counter for the next epoch.  Columns are independent, so the arithmetic is theirs.
// 1024 threads: the fold's partials (one per workgroup of the tile launch since round 6, 176 on ML-1M; the
// other schedules' per-block partials) are at most a few loads per thread and a wave-shuffle sum -- round 5's
// 2816 per-wave partials took 7-8 us per epoch (profiles/r05/final/bench_kernel_stats.csv).
constexpr int kEpilogueThreads = 1024;
__global__ __launch_bounds__(kEpilogueThreads) void svd_epoch_epilogue_kernel(
    int32_t* __restrict__ Q, const int4* __restrict__ meta, int32_t* __restrict__ qlast, int32_t n_live,
    float* __restrict__ P, float* __restrict__ dP, const int32_t* __restrict__ rows, int32_t n_split,
    int32_t ld, const double* __restrict__ partial, int64_t n_partial, double* __restrict__ gb,
    double inv_nnz, int32_t* __restrict__ done, const float* __restrict__ loss_part, double* __restrict__ loss_state,
    int32_t* __restrict__ flag, double inv_lr2, const double* __restrict__ smooth, double a_all) {
    const int b = static_cast<int>(blockIdx.x);
    const int tid = static_cast<int>(threadIdx.x);
    if (b < n_live) {
        const int4 m = meta[b];
        auto row = [&](int32_t c) { return static_cast<int64_t>(c == 0 ? m.x : m.y + c - 1) * ld; };
        int32_t* L = qlast + static_cast<int64_t>(b) * ld;
        for (int32_t col = tid; col < ld; col += kEpilogueThreads) {
            const uint32_t l = static_cast<uint32_t>(L[col]);
            uint32_t v = l;
            for (int32_t c = 0; c < m.z; ++c) v += static_cast<uint32_t>(Q[row(c) + col]) - l;
            for (int32_t c = 0; c < m.z; ++c) Q[row(c) + col] = static_cast<int32_t>(v);
            L[col] = static_cast<int32_t>(v);
        }
        return;
    }
    if (b < n_live + n_split) {
        const int64_t r = static_cast<int64_t>(rows[b - n_live]) * ld;
        for (int32_t c = tid; c < ld; c += kEpilogueThreads) {
            P[r + c] += dP[r + c];
            dP[r + c] = 0.f;
        }
        return;
    }
    constexpr int NWV = kEpilogueThreads / 64;
    __shared__ double sh[NWV], sl[NWV], sn[NWV], sd[NWV];
    // thread 0's own operands are loaded first, so their latency overlaps the partials' loads instead of
    // following the reduction
    double gb_old = 0.0, prev = 0.0;
    if (tid == 0) {
        gb_old = gb[0];
        if (loss_part && loss_state) prev = loss_state[0];
    }
    double t = 0.0, l = 0.0, nm = 0.0, dn = 0.0;
    for (int64_t x = tid; x < n_partial; x += kEpilogueThreads) {
        t += partial[x];
        if (loss_part) l += static_cast<double>(loss_part[x]);
        if (smooth) {
            nm += smooth[2 * x];
            dn += smooth[2 * x + 1];
        }
    }
    for (int o = 32; o > 0; o >>= 1) {  // fixed order: the same bits on every run
        t += __shfl_xor(t, o);
        l += __shfl_xor(l, o);
        nm += __shfl_xor(nm, o);
        dn += __shfl_xor(dn, o);
    }
    if ((tid & 63) == 0) {
        sh[tid >> 6] = t;
        sl[tid >> 6] = l;
        sn[tid >> 6] = nm;
        sd[tid >> 6] = dn;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < NWV; ++w) {
            sh[0] += sh[w];
            sl[0] += sl[w];
            sn[0] += sn[w];
            sd[0] += sd[w];
        }
        // the tile epoch's smoothed fold (sgd_tile.hip header): gb' = A gb + (1 - A) T, T = sum b / sum (1 - a);
        // the other schedules: the count-weighted mean of the streams' moves
        if (smooth) gb[0] = sd[0] > 0.0 ? a_all * gb_old + (1.0 - a_all) * (sn[0] / sd[0]) : gb_old;
        else gb[0] = gb_old + sh[0] * inv_nnz;
        if (done) *done = 0;
        if (loss_part && loss_state) {
            // the divergence guard's second signal: this epoch's training MSE (at the ratings' pre-update
            // residuals) more than 1.03x the previous epoch's -- SGD at a stable rate does not raise it
            const double mse = sl[0] * inv_nnz * inv_lr2;
            if (!(mse < 1e30) || (prev > 0.0 && mse > 1.03 * prev)) flag[0] = 1;
            loss_state[0] = mse;
        }
    }
}

// Multi-GPU: the all-reduced weighted user deltas and global-bias sum are applied in place.
__global__ __launch_bounds__(256) void svd_apply_delta_kernel(float4* __restrict__ P,
                                                              const float4* __restrict__ dP, int64_t n4,
                                                              double* __restrict__ gb,
                                                              const double* __restrict__ gbsum,
                                                              double inv_total) {
    for (int64_t t = blockIdx.x * 256 + threadIdx.x; t < n4; t += static_cast<int64_t>(gridDim.x) * 256) {
        float4 a = P[t];
        const float4 d = dP[t];
        a.x += d.x; a.y += d.y; a.z += d.z; a.w += d.w;
        P[t] = a;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) gb[0] += gbsum[0] * inv_total;
}

// User-sharded mode: dQ = w_i (Q - Q0) for the n_items item rows, and Q is restored to Q0.
__global__ __launch_bounds__(256) void svd_qdelta_kernel(float* __restrict__ Q, const float* __restrict__ Q0,
                                                         const float* __restrict__ w, float* __restrict__ dQ,
                                                         int64_t n, int32_t ld) {
    for (int64_t t = blockIdx.x * 256 + threadIdx.x; t < n; t += static_cast<int64_t>(gridDim.x) * 256) {
        const float q0 = Q0[t];
        dQ[t] = w[t / ld] * (Q[t] - q0);
        Q[t] = q0;
    }
}

// sum of block partials in fixed order (multi-GPU: the ranks' sums are all-reduced, then applied)
__global__ __launch_bounds__(256) void gb_sum_kernel(const double* __restrict__ partial, int64_t n,
                                                     double* __restrict__ out) {
    __shared__ double s[256];
    double t = 0.0;
    for (int64_t x = threadIdx.x; x < n; x += 256) t += partial[x];
    s[threadIdx.x] = t;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (static_cast<int>(threadIdx.x) < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = s[0];
}

// --------------------------------------------------------------------------------------------
// Batched Predict / RMSE / MAE on the plan's device factors.
// svd.go:32-51 per (user, item) pair, -1 = unknown id (data.go:129): gb + b_u [u known] + b_i
// [i known] + p_u . q_i [both known], evaluated in float64 on the fp32 factors.  One 16-lane group
// per pair (lane l sums columns l + 16 x in order, then a fixed DPP tree).  With ratings, the block's
// squared and absolute errors go to fixed per-block partials (utils.go:162-180), folded in order.
__global__ __launch_bounds__(256) void svd_predict_kernel(
    const float* __restrict__ P, const float* __restrict__ Q, int32_t ld, int32_t k, int32_t n_users,
    int32_t n_items, const double* __restrict__ gb, int64_t n, const int32_t* __restrict__ users,
    const int32_t* __restrict__ items, const double* __restrict__ ratings, double* __restrict__ out,
    double* __restrict__ partial) {
    __shared__ double s_sq[16], s_abs[16];
    const int gl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int64_t t = static_cast<int64_t>(blockIdx.x) * 16 + grp;
    double pred = 0.0;
    if (t < n) {
        const int32_t u = users[t], i = items[t];
        const bool ku = u >= 0 && u < n_users, ki = i >= 0 && i < n_items;
        double d = 0.0;
        if (ku && ki) {
            const float* pu = P + static_cast<int64_t>(u) * ld;
            const float* qi = Q + static_cast<int64_t>(i) * ld;
            for (int32_t c = gl; c < k; c += 16) d += static_cast<double>(pu[c]) * static_cast<double>(qi[c]);
        }
        d += __shfl_xor(d, 1, 16);
        d += __shfl_xor(d, 2, 16);
        d += __shfl_xor(d, 4, 16);
        d += __shfl_xor(d, 8, 16);
        pred = gb[0];
        if (ku) pred += static_cast<double>(P[static_cast<int64_t>(u) * ld + k]);  // bias column k
        if (ki) pred += static_cast<double>(Q[static_cast<int64_t>(i) * ld + k]);
        if (ku && ki) pred += d;
        if (out && gl == 0) out[t] = pred;
    }
    if (partial) {
        const double e = t < n ? pred - ratings[t] : 0.0;
        if (gl == 0) {
            s_sq[grp] = e * e;
            s_abs[grp] = fabs(e);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double a = 0.0, b = 0.0;
            for (int x = 0; x < 16; ++x) {
                a += s_sq[x];
                b += s_abs[x];
            }
            partial[2 * blockIdx.x] = a;
            partial[2 * blockIdx.x + 1] = b;
        }
    }
}

// out = {sum of even partials, sum of odd partials} in fixed order (one block)
__global__ __launch_bounds__(256) void pair_sum_kernel(const double* __restrict__ partial, int64_t n_blocks,
                                                       double* __restrict__ out) {
    __shared__ double s[2][256];
    double a = 0.0, b = 0.0;
    for (int64_t x = threadIdx.x; x < n_blocks; x += 256) {
        a += partial[2 * x];
        b += partial[2 * x + 1];
    }
    s[0][threadIdx.x] = a;
    s[1][threadIdx.x] = b;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (static_cast<int>(threadIdx.x) < w) {
            s[0][threadIdx.x] += s[0][threadIdx.x + w];
            s[1][threadIdx.x] += s[1][threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = s[0][0];
        out[1] = s[1][0];
    }
}


}  // namespace rs

// ------------------------------------------------------------------------------------------------
// Plan (device-resident CSR + factors): struct rs_svd_plan lives in sgd_plan.hpp (shared with
// sgd_tile.hip, the tile schedule).


namespace rs {

constexpr int32_t kMaxFactors = 510;  // the tile kernel's registers hold k + 2 columns (<= 512)

// Light blocks of the hybrid launch: 1.5 per CU (6 light waves per CU).  Measured on the ML-1M shape
// (DESIGN.md K1): one wave per user puts ~6,000 waves' atomics in flight and the memory-side queue
// latency that every q_i load then pays sets the heavy users' pace; 256-512 light blocks each
// striding over the LPT-ordered light users keep the atomic unit as busy with far shorter queues.
int32_t default_light_blocks(const rs_ctx* ctx) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
        cus = 256;
    return (3 * cus) / 2;
}

// Blocks of the FAST launch: four work items per block (direct write-back), or one block per heavy
// work item plus four light items per block (hybrid).  gb partials are one per block.
int32_t fast_blocks(const rs_svd_plan* pl) {
    if (pl->write_back == RS_SGD_WB_ATOMIC) {
        int32_t light = (pl->n_work - pl->n_heavy + 3) / 4;
        if (pl->light_blocks > 0) light = std::min(light, pl->light_blocks);
        return std::max<int32_t>(1, pl->n_heavy + light) + (pl->n_live + 3) / 4;  // + live mergers
    }
    return std::max<int32_t>(1, (pl->n_work + 3) / 4);
}

template <int E, int D, int WB>
static void launch_fast_t(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP) {
    const int32_t q_bytes = buffer_bytes32(pl->Q.n, sizeof(float), "item factor matrix");
    // multi-GPU delta mode (caller's dP, shard weights): every item adds its weighted delta;
    // single GPU: whole rows store P directly, pieces of split users add into the plan's dPs
    const bool multi = dP != nullptr;
    float* d = multi ? dP : (pl->n_split > 0 ? pl->dPs.p : nullptr);
    pl->n_blocks = fast_blocks(pl);
    if constexpr (WB == 2 || WB == 5) {
        if (WB == 2 && pl->fixed_q) {
            if (pl->n_live > 0 && !pl->hoisted) RS_HIP(hipMemsetAsync(pl->done.p, 0, sizeof(int32_t), s));
            auto kern = pl->n_live > 0 ? svd_epoch_hybrid_kernel<E, D, false, true, true>
                                       : svd_epoch_hybrid_kernel<E, D, false, false, true>;
            hipLaunchKernelGGL(kern, dim3(pl->n_blocks), dim3(256), 0, s,
                               pl->wk_user.p, pl->wk_rng.p, pl->wk_frac.p, pl->n_work, pl->n_heavy,
                               pl->items.p, pl->ratings.p, pl->P.p, pl->Q.p, q_bytes, pl->gb.p,
                               pl->partial.p, lr, reg, d, multi ? pl->uw.p : nullptr, multi ? 0 : 1,
                               pl->trace.n ? pl->trace.p : nullptr, pl->n_live > 0 ? pl->live_meta.p : nullptr,
                               pl->n_live, pl->n_live > 0 ? pl->qlast.p : nullptr, pl->n_live > 0 ? pl->done.p : nullptr,
                               pl->k, pl->fx());
        } else if (pl->n_live > 0) {
            RS_HIP(hipMemsetAsync(pl->done.p, 0, sizeof(int32_t), s));
            hipLaunchKernelGGL((svd_epoch_hybrid_kernel<E, D, WB == 5, true>), dim3(pl->n_blocks), dim3(256), 0, s,
                               pl->wk_user.p, pl->wk_rng.p, pl->wk_frac.p, pl->n_work, pl->n_heavy,
                               pl->items.p, pl->ratings.p, pl->P.p, pl->Q.p, q_bytes, pl->gb.p,
                               pl->partial.p, lr, reg, d, multi ? pl->uw.p : nullptr, multi ? 0 : 1,
                               pl->trace.n ? pl->trace.p : nullptr, pl->live_meta.p, pl->n_live, pl->qlast.p,
                               pl->done.p, pl->k, 1.f);
        } else {
            hipLaunchKernelGGL((svd_epoch_hybrid_kernel<E, D, WB == 5, false>), dim3(pl->n_blocks), dim3(256), 0, s,
                               pl->wk_user.p, pl->wk_rng.p, pl->wk_frac.p, pl->n_work, pl->n_heavy,
                               pl->items.p, pl->ratings.p, pl->P.p, pl->Q.p, q_bytes, pl->gb.p,
                               pl->partial.p, lr, reg, d, multi ? pl->uw.p : nullptr, multi ? 0 : 1,
                               pl->trace.n ? pl->trace.p : nullptr, nullptr, 0, nullptr, nullptr, pl->k, 1.f);
        }
    } else {
        hipLaunchKernelGGL((svd_epoch_fast_kernel<E, D, WB>), dim3(pl->n_blocks), dim3(256), 0, s,
                           pl->wk_user.p, pl->wk_rng.p, pl->wk_frac.p, pl->n_work, pl->items.p,
                           pl->ratings.p, pl->P.p, pl->Q.p, q_bytes, pl->gb.p, pl->partial.p, lr, reg,
                           d, multi ? pl->uw.p : nullptr, multi ? 0 : 1, pl->k);
    }
}

template <int D, int WB>
static void launch_fast_e(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP) {
    switch (pl->ld / 64) {
        case 1: launch_fast_t<1, D, WB>(pl, lr, reg, s, dP); break;
        case 2: launch_fast_t<2, D, WB>(pl, lr, reg, s, dP); break;
        case 3: launch_fast_t<3, D, WB>(pl, lr, reg, s, dP); break;
        case 4: launch_fast_t<4, D, WB>(pl, lr, reg, s, dP); break;
        case 5: launch_fast_t<5, D, WB>(pl, lr, reg, s, dP); break;
        case 6: launch_fast_t<6, D, WB>(pl, lr, reg, s, dP); break;
        case 7: launch_fast_t<7, D, WB>(pl, lr, reg, s, dP); break;
        default: launch_fast_t<8, D, WB>(pl, lr, reg, s, dP); break;
    }
}

template <int WB>
static void launch_fast_d(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP) {
    switch (pl->ring_depth) {
        case 4: launch_fast_e<4, WB>(pl, lr, reg, s, dP); break;
        case 16: launch_fast_e<16, WB>(pl, lr, reg, s, dP); break;
        default: launch_fast_e<8, WB>(pl, lr, reg, s, dP); break;
    }
}

static void launch_fast(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP = nullptr) {
    if (pl->write_back == RS_SGD_WB_TILE) {  // sgd_tile.hip; Q is int32 fixed point inside
        if (pl->hoisted) {
            tile_launch(pl, lr, reg, s, dP);
            return;
        }
        const int64_t qn = static_cast<int64_t>(pl->Q.n);
        const int fx_blocks = static_cast<int>(std::min<int64_t>(2048, (qn + 255) / 256));
        hipLaunchKernelGGL(svd_q_fixed_kernel, dim3(fx_blocks), dim3(256), 0, s, pl->Q.p, qn, 1, numflag(pl), pl->fx_shift);
        tile_launch(pl, lr, reg, s, dP);
        hipLaunchKernelGGL(svd_q_fixed_kernel, dim3(fx_blocks), dim3(256), 0, s, pl->Q.p, qn, 0, numflag(pl), pl->fx_shift);
        RS_HIP(hipGetLastError());
        return;
    }
    if (pl->hoisted) {  // plan_epochs does the conversions and the epilogue around its epoch loop
        launch_fast_d<2>(pl, lr, reg, s, dP);
        RS_HIP(hipGetLastError());
        return;
    }
    const bool fx = pl->fixed_q && pl->write_back == RS_SGD_WB_ATOMIC;
    const int64_t qn = static_cast<int64_t>(pl->Q.n);
    const int fx_blocks = static_cast<int>(std::min<int64_t>(2048, (qn + 255) / 256));
    if (fx) hipLaunchKernelGGL(svd_q_fixed_kernel, dim3(fx_blocks), dim3(256), 0, s, pl->Q.p, qn, 1, numflag(pl), pl->fx_shift);
    if (pl->n_live > 0)  // L = the live items' rows at the epoch start (a bit copy: int32 rows too)
        hipLaunchKernelGGL(svd_live_merge_kernel, dim3(pl->n_live), dim3(64), 0, s, pl->Q.p, pl->live_meta.p,
                           pl->qlast.p, pl->ld, 0);
    switch (pl->write_back) {
        case RS_SGD_WB_STORE: launch_fast_d<0>(pl, lr, reg, s, dP); break;          // write-through stores
        case RS_SGD_WB_ATOMIC_DIRECT: launch_fast_d<1>(pl, lr, reg, s, dP); break;  // per-wave atomics
        default: launch_fast_d<2>(pl, lr, reg, s, dP); break;                       // hybrid
    }
    if (fx) {  // final live round on the int32 rows, then back to fp32 (live_merge_after skips)
        if (pl->n_live > 0) {
            hipLaunchKernelGGL(svd_live_merge_fx_kernel, dim3(pl->n_live), dim3(64), 0, s,
                               reinterpret_cast<int32_t*>(pl->Q.p), pl->live_meta.p,
                               reinterpret_cast<int32_t*>(pl->qlast.p), pl->ld);
            pl->live_merged = true;
        }
        hipLaunchKernelGGL(svd_q_fixed_kernel, dim3(fx_blocks), dim3(256), 0, s, pl->Q.p, qn, 0, numflag(pl), pl->fx_shift);
    }
    RS_HIP(hipGetLastError());
}

// After an epoch: the live items' final merge round (their copies leave the epoch equal).
static void live_merge_after(rs_svd_plan* pl, hipStream_t s) {
    if (pl->live_merged) {
        pl->live_merged = false;
        return;
    }
    if (pl->n_live > 0)
        hipLaunchKernelGGL(svd_live_merge_kernel, dim3(pl->n_live), dim3(64), 0, s, pl->Q.p, pl->live_meta.p,
                           pl->qlast.p, pl->ld, 1);
}

// Split users' pieces (count-weighted deltas in dPs) merged into P after an epoch.
static void merge_split_rows(rs_svd_plan* pl, hipStream_t s) {
    const bool tile = pl->write_back == RS_SGD_WB_TILE;
    const int32_t n = tile ? pl->t_n_split : pl->n_split;
    if (n > 0)
        hipLaunchKernelGGL(svd_merge_rows_kernel, dim3(n), dim3(64), 0, s, pl->P.p, pl->dPs.p,
                           tile ? pl->t_split_rows.p : pl->split_rows.p, pl->ld);
}


int32_t fast_ld(int32_t k) { return 64 * ((k + 1 + 63) / 64); }

void q_convert(rs_svd_plan* pl, hipStream_t s, int32_t to_fixed) {
    const int64_t qn = static_cast<int64_t>(pl->Q.n);
    if (qn == 0) return;
    const int fx_blocks = static_cast<int>(std::min<int64_t>(2048, (qn + 255) / 256));
    hipLaunchKernelGGL(svd_q_fixed_kernel, dim3(fx_blocks), dim3(256), 0, s, pl->Q.p, qn, to_fixed, numflag(pl), pl->fx_shift);
    RS_HIP(hipGetLastError());
}

void merge_tile_split_rows(rs_svd_plan* pl, int32_t r0, int32_t r1, hipStream_t s) {
    if (r1 <= r0) return;
    hipLaunchKernelGGL(svd_merge_rows_kernel, dim3(r1 - r0), dim3(64), 0, s, pl->P.p, pl->dPs.p,
                       pl->t_split_rows.p + r0, pl->ld);
    RS_HIP(hipGetLastError());
}

void gb_sum(const double* partial, int64_t n, double* out, hipStream_t s) {
    hipLaunchKernelGGL(gb_sum_kernel, dim3(1), dim3(256), 0, s, partial, n, out);
    RS_HIP(hipGetLastError());
}

int32_t* numflag(rs_svd_plan* pl) {
    if (!pl->numflag.p) {
        pl->numflag.alloc(1);
        RS_HIP(hipMemsetAsync(pl->numflag.p, 0, sizeof(int32_t), pl->ctx->stream));
        RS_HIP(hipStreamSynchronize(pl->ctx->stream));
    }
    return pl->numflag.p;
}

void plan_sync_last(rs_svd_plan* pl) {
    if (pl->last_stream) RS_HIP(hipStreamSynchronize(pl->last_stream));
}

// new factors: the guard's loss history starts over
static void reset_loss(rs_svd_plan* pl, hipStream_t s) {
    if (pl->loss_state.p) RS_HIP(hipMemsetAsync(pl->loss_state.p, 0, sizeof(double), s));
}


// Item row copies from the host CSR: an item with deg > cap gets R = ceil(deg / cap) rows (its own
// plus R - 1 appended after n_items); its ratings are dealt in user-CSR order, the s-th rating of the
// item going to piece floor(s R / deg), so piece c takes positions [ceil(c deg / R), ceil((c + 1) deg
// / R)) and its merge weight is that count / deg.  cap = item_cap when set; with item_cap = 0 (the
// default) only the items too hot for hot replicas (deg > kAutoItemCap x live_copies) are cut, into
// kAutoItemCap-rating pieces.  Q is (re)allocated to n_qrows rows keeping the item rows; copies are
// synced from them.
static void sync_item_copies(rs_svd_plan* pl, hipStream_t s, int32_t mode) {
    if (pl->n_isplit > 0)
        hipLaunchKernelGGL(svd_item_merge_kernel, dim3(pl->n_isplit), dim3(64), 0, s, pl->Q.p,
                           pl->isplit_meta.p, pl->isplit_frac.p, pl->ld, mode);
    if (pl->n_live > 0) {
        if (mode == 0)
            live_merge_after(pl, s);  // delta-sum round (live items are never averaged)
        else
            hipLaunchKernelGGL(svd_item_merge_kernel, dim3(pl->n_live), dim3(64), 0, s, pl->Q.p,
                               pl->live_meta.p, pl->isplit_frac.p, pl->ld, 1);
    }
}

// measured at configs[4] (Zipf head of 3.4M ratings in a 1/8 shard): 8 live copies of such an item
// diverge to NaN within 5 epochs where 52 averaged copies of 65536 ratings train
constexpr int64_t kAutoItemCap = 65536;

static void build_items(rs_svd_plan* pl) {
    hipStream_t s = pl->ctx->stream;
    const int32_t ni = pl->n_items;
    const std::vector<int32_t>& cols = pl->h_cols;
    std::vector<int64_t> deg(std::max(1, ni), 0);
    for (int32_t c : cols) deg[c]++;
    std::vector<int32_t> R(std::max(1, ni), 1), first(std::max(1, ni), 0);
    std::vector<int4> meta, live;
    std::vector<float> frac;
    int32_t extra = 0;
    // hot replicas (live-merged copies): the live_req most-rated items with at least one rating per copy
    std::vector<uint8_t> is_live(std::max(1, ni), 0);
    const int64_t cap = pl->item_cap > 0 ? pl->item_cap : kAutoItemCap;
    const int64_t split_above = pl->item_cap > 0 ? cap : cap * pl->live_copies;
    if (pl->live_req > 0) {
        std::vector<int32_t> order;
        // an item that the cap would cut into more than live_copies pieces is split instead
        for (int32_t x = 0; x < ni; ++x)
            if (deg[x] >= pl->live_copies && deg[x] <= cap * pl->live_copies) order.push_back(x);
        const size_t nh = std::min(order.size(), static_cast<size_t>(pl->live_req));
        std::partial_sort(order.begin(), order.begin() + nh, order.end(), [&](int32_t a, int32_t b) {
            return deg[a] != deg[b] ? deg[a] > deg[b] : a < b;
        });
        for (size_t h = 0; h < nh; ++h) is_live[order[h]] = 1;
    }
    for (int32_t x = 0; x < ni; ++x) {
        if (is_live[x]) {
            R[x] = pl->live_copies;
            first[x] = ni + extra;
            live.push_back(make_int4(x, ni + extra, R[x], 0));
            extra += R[x] - 1;
        } else if (deg[x] > split_above) {
            R[x] = static_cast<int32_t>((deg[x] + cap - 1) / cap);
            first[x] = ni + extra;
            meta.push_back(make_int4(x, ni + extra, R[x], static_cast<int32_t>(frac.size())));
            for (int32_t c = 0; c < R[x]; ++c) {  // the deal's own bounds (see deal below)
                const int64_t lo = (deg[x] * c + R[x] - 1) / R[x], hi = (deg[x] * (c + 1) + R[x] - 1) / R[x];
                frac.push_back(static_cast<float>(static_cast<double>(hi - lo) / deg[x]));
            }
            extra += R[x] - 1;
        }
    }
    std::vector<int32_t> remap(cols.size() + 128, 0);
    if (extra == 0) {
        std::copy(cols.begin(), cols.end(), remap.begin());  // no copies: the item ids as they are
    } else {
        // Two passes over column chunks on host threads: the per-item position counter of a hot item is a
        // serial store-to-load chain, so one thread walks ~10 ns per hot rating. Pass 1 counts each
        // chunk's ratings of split/live items, an exclusive prefix over chunks gives each chunk its
        // starting positions, pass 2 deals pieces exactly as the serial walk would (same output).
        const size_t n = cols.size();
        const int nt = n >= (size_t{1} << 18) ? 8 : 1;
        std::vector<std::vector<int64_t>> cnt(nt, std::vector<int64_t>(std::max(1, ni), 0));
        auto range = [&](int c, size_t& b, size_t& e) { b = n * c / nt; e = n * (c + 1) / nt; };
        auto count = [&](int c) {
            size_t b, e;
            range(c, b, e);
            std::vector<int64_t>& k = cnt[c];
            for (size_t t = b; t < e; ++t)
                if (R[cols[t]] > 1) k[cols[t]]++;
        };
        auto deal = [&](int c) {
            size_t b, e;
            range(c, b, e);
            std::vector<int64_t>& seen = cnt[c];
            for (size_t t = b; t < e; ++t) {
                const int32_t x = cols[t];
                if (R[x] == 1) {  // the common case: no 64-bit division per rating
                    remap[t] = x;
                    continue;
                }
                const int32_t p = static_cast<int32_t>(seen[x]++ * R[x] / deg[x]);
                remap[t] = p == 0 ? x : first[x] + p - 1;
            }
        };
        auto run = [&](auto&& fn) {
            std::vector<std::thread> th;
            for (int c = 1; c < nt; ++c) th.emplace_back(fn, c);
            fn(0);
            for (std::thread& t : th) t.join();
        };
        run(count);
        for (int32_t x = 0; x < ni; ++x) {
            if (R[x] == 1) continue;
            int64_t acc = 0;
            for (int c = 0; c < nt; ++c) {
                const int64_t v = cnt[c][x];
                cnt[c][x] = acc;
                acc += v;
            }
        }
        run(deal);
    }
    const int32_t rows = ni + extra;
    if (static_cast<int64_t>(std::max(1, rows)) * pl->ld * 4 >= (int64_t{1} << 31) - 64)
        throw std::invalid_argument("item rows * n_factors too large for 32-bit buffer offsets");
    plan_sync_last(pl);
    pl->items.alloc(remap.size());
    pl->items.upload(remap.data(), remap.size(), s);
    pl->n_live = static_cast<int32_t>(live.size());
    pl->live_meta.alloc(std::max<size_t>(1, live.size()));
    pl->live_meta.upload(live.data(), live.size(), s);
    pl->qlast.alloc(static_cast<size_t>(std::max(1, pl->n_live)) * pl->ld);
    if (!pl->done.p) pl->done.alloc(1);
    pl->n_isplit = static_cast<int32_t>(meta.size());
    pl->isplit_meta.alloc(std::max<size_t>(1, meta.size()));
    pl->isplit_frac.alloc(std::max<size_t>(1, frac.size()));
    pl->isplit_meta.upload(meta.data(), meta.size(), s);
    pl->isplit_frac.upload(frac.data(), frac.size(), s);
    const size_t need = static_cast<size_t>(std::max(1, rows)) * pl->ld;
    if (pl->Q.n != need) {
        DevBuf<float> q(need);
        RS_HIP(hipMemsetAsync(q.p, 0, need * sizeof(float), s));
        if (pl->Q.p)
            RS_HIP(hipMemcpyAsync(q.p, pl->Q.p, static_cast<size_t>(std::max(1, ni)) * pl->ld * sizeof(float),
                                  hipMemcpyDeviceToDevice, s));
        pl->Q = std::move(q);
    }
    pl->n_qrows = rows;
    sync_item_copies(pl, s, 1);
    RS_HIP(hipStreamSynchronize(s));  // host vectors die with this scope
}

// Work items from the host CSR: whole user rows, users with more than split_cap ratings cut into
// ceil(deg / split_cap) near-equal pieces (the split of or_svd_fit_chunked); LPT order (longest
// first, ties by user then piece); empty users dropped.
static void build_work(rs_svd_plan* pl) {
    hipStream_t s = pl->ctx->stream;
    const std::vector<int64_t>& rp = pl->h_rowptr;
    struct Item { int32_t u; int64_t b, e; float frac; };
    std::vector<Item> wk;
    std::vector<int32_t> split;
    for (int32_t u = 0; u < pl->n_users; ++u) {
        const int64_t d = rp[u + 1] - rp[u];
        if (d == 0) continue;
        const int64_t pieces = pl->split_cap > 0 ? (d + pl->split_cap - 1) / pl->split_cap : 1;
        if (pieces > 1) split.push_back(u);
        for (int64_t x = 0; x < pieces; ++x) {
            const int64_t b = rp[u] + d * x / pieces, e = rp[u] + d * (x + 1) / pieces;
            wk.push_back({u, b, e, pieces > 1 ? static_cast<float>(static_cast<double>(e - b) / d) : 1.f});
        }
    }
    std::stable_sort(wk.begin(), wk.end(), [](const Item& x, const Item& y) { return x.e - x.b > y.e - y.b; });
    std::vector<int32_t> wu(wk.size());
    std::vector<int64_t> wr(2 * wk.size());
    std::vector<float> wf(wk.size());
    for (size_t x = 0; x < wk.size(); ++x) {
        wu[x] = wk[x].u;
        wr[2 * x] = wk[x].b;
        wr[2 * x + 1] = wk[x].e;
        wf[x] = wk[x].frac;
    }
    plan_sync_last(pl);
    pl->n_work = static_cast<int32_t>(wk.size());
    pl->n_heavy = 0;
    if (pl->heavy_min > 0)
        while (pl->n_heavy < pl->n_work && wr[2 * pl->n_heavy + 1] - wr[2 * pl->n_heavy] >= pl->heavy_min) ++pl->n_heavy;
    pl->n_blocks = fast_blocks(pl);
    pl->wk_user.alloc(std::max<size_t>(1, wu.size()));
    pl->wk_rng.alloc(std::max<size_t>(2, wr.size()));
    pl->wk_frac.alloc(std::max<size_t>(1, wf.size()));
    pl->partial.alloc(pl->n_work + 1 + (pl->n_live + 3) / 4);  // >= blocks of any mode (+ live mergers)
    pl->wk_user.upload(wu.data(), wu.size(), s);
    pl->wk_rng.upload(wr.data(), wr.size(), s);
    pl->wk_frac.upload(wf.data(), wf.size(), s);
    pl->n_split = static_cast<int32_t>(split.size());
    pl->split_rows.alloc(std::max<size_t>(1, split.size()));
    pl->split_rows.upload(split.data(), split.size(), s);
    if (pl->n_split > 0 && pl->dPs.n != static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld) {
        pl->dPs.alloc(static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld);
        RS_HIP(hipMemsetAsync(pl->dPs.p, 0, pl->dPs.n * sizeof(float), s));
    }
    RS_HIP(hipStreamSynchronize(s));  // host vectors die with this scope
}

// The per-user schedules' structures (hybrid / direct / store write-back): the user-CSR item ids
// with hot-item copies, the ratings and the work list.  Built when a plan first runs in one of those
// modes (the tile schedule, the default, has its own arrays).
static void ensure_hybrid(rs_svd_plan* pl) {
    if (pl->hybrid_built) return;
    ensure_host_csr(pl);
    hipStream_t s = pl->ctx->stream;
    // items / ratings padded by 128 entries: the kernels read 32-entry chunks up to two ahead
    // (entries < e + 96 for a row ending at e)
    std::vector<float> v(pl->h_vals);
    v.resize(v.size() + 128, 0.f);
    plan_sync_last(pl);
    pl->ratings.alloc(v.size());
    pl->ratings.upload(v.data(), v.size(), s);
    build_items(pl);
    build_work(pl);
    pl->hybrid_built = true;
    RS_HIP(hipStreamSynchronize(s));
}

// Plan from a user-CSR (data order inside each row); the COO entry point builds it first.
static void plan_build_csr(rs_ctx* ctx, int32_t n_users, int32_t n_items, UserCSR&& csr, int32_t k,
                           rs_svd_plan* pl) {
    hipStream_t s = ctx->stream;
    pl->ctx = ctx;
    pl->light_blocks = default_light_blocks(ctx);
    pl->n_users = n_users;
    pl->n_items = n_items;
    pl->k = k;
    pl->ld = fast_ld(k);
    pl->nnz = static_cast<int64_t>(csr.cols.size());
    {
        double sum = 0.0, lo = 0.0, hi = 0.0;
        for (size_t t = 0; t < csr.vals.size(); ++t) {
            const double v = csr.vals[t];
            sum += v;
            lo = t == 0 ? v : std::min(lo, v);
            hi = t == 0 ? v : std::max(hi, v);
        }
        pl->mean_rating = pl->nnz > 0 ? sum / static_cast<double>(pl->nnz) : 0.0;
        pl->fx_shift = fx_shift_for(lo, hi, pl->mean_rating);  // the fixed-point scale follows the ratings
    }
    pl->h_rowptr = std::move(csr.rowptr);
    pl->h_cols = std::move(csr.cols);
    pl->h_vals = std::move(csr.vals);
    pl->P.alloc(static_cast<size_t>(std::max(1, n_users)) * pl->ld);
    RS_HIP(hipMemsetAsync(pl->P.p, 0, pl->P.n * sizeof(float), s));
    (void)buffer_bytes32(static_cast<size_t>(std::max(1, n_items)) * pl->ld, sizeof(float), "item factor matrix");
    pl->Q.alloc(static_cast<size_t>(std::max(1, n_items)) * pl->ld);
    RS_HIP(hipMemsetAsync(pl->Q.p, 0, pl->Q.n * sizeof(float), s));
    pl->n_qrows = n_items;
    static const bool trace = std::getenv("RSGPU_FIT_TRACE") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    if (pl->write_back == RS_SGD_WB_TILE) tile_build(pl);
    else ensure_hybrid(pl);
    if (trace)
        std::fprintf(stderr, "fit-trace   schedule %8.3f ms\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    pl->gb.alloc(1);
    RS_HIP(hipMemsetAsync(pl->gb.p, 0, sizeof(double), s));
    RS_HIP(hipEventCreate(&pl->ev0));
    RS_HIP(hipEventCreate(&pl->ev1));
    RS_HIP(hipStreamSynchronize(s));  // host CSR vectors die with this scope
}

// One-shot Fit's plan (RS_SGD_WB_TILE, at most kDeviceBuildMaxNnz ratings): the COO goes to the device as it
// is (ratings rounded to f32 on the host threads, one pinned staging buffer, three DMAs) and the tile
// schedule is built there (RS_TILE_RULE_FILL_DEVICE, sched_dev.hip): no host CSR, no host schedule.  Where
// the rule does not apply, tile_build falls back to the host CSR (downloaded COO) and the LPT build.
constexpr int64_t kDeviceBuildMaxNnz = int64_t{1} << 24;
static void plan_build_coo_device(rs_ctx* ctx, const rs_ratings* r, int32_t k, rs_svd_plan* pl) {
    hipStream_t s = ctx->stream;
    pl->ctx = ctx;
    pl->light_blocks = default_light_blocks(ctx);
    pl->n_users = r->n_users;
    pl->n_items = r->n_items;
    pl->k = k;
    pl->ld = fast_ld(k);
    pl->nnz = r->nnz;
    pl->tile_rule = RS_TILE_RULE_FILL_DEVICE;
    const size_t n = static_cast<size_t>(r->nnz);
    char* st = static_cast<char*>(pinned_staging(ctx, 12 * n));
    int32_t* su = reinterpret_cast<int32_t*>(st);
    int32_t* si = su + n;
    float* sv = reinterpret_cast<float*>(si + n);
    std::mutex mx;
    double lo = 0.0, hi = 0.0, sum = 0.0;
    bool any = false;
    parallel_ranges(r->nnz, 16, [&](int64_t b, int64_t e) {
        std::memcpy(su + b, r->users + b, static_cast<size_t>(e - b) * 4);
        std::memcpy(si + b, r->items + b, static_cast<size_t>(e - b) * 4);
        double l = 0.0, h = 0.0, sm = 0.0;
        for (int64_t t = b; t < e; ++t) {
            const double v = r->ratings[t];
            sv[t] = static_cast<float>(v);
            l = t == b ? v : std::min(l, v);
            h = t == b ? v : std::max(h, v);
            sm += v;
        }
        if (e > b) {
            std::lock_guard<std::mutex> g(mx);
            lo = any ? std::min(lo, l) : l;
            hi = any ? std::max(hi, h) : h;
            sum += sm;
            any = true;
        }
    });
    // the fixed-point scale follows the ratings' spread (fx_shift_for); the mean only places the range
    pl->fx_shift = fx_shift_for(lo, hi, r->nnz > 0 ? sum / static_cast<double>(r->nnz) : 0.0);
    // (buffers recycled from the previous Fit's plan are kept where large enough; P and Q must fit exactly)
    if (pl->coo_users.n < n) pl->coo_users.alloc(n);
    if (pl->coo_items.n < n) pl->coo_items.alloc(n);
    if (pl->coo_vals.n < n) pl->coo_vals.alloc(n);
    pl->coo_users.upload(su, n, s);
    pl->coo_items.upload(si, n, s);
    pl->coo_vals.upload(sv, n, s);
    const size_t pn = static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld, qn = static_cast<size_t>(std::max(1, pl->n_items)) * pl->ld;
    (void)buffer_bytes32(qn, sizeof(float), "item factor matrix");
    if (pl->P.n != pn) {
        pl->P.alloc(pn);
        RS_HIP(hipMemsetAsync(pl->P.p, 0, pn * sizeof(float), s));
    }
    if (pl->Q.n != qn) {
        pl->Q.alloc(qn);
        RS_HIP(hipMemsetAsync(pl->Q.p, 0, qn * sizeof(float), s));
    }
    pl->n_qrows = pl->n_items;
    if (!pl->gb.p) pl->gb.alloc(1);
    RS_HIP(hipMemsetAsync(pl->gb.p, 0, sizeof(double), s));
    if (!pl->ev0) RS_HIP(hipEventCreate(&pl->ev0));
    if (!pl->ev1) RS_HIP(hipEventCreate(&pl->ev1));
    static const bool trace = std::getenv("RSGPU_FIT_TRACE") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    tile_build(pl);  // syncs the stream (the staging buffer is free again)
    if (trace)
        std::fprintf(stderr, "fit-trace   schedule %8.3f ms (%s)\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                     pl->tile_rule == RS_TILE_RULE_FILL_DEVICE ? "device" : "host fallback");
}

// A new one-shot Fit plan takes over the previous one's device buffers (hipMalloc / hipFree cost tens of us
// each and hipFree waits for the device): the COO, the schedule and its workspace by capacity, P and Q when
// their shapes match, the flag, GlobalBias and the events.
static void plan_recycle(rs_svd_plan* pl, rs_svd_plan* old, int32_t n_users, int32_t n_items, int32_t k) {
    plan_sync_last(old);
    pl->coo_users = std::move(old->coo_users);
    pl->coo_items = std::move(old->coo_items);
    pl->coo_vals = std::move(old->coo_vals);
    pl->sched_ws = std::move(old->sched_ws);
    pl->t_tiles = std::move(old->t_tiles);
    pl->t_users = std::move(old->t_users);
    pl->t_streams = std::move(old->t_streams);
    pl->t_runs = std::move(old->t_runs);
    pl->t_recs = std::move(old->t_recs);
    pl->t_split_rows = std::move(old->t_split_rows);
    pl->partial = std::move(old->partial);
    pl->numflag = std::move(old->numflag);  // (zero: a raised flag is cleared when it is reported)
    if (old->P_snap.n == static_cast<size_t>(std::max(1, n_users)) * fast_ld(k)) pl->P_snap = std::move(old->P_snap);
    if (old->Q_snap.n == static_cast<size_t>(std::max(1, n_items)) * fast_ld(k)) pl->Q_snap = std::move(old->Q_snap);
    pl->gb_snap = std::move(old->gb_snap);
    pl->loss_part = std::move(old->loss_part);    // (the loss history is reset by the upload)
    pl->loss_state = std::move(old->loss_state);
    pl->guard_flag = std::move(old->guard_flag);  // (zero: cleared after every check)
    pl->gb = std::move(old->gb);
    if (old->ld == fast_ld(k) && old->n_users == n_users) pl->P = std::move(old->P);
    if (old->ld == fast_ld(k) && old->n_items == n_items && old->n_qrows == old->n_items) pl->Q = std::move(old->Q);
    std::swap(pl->ev0, old->ev0);
    std::swap(pl->ev1, old->ev1);
}

// rs_svd_fit's factor transfers: f64 <-> the f32 row layout [p, b] on the host threads through pinned
// staging slot 1 (one DMA per matrix, no intermediate vectors); past 256 MiB of rows the plan_upload /
// plan_download path (pageable) is taken instead.
constexpr size_t kFitStageMax = size_t{256} << 20;
// pinned scalars of rs_svd_fit's copies (a copy to or from pageable memory waits for the stream's earlier work,
// which would serialise the host work meant to run under the epochs): [0] GlobalBias in, [1] GlobalBias out,
// [2] flag out (int32) -- the ctx's kPinFit slot
static double* fit_scalars(rs_ctx* ctx) { return static_cast<double*>(pinned_small(ctx, kPinFit)); }

// host half: the rows packed into staging slot 1 (false: too large, nothing done)
static bool plan_pack_fit(rs_svd_plan* pl, const double* P, const double* Q, const double* bu, const double* bi) {
    const size_t pn = static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld, qn = static_cast<size_t>(std::max(1, pl->n_items)) * pl->ld;
    if ((pn + qn) * 4 > kFitStageMax) return false;
    float* st = static_cast<float*>(pinned_staging(pl->ctx, (pn + qn) * 4, 1));
    const int32_t k = pl->k, ld = pl->ld;
    const int64_t nu = pl->n_users, ni = pl->n_items;
    parallel_ranges(nu + ni, 16, [&](int64_t r0, int64_t r1) {  // P rows then Q rows, one pass
        for (int64_t r = r0; r < r1; ++r) {
            const bool u = r < nu;
            const int64_t x = u ? r : r - nu;
            float* d = (u ? st : st + pn) + x * ld;
            const double* F = (u ? P : Q) + x * k;
            for (int32_t f = 0; f < k; ++f) d[f] = static_cast<float>(F[f]);
            d[k] = static_cast<float>((u ? bu : bi)[x]);
            for (int32_t f = k + 1; f < ld; ++f) d[f] = 0.f;
        }
    });
    return true;
}

// device half: the DMAs of the packed rows and GlobalBias (after plan_pack_fit)
static void plan_dma_fit(rs_svd_plan* pl, const double* gb) {
    const size_t pn = static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld, qn = static_cast<size_t>(std::max(1, pl->n_items)) * pl->ld;
    plan_sync_last(pl);
    hipStream_t s = pl->ctx->stream;
    float* st = static_cast<float*>(pinned_staging(pl->ctx, (pn + qn) * 4, 1));
    pl->P.upload(st, static_cast<size_t>(pl->n_users) * pl->ld, s);
    pl->Q.upload(st + pn, static_cast<size_t>(pl->n_items) * pl->ld, s);
    sync_item_copies(pl, s, 1);
    double* sc = fit_scalars(pl->ctx);
    sc[0] = *gb;
    pl->gb.upload(sc, 1, s);
    reset_loss(pl, s);
}

static bool plan_upload_fit(rs_svd_plan* pl, const double* P, const double* Q, const double* bu, const double* bi,
                            const double* gb) {
    if (!plan_pack_fit(pl, P, Q, bu, bi)) return false;
    plan_dma_fit(pl, gb);
    return true;
}

static bool fit_fits_staging(const rs_svd_plan* pl) {
    const size_t pn = static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld, qn = static_cast<size_t>(std::max(1, pl->n_items)) * pl->ld;
    return (pn + qn) * 4 <= kFitStageMax;
}

// enqueues the D2H of P and Q (staging slot 1), GlobalBias and the numeric flag (pinned scalars) on the ctx
// stream; plan_fetch_result reads the scalars after the wait
static void plan_fetch_enqueue(rs_svd_plan* pl) {
    const size_t pn = static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld, qn = static_cast<size_t>(std::max(1, pl->n_items)) * pl->ld;
    hipStream_t s = pl->ctx->stream;
    float* st = static_cast<float*>(pinned_staging(pl->ctx, (pn + qn) * 4, 1));
    double* sc = fit_scalars(pl->ctx);
    pl->P.download(st, static_cast<size_t>(pl->n_users) * pl->ld, s);
    pl->Q.download(st + pn, static_cast<size_t>(pl->n_items) * pl->ld, s);
    pl->gb.download(sc + 1, 1, s);
    int32_t* f = reinterpret_cast<int32_t*>(sc + 2);
    *f = 0;
    if (pl->numflag.p) RS_HIP(hipMemcpyAsync(f, pl->numflag.p, sizeof(int32_t), hipMemcpyDeviceToHost, s));
}
static void plan_fetch_result(rs_ctx* ctx, double* gb, int32_t* flag) {
    const double* sc = fit_scalars(ctx);
    *gb = sc[1];
    *flag = *reinterpret_cast<const int32_t*>(sc + 2);
}


static void plan_clear_flag(rs_svd_plan* pl) {
    RS_HIP(hipMemsetAsync(pl->numflag.p, 0, sizeof(int32_t), pl->ctx->stream));
    RS_HIP(hipStreamSynchronize(pl->ctx->stream));
}

// after plan_fetch_enqueue and a wait: the f64 rows; a raised flag is cleared and reported (values already written)
static void plan_finish_fit(rs_svd_plan* pl, double* P, double* Q, double* bu, double* bi, int32_t flag) {
    const size_t pn = static_cast<size_t>(std::max(1, pl->n_users)) * pl->ld;
    const float* st = static_cast<const float*>(pinned_staging(pl->ctx, 0, 1));
    const int32_t k = pl->k, ld = pl->ld;
    const int64_t nu = pl->n_users, ni = pl->n_items;
    parallel_ranges(nu + ni, 16, [&](int64_t r0, int64_t r1) {  // P rows then Q rows, one pass
        for (int64_t r = r0; r < r1; ++r) {
            const bool u = r < nu;
            const int64_t x = u ? r : r - nu;
            const float* a = (u ? st : st + pn) + x * ld;
            double* F = (u ? P : Q) + x * k;
            for (int32_t f = 0; f < k; ++f) F[f] = a[f];
            (u ? bu : bi)[x] = a[k];
        }
    });
    if (flag) {
        plan_clear_flag(pl);
        throw NumericError{"item factors left the fixed-point range (non-finite or |q| >= 2^(31 - shift)) during "
                           "an epoch; the returned model is not trustworthy"};
    }
}


static void plan_build(rs_ctx* ctx, const rs_ratings* r, int32_t k, rs_svd_plan* pl) {
    UserCSR csr;
    build_csr(r->nnz, r->n_users, r->users, r->items, r->ratings, csr);
    plan_build_csr(ctx, r->n_users, r->n_items, std::move(csr), k, pl);
}

// Factor init on the device (svd.go:77-85: biases 0, factor entries N(mean, std), users then items;
// the Go draws come from the unseeded global math/rand, Q4, so only the distribution is kept): entry
// (row, f) of the P-then-Q row sequence is mean + std * Box-Muller(hash(seed, row, f)).
__device__ __forceinline__ uint64_t dev_splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void init_normal_kernel(float* __restrict__ F, int64_t rows, int64_t row0,
                                                          int32_t k, int32_t ld, double mean, double sd,
                                                          uint64_t seed) {
    const int64_t n = rows * ld;
    for (int64_t x = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; x < n;
         x += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t r = x / ld;
        const int32_t f = static_cast<int32_t>(x - r * ld);
        float v = 0.f;
        if (f < k) {
            const uint64_t h = dev_splitmix(dev_splitmix(seed ^ static_cast<uint64_t>(row0 + r)) ^ static_cast<uint64_t>(f));
            const double u1 = (static_cast<double>(h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
            const double u2 = (static_cast<double>(dev_splitmix(h) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
            v = static_cast<float>(mean + sd * (sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2)));
        }
        F[x] = v;
    }
}

static void plan_init_normal(rs_svd_plan* pl, double mean, double sd, uint64_t seed) {
    plan_sync_last(pl);
    hipStream_t s = pl->ctx->stream;
    hipLaunchKernelGGL(init_normal_kernel, dim3(4096), dim3(256), 0, s, pl->P.p, static_cast<int64_t>(pl->n_users),
                       int64_t{0}, pl->k, pl->ld, mean, sd, seed);
    hipLaunchKernelGGL(init_normal_kernel, dim3(4096), dim3(256), 0, s, pl->Q.p, static_cast<int64_t>(pl->n_items),
                       static_cast<int64_t>(pl->n_users), pl->k, pl->ld, mean, sd, seed);
    RS_HIP(hipGetLastError());
    sync_item_copies(pl, s, 1);
    // FAST GlobalBias warm start (common.hpp gb_warm_start) with zero biases: the mean rating
    const double gb = pl->mean_rating;
    pl->gb.upload(&gb, 1, s);
    RS_HIP(hipStreamSynchronize(s));
}

// f64 factor rows (stride k) + bias -> f32 rows of ld floats with the bias in column k
static void pack_with_bias(const double* F, const double* bias, int64_t rows, int32_t k, int32_t ld,
                           const std::vector<float>& old, std::vector<float>& dst) {
    dst.assign(static_cast<size_t>(rows) * ld, 0.f);
    for (int64_t r = 0; r < rows; ++r) {
        float* d = dst.data() + r * ld;
        if (F) for (int32_t f = 0; f < k; ++f) d[f] = static_cast<float>(F[r * k + f]);
        else for (int32_t f = 0; f < k; ++f) d[f] = old[r * ld + f];
        d[k] = bias ? static_cast<float>(bias[r]) : old[r * ld + k];
    }
}

static void plan_upload(rs_svd_plan* pl, const double* P, const double* Q, const double* bu,
                        const double* bi, const double* gb) {
    plan_sync_last(pl);
    reset_loss(pl, pl->ctx->stream);
    hipStream_t s = pl->ctx->stream;
    std::vector<float> old, tmp;
    auto put = [&](DevBuf<float>& d, int64_t rows, const double* F, const double* bias) {
        if (!F && !bias) return;
        if (!F || !bias) {  // partial update: keep the other half of the row
            old.resize(static_cast<size_t>(rows) * pl->ld);
            d.download(old.data(), old.size(), s);
            RS_HIP(hipStreamSynchronize(s));
        }
        pack_with_bias(F, bias, rows, pl->k, pl->ld, old, tmp);
        d.upload(tmp.data(), tmp.size(), s);
        RS_HIP(hipStreamSynchronize(s));
    };
    put(pl->P, pl->n_users, P, bu);
    put(pl->Q, pl->n_items, Q, bi);  // item rows; their copies follow
    if (Q || bi) {
        sync_item_copies(pl, s, 1);
        RS_HIP(hipStreamSynchronize(s));
    }
    if (gb) {
        pl->gb.upload(gb, 1, s);
        RS_HIP(hipStreamSynchronize(s));
    }
}

static void plan_download(rs_svd_plan* pl, double* P, double* Q, double* bu, double* bi,
                          double* gb) {
    plan_sync_last(pl);
    hipStream_t s = pl->ctx->stream;
    std::vector<float> tmp;
    auto get = [&](const DevBuf<float>& d, int64_t rows, double* F, double* bias) {
        if (!F && !bias) return;
        tmp.resize(static_cast<size_t>(rows) * pl->ld);
        d.download(tmp.data(), tmp.size(), s);
        RS_HIP(hipStreamSynchronize(s));
        for (int64_t r = 0; r < rows; ++r) {
            if (F) for (int32_t f = 0; f < pl->k; ++f) F[r * pl->k + f] = tmp[r * pl->ld + f];
            if (bias) bias[r] = tmp[r * pl->ld + pl->k];
        }
    };
    get(pl->P, pl->n_users, P, bu);
    get(pl->Q, pl->n_items, Q, bi);
    if (gb) {
        pl->gb.download(gb, 1, s);
        RS_HIP(hipStreamSynchronize(s));
    }
    if (pl->numflag.p) {  // raised by a Q conversion: report once, values already returned
        int32_t f = 0;
        pl->numflag.download(&f, 1, s);
        RS_HIP(hipStreamSynchronize(s));
        if (f) {
            RS_HIP(hipMemsetAsync(pl->numflag.p, 0, sizeof(int32_t), s));
            RS_HIP(hipStreamSynchronize(s));
            throw NumericError{"item factors left the fixed-point range (non-finite or |q| >= 2^(31 - shift)) during "
                               "an epoch; the returned model is not trustworthy"};
        }
    }
}

// rows with an entry at or past `bound` (or non-finite): flag.  The guard scans P and Q at a quarter of the
// plan's fixed-point range (32 on star ratings; the range follows the ratings' spread, fx_shift_for), far past
// any trained factor or bias, so a run-away row is caught while the call can still be redone from a sane start
__global__ __launch_bounds__(256) void range_kernel(const float* __restrict__ P, int64_t np, const float* __restrict__ Q,
                                                   int64_t nq, float bound, int32_t* __restrict__ flag) {
    bool bad = false;
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; t < np + nq; t += static_cast<int64_t>(gridDim.x) * 256)
        bad |= !(fabsf(t < np ? P[t] : Q[t - np]) < bound);
    if (bad) flag[0] = 1;
}

// every P and Q entry finite and below the plan's guard bound (one launch, one readback; the stream is synced)
bool plan_range_ok(rs_svd_plan* pl) {
    plan_sync_last(pl);
    hipStream_t s = pl->ctx->stream;
    if (!pl->guard_flag.p) pl->guard_flag.alloc(1);
    RS_HIP(hipMemsetAsync(pl->guard_flag.p, 0, sizeof(int32_t), s));
    const int64_t pn = static_cast<int64_t>(pl->P.n), qn = static_cast<int64_t>(pl->Q.n);
    hipLaunchKernelGGL(range_kernel, dim3(static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(1024, (pn + qn + 255) / 256)))),
                       dim3(256), 0, s, pl->P.p, pn, pl->Q.p, qn, pl->guard_bound(), pl->guard_flag.p);
    RS_HIP(hipGetLastError());
    int32_t f = 0;
    pl->guard_flag.download(&f, 1, s);
    RS_HIP(hipStreamSynchronize(s));
    if (f) {
        RS_HIP(hipMemsetAsync(pl->guard_flag.p, 0, sizeof(int32_t), s));
        RS_HIP(hipStreamSynchronize(s));
    }
    return f == 0;
}

static void plan_epochs_once(rs_svd_plan* pl, int32_t epochs, float lr, float reg, hipStream_t s) {
    const double inv_nnz = pl->nnz > 0 ? 1.0 / static_cast<double>(pl->nnz) : 0.0;
    if (pl->timing) {
        while (static_cast<int32_t>(pl->tev.size()) < 2 * epochs) {
            hipEvent_t e;
            RS_HIP(hipEventCreate(&e));
            pl->tev.push_back(e);
        }
        pl->tev_used = 2 * epochs;
    }
    RS_HIP(hipEventRecord(pl->ev0, s));
    // Fixed-point runs without item splitting keep Q in int32 for all their epochs: one conversion
    // each way per call, and per epoch the SGD kernel plus one epilogue launch (merge rounds, split
    // rows, GlobalBias fold) instead of six small launches.
    const bool tile = pl->write_back == RS_SGD_WB_TILE;
    const bool hoist = (tile || (pl->fixed_q && pl->write_back == RS_SGD_WB_ATOMIC && pl->n_isplit == 0)) && epochs > 0;
    const int64_t qn = static_cast<int64_t>(pl->Q.n);
    const int fx_blocks = static_cast<int>(std::min<int64_t>(2048, (qn + 255) / 256));
    if (hoist) {
        hipLaunchKernelGGL(svd_q_fixed_kernel, dim3(fx_blocks), dim3(256), 0, s, pl->Q.p, qn, 1, numflag(pl), pl->fx_shift);
        if (!tile && pl->n_live > 0) {
            hipLaunchKernelGGL(svd_live_merge_kernel, dim3(pl->n_live), dim3(64), 0, s, pl->Q.p, pl->live_meta.p,
                               pl->qlast.p, pl->ld, 0);
            RS_HIP(hipMemsetAsync(pl->done.p, 0, sizeof(int32_t), s));
        }
        // the guard's loss check: tile epochs of a guarded plan (loss partials written by the kernel)
        const bool loss_on = tile && pl->guard && lr > 0.f && pl->loss_state.p && pl->guard_flag.p &&
                             pl->loss_part.n >= pl->partial.n;
        struct HoistScope {  // launch_fast sees the hoisted state only inside this loop, even on a throw
            rs_svd_plan* p;
            ~HoistScope() { p->hoisted = false; }
        } scope{pl};
        pl->hoisted = true;
        for (int32_t e = 0; e < epochs; ++e) {
            if (pl->timing) RS_HIP(hipEventRecord(pl->tev[2 * e], s));
            launch_fast(pl, lr, reg, s);
            if (pl->timing) RS_HIP(hipEventRecord(pl->tev[2 * e + 1], s));
            const int32_t n_live = tile ? 0 : pl->n_live, n_split = tile ? pl->t_n_split : pl->n_split;
            hipLaunchKernelGGL(svd_epoch_epilogue_kernel, dim3(n_live + n_split + 1), dim3(kEpilogueThreads), 0, s,
                               reinterpret_cast<int32_t*>(pl->Q.p), pl->live_meta.p,
                               reinterpret_cast<int32_t*>(pl->qlast.p), n_live, pl->P.p, pl->dPs.p,
                               tile ? pl->t_split_rows.p : pl->split_rows.p, n_split, pl->ld, pl->partial.p,
                               static_cast<int64_t>(pl->n_blocks), pl->gb.p, inv_nnz,
                               n_live > 0 ? pl->done.p : nullptr, loss_on ? pl->loss_part.p : nullptr,
                               loss_on ? pl->loss_state.p : nullptr, loss_on ? pl->guard_flag.p : nullptr,
                               1.0 / (static_cast<double>(lr) * static_cast<double>(lr)),
                               tile && pl->gb_fold == RS_GB_FOLD_SMOOTH ? pl->gb_smooth.p : nullptr,
                               std::exp(static_cast<double>(pl->nnz) * std::log1p(-static_cast<double>(lr))));
            RS_HIP(hipGetLastError());
        }
        pl->hoisted = false;
        hipLaunchKernelGGL(svd_q_fixed_kernel, dim3(fx_blocks), dim3(256), 0, s, pl->Q.p, qn, 0, numflag(pl), pl->fx_shift);
        RS_HIP(hipGetLastError());
        RS_HIP(hipEventRecord(pl->ev1, s));
        pl->last_launches = pl->timing ? epochs : 2 * epochs;  // SGD + epilogue (conversions in the span)
        pl->last_stream = s;
        pl->last_ms = -1.0;
        return;
    }
    for (int32_t e = 0; e < epochs; ++e) {
        if (pl->timing) RS_HIP(hipEventRecord(pl->tev[2 * e], s));
        launch_fast(pl, lr, reg, s);
        if (pl->timing) RS_HIP(hipEventRecord(pl->tev[2 * e + 1], s));
        merge_split_rows(pl, s);
        sync_item_copies(pl, s, 0);
        hipLaunchKernelGGL(gb_fold_kernel, dim3(1), dim3(256), 0, s, pl->partial.p,
                           static_cast<int64_t>(pl->n_blocks), pl->gb.p, inv_nnz);
        RS_HIP(hipGetLastError());
    }
    RS_HIP(hipEventRecord(pl->ev1, s));
    pl->last_launches = pl->timing ? epochs : (2 + (pl->n_split > 0) + (pl->n_isplit > 0)) * epochs;
    pl->last_stream = s;
    pl->last_ms = -1.0;  // resolved lazily by rs_svd_plan_last_kernel_ms
}

// The divergence guard (tile schedule).  What diverges under the FAST schedule is a hot item's
// q_i / b_i: the updates other runs apply between a run's read of the row and its write grow with the
// chip-wide update rate, i.e. with the workgroups in flight, and halving them (and
// the run cap: the automatic cap would grow as the grid shrinks) halves that staleness.  So a call's epochs are checked once, at the end (the Q conversion's range flag, a P range
// scan, a finite GlobalBias: one small readback), and a call that failed is redone from its start state --
// P, Q and GlobalBias copied on the device before the first epoch -- on a quarter of the workgroups, up to three
// times; the plan keeps the smaller grid and cap where a hard signal (range flag, non-finite) fired or soft redos
// keep coming (see the end of the loop).  Only then does the caller see the flag (RS_ERR_NUMERIC at download).
// `under` is host work run while the first attempt's kernels execute.
static void plan_epochs(rs_svd_plan* pl, int32_t epochs, float lr, float reg, hipStream_t s,
                        const std::function<void()>& under = nullptr, const std::function<void()>& after = nullptr) {
    // `after` enqueues the caller's follow-up copies (rs_svd_fit: the results' download) before the guard's wait
    if (pl->tiles_deferred && !pl->tiles_built && pl->write_back == RS_SGD_WB_TILE) {  // (after a soft redo)
        tile_build(pl);
        pl->n_blocks = tile_partials(pl);
    }
    pl->tiles_deferred = false;
    const bool guarded = pl->guard && pl->write_back == RS_SGD_WB_TILE && epochs > 0 && pl->tiles_built;
    if (!guarded) {
        plan_epochs_once(pl, epochs, lr, reg, s);
        if (after) after();
        if (under) under();
        return;
    }
    if (pl->P_snap.n != pl->P.n) pl->P_snap.alloc(pl->P.n);
    if (pl->Q_snap.n != pl->Q.n) pl->Q_snap.alloc(pl->Q.n);
    if (!pl->gb_snap.p) pl->gb_snap.alloc(2);
    if (pl->loss_part.n < pl->partial.n) pl->loss_part.alloc(pl->partial.n);
    if (!pl->loss_state.p) {
        pl->loss_state.alloc(1);
        RS_HIP(hipMemsetAsync(pl->loss_state.p, 0, sizeof(double), s));
    }
    if (!pl->guard_flag.p) {  // (zero between calls: cleared after every check)
        pl->guard_flag.alloc(1);
        RS_HIP(hipMemsetAsync(pl->guard_flag.p, 0, sizeof(int32_t), s));
    }
    RS_HIP(hipMemcpyAsync(pl->P_snap.p, pl->P.p, pl->P.n * sizeof(float), hipMemcpyDeviceToDevice, s));
    RS_HIP(hipMemcpyAsync(pl->Q_snap.p, pl->Q.p, pl->Q.n * sizeof(float), hipMemcpyDeviceToDevice, s));
    RS_HIP(hipMemcpyAsync(pl->gb_snap.p, pl->gb.p, sizeof(double), hipMemcpyDeviceToDevice, s));
    RS_HIP(hipMemcpyAsync(pl->gb_snap.p + 1, pl->loss_state.p, sizeof(double), hipMemcpyDeviceToDevice, s));
    struct Check {  // pinned readback slot: the ctx's kPinGuard
        int64_t* p;
    } ck{static_cast<int64_t*>(pinned_small(pl->ctx, kPinGuard))};
    int32_t* flag = numflag(pl);
    bool hard = false;  // a hard signal (the fixed-point range flag, a non-finite GlobalBias) in this call
    const int32_t wg0 = pl->tile_wg, cap0 = pl->tile_run_cap;
    for (int attempt = 0;; ++attempt) {
        plan_epochs_once(pl, epochs, lr, reg, s);
        const int64_t pn = static_cast<int64_t>(pl->P.n), qn = static_cast<int64_t>(pl->Q.n);
        hipLaunchKernelGGL(range_kernel, dim3(static_cast<int>(std::min<int64_t>(1024, (pn + qn + 255) / 256))), dim3(256), 0, s,
                           pl->P.p, pn, pl->Q.p, qn, pl->guard_bound(), pl->guard_flag.p);
        RS_HIP(hipGetLastError());
        RS_HIP(hipMemcpyAsync(ck.p, pl->gb.p, sizeof(double), hipMemcpyDeviceToHost, s));
        RS_HIP(hipMemcpyAsync(ck.p + 1, flag, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        RS_HIP(hipMemcpyAsync(reinterpret_cast<int32_t*>(ck.p + 1) + 1, pl->guard_flag.p, sizeof(int32_t),
                              hipMemcpyDeviceToHost, s));
        if (after) after();
        if (attempt == 0 && under) under();
        RS_HIP(hipStreamSynchronize(s));
        double g;
        std::memcpy(&g, ck.p, 8);
        const int32_t* fl = reinterpret_cast<const int32_t*>(ck.p + 1);
        const bool bad_hard = fl[0] != 0 || !std::isfinite(g), bad = bad_hard || fl[1] != 0;
        hard = hard || bad_hard;
        static const bool trace_check = std::getenv("RSGPU_FIT_TRACE") != nullptr;
        if (trace_check) {  // every check: the signals and this epoch's training MSE
            double mse = 0.0;
            RS_HIP(hipMemcpy(&mse, pl->loss_state.p, sizeof(double), hipMemcpyDeviceToHost));
            std::fprintf(stderr, "fit-trace check: attempt %d range %d guard %d gb %.6f training mse %.6f\n", attempt, fl[0], fl[1], g, mse);
        }
        RS_HIP(hipMemsetAsync(pl->guard_flag.p, 0, sizeof(int32_t), s));  // (the guard's own signal is never an error)
        if (!bad || attempt == 3 || pl->tile_grid <= 1) {  // (a range flag still raised reaches the download)
            // Redos that only the guard's own signals asked for (a rising loss, a factor past the guard bound) may
            // be false positives: the plan returns to the caller's grid and cap for its next call instead of keeping
            // a quarter of the workgroups for good -- until such redos have come three times, or a hard signal (range
            // flag, non-finite) came in this call, when the smaller grid stays.  The schedule is rebuilt by whatever
            // next runs or reads it (tiles_built; rs_svd_fit's plan may never run again).
            if (attempt > 0 && !bad && !hard && ++pl->soft_refits < 3 &&
                (pl->tile_wg != wg0 || pl->tile_run_cap != cap0)) {
                pl->tile_wg = wg0;
                pl->tile_run_cap = cap0;
                pl->tiles_built = false;
                pl->tiles_deferred = true;
            }
            return;
        }
        RS_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
        RS_HIP(hipMemcpyAsync(pl->P.p, pl->P_snap.p, pl->P.n * sizeof(float), hipMemcpyDeviceToDevice, s));
        RS_HIP(hipMemcpyAsync(pl->Q.p, pl->Q_snap.p, pl->Q.n * sizeof(float), hipMemcpyDeviceToDevice, s));
        RS_HIP(hipMemcpyAsync(pl->gb.p, pl->gb_snap.p, sizeof(double), hipMemcpyDeviceToDevice, s));
        RS_HIP(hipMemcpyAsync(pl->loss_state.p, pl->gb_snap.p + 1, sizeof(double), hipMemcpyDeviceToDevice, s));
        RS_HIP(hipStreamSynchronize(s));
        const int32_t cap = tile_cap_in_use(pl);  // (before the grid changes: the automatic cap depends on it)
        pl->tile_wg = std::max(1, pl->tile_grid / 4);
        pl->tile_run_cap = std::max(2, cap / 2);
        tile_build(pl);
        pl->n_blocks = tile_partials(pl);
        ++pl->refits;
        static const bool trace = std::getenv("RSGPU_FIT_TRACE") != nullptr;
        if (trace) std::fprintf(stderr, "fit-trace diverged: redone on %d workgroups\n", pl->tile_wg);
    }
}

static int check_sgd(rs_ctx* ctx, const rs_ratings* r, const rs_sgd_params* p) {
    int st = check_ratings(ctx, r);
    if (st != RS_OK) return st;
    if (!p) return set_error(ctx, RS_ERR_INVALID, "params is NULL");
    if (p->n_factors < 1 || p->n_factors > kMaxFactors)
        return set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 510]");
    if (p->n_epochs < 0) return set_error(ctx, RS_ERR_INVALID, "n_epochs < 0");
    if (p->mode != RS_SGD_FAST && p->mode != RS_SGD_ORDERED)
        return set_error(ctx, RS_ERR_INVALID, "unknown SGD mode");
    return RS_OK;
}

}  // namespace rs

// ------------------------------------------------------------------------------------------------
// C-ABI

extern "C" int rs_svd_plan_create(rs_ctx* ctx, const rs_ratings* r, int32_t n_factors,
                                  rs_svd_plan** out) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        if (!out) return rs::set_error(ctx, RS_ERR_INVALID, "out is NULL");
        *out = nullptr;
        int st = rs::check_ratings(ctx, r);
        if (st != RS_OK) return st;
        if (n_factors < 1 || n_factors > rs::kMaxFactors)
            return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 510]");
        auto* pl = new rs_svd_plan();
        try {
            rs::plan_build(ctx, r, n_factors, pl);
        } catch (...) {
            delete pl;
            throw;
        }
        *out = pl;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_create_csr(rs_ctx* ctx, int32_t n_users, int32_t n_items, const int64_t* rowptr,
                                      const int32_t* cols, const float* vals, int32_t n_factors,
                                      rs_svd_plan** out) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        if (!out) return rs::set_error(ctx, RS_ERR_INVALID, "out is NULL");
        *out = nullptr;
        if (n_users < 0 || n_items < 0 || !rowptr) return rs::set_error(ctx, RS_ERR_INVALID, "bad CSR sizes");
        if (n_factors < 1 || n_factors > rs::kMaxFactors)
            return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 510]");
        if (rowptr[0] != 0) return rs::set_error(ctx, RS_ERR_INVALID, "rowptr[0] != 0");
        for (int32_t u = 0; u < n_users; ++u)
            if (rowptr[u + 1] < rowptr[u]) return rs::set_error(ctx, RS_ERR_INVALID, "rowptr not monotone at " + std::to_string(u));
        const int64_t nnz = rowptr[n_users];
        if (nnz > 0 && (!cols || !vals)) return rs::set_error(ctx, RS_ERR_INVALID, "cols / vals are NULL");
        for (int64_t t = 0; t < nnz; ++t)
            if (cols[t] < 0 || cols[t] >= n_items)
                return rs::set_error(ctx, RS_ERR_INVALID, "item id out of range at " + std::to_string(t));
        rs::UserCSR csr;
        csr.rowptr.assign(rowptr, rowptr + n_users + 1);
        csr.cols.assign(cols, cols + nnz);
        csr.vals.assign(vals, vals + nnz);
        auto* pl = new rs_svd_plan();
        try {
            rs::plan_build_csr(ctx, n_users, n_items, std::move(csr), n_factors, pl);
        } catch (...) {
            delete pl;
            throw;
        }
        *out = pl;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_init_normal(rs_svd_plan* pl, double mean, double std_dev, uint64_t seed) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_init_normal(pl, mean, std_dev, seed);
        rs::reset_loss(pl, pl->ctx->stream);
        return RS_OK;
    });
}

extern "C" void rs_svd_plan_destroy(rs_svd_plan* pl) {
    if (!pl) return;
    // Destroy before closing the owning ctx (its stream may be the last one used).
    (void)hipSetDevice(pl->ctx->device);
    if (pl->last_stream) (void)hipStreamSynchronize(pl->last_stream);
    delete pl;
}

extern "C" int rs_svd_plan_set_user_weights(rs_svd_plan* pl, const float* w) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (!w) {
            pl->uw.release();
            return RS_OK;
        }
        pl->uw.alloc(std::max(1, pl->n_users));
        pl->uw.upload(w, pl->n_users, pl->ctx->stream);
        RS_HIP(hipStreamSynchronize(pl->ctx->stream));
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_epoch_delta(rs_svd_plan* pl, float lr, float reg, void* dP, void* gbsum,
                                       void* stream) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (!dP || !gbsum) return rs::set_error(pl->ctx, RS_ERR_INVALID, "delta buffers are NULL");
        if (!pl->uw.p) return rs::set_error(pl->ctx, RS_ERR_INVALID, "user weights not set");
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : pl->ctx->stream;
        RS_HIP(hipMemsetAsync(dP, 0, pl->P.n * sizeof(float), s));  // users absent from the shard
        if (pl->timing) {
            if (pl->tev.size() < 2) {
                for (int x = 0; x < 2; ++x) {
                    hipEvent_t e;
                    RS_HIP(hipEventCreate(&e));
                    pl->tev.push_back(e);
                }
            }
            pl->tev_used = 2;
            RS_HIP(hipEventRecord(pl->tev[0], s));
        }
        RS_HIP(hipEventRecord(pl->ev0, s));
        rs::launch_fast(pl, lr, reg, s, static_cast<float*>(dP));
        if (pl->write_back != RS_SGD_WB_TILE) rs::sync_item_copies(pl, s, 0);  // shard-local hot-item copies
        if (pl->timing) RS_HIP(hipEventRecord(pl->tev[1], s));
        hipLaunchKernelGGL(rs::gb_sum_kernel, dim3(1), dim3(256), 0, s, pl->partial.p,
                           static_cast<int64_t>(pl->n_blocks), static_cast<double*>(gbsum));
        RS_HIP(hipGetLastError());
        RS_HIP(hipEventRecord(pl->ev1, s));
        pl->last_launches = pl->timing ? 1 : 2;
        pl->last_stream = s;
        pl->last_ms = -1.0;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_item_weights(rs_svd_plan* pl, const float* w) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (!w) {
            pl->iw.release();
            return RS_OK;
        }
        pl->iw.alloc(std::max(1, pl->n_items));
        pl->iw.upload(w, pl->n_items, pl->ctx->stream);
        RS_HIP(hipStreamSynchronize(pl->ctx->stream));
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_epoch_qdelta(rs_svd_plan* pl, float lr, float reg, void* dQ, void* gbsum,
                                        void* stream) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (!dQ || !gbsum) return rs::set_error(pl->ctx, RS_ERR_INVALID, "delta buffers are NULL");
        if (!pl->iw.p) return rs::set_error(pl->ctx, RS_ERR_INVALID, "item weights not set");
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : pl->ctx->stream;
        const int64_t n = static_cast<int64_t>(pl->n_items) * pl->ld;
        if (pl->Q0.n != static_cast<size_t>(std::max<int64_t>(1, n))) pl->Q0.alloc(std::max<int64_t>(1, n));
        if (n) RS_HIP(hipMemcpyAsync(pl->Q0.p, pl->Q.p, n * sizeof(float), hipMemcpyDeviceToDevice, s));
        if (pl->timing) {
            if (pl->tev.size() < 2) {
                for (int x = 0; x < 2; ++x) {
                    hipEvent_t e;
                    RS_HIP(hipEventCreate(&e));
                    pl->tev.push_back(e);
                }
            }
            pl->tev_used = 2;
            RS_HIP(hipEventRecord(pl->tev[0], s));
        }
        RS_HIP(hipEventRecord(pl->ev0, s));
        rs::launch_fast(pl, lr, reg, s);  // whole user rows: P stored in place (users are exclusive)
        if (pl->timing) RS_HIP(hipEventRecord(pl->tev[1], s));
        rs::merge_split_rows(pl, s);
        if (pl->write_back != RS_SGD_WB_TILE) rs::sync_item_copies(pl, s, 0);  // copies into the item rows
        if (n)
            hipLaunchKernelGGL(rs::svd_qdelta_kernel, dim3(1024), dim3(256), 0, s, pl->Q.p, pl->Q0.p,
                               pl->iw.p, static_cast<float*>(dQ), n, pl->ld);
        hipLaunchKernelGGL(rs::gb_sum_kernel, dim3(1), dim3(256), 0, s, pl->partial.p,
                           static_cast<int64_t>(pl->n_blocks), static_cast<double*>(gbsum));
        RS_HIP(hipGetLastError());
        RS_HIP(hipEventRecord(pl->ev1, s));
        pl->last_launches = pl->timing ? 1 : 3;
        pl->last_stream = s;
        pl->last_ms = -1.0;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_apply_qdelta(rs_svd_plan* pl, const void* dQ, const void* gbsum,
                                        double inv_total_nnz, void* stream) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (!dQ || !gbsum) return rs::set_error(pl->ctx, RS_ERR_INVALID, "delta buffers are NULL");
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : pl->ctx->stream;
        const int64_t n4 = static_cast<int64_t>(pl->n_items) * pl->ld / 4;
        hipLaunchKernelGGL(rs::svd_apply_delta_kernel, dim3(1024), dim3(256), 0, s,
                           reinterpret_cast<float4*>(pl->Q.p), static_cast<const float4*>(dQ), n4,
                           pl->gb.p, static_cast<const double*>(gbsum), inv_total_nnz);
        RS_HIP(hipGetLastError());
        rs::sync_item_copies(pl, s, 1);  // copies follow the merged item rows
        pl->last_stream = s;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_apply_delta(rs_svd_plan* pl, const void* dP, const void* gbsum,
                                       double inv_total_nnz, void* stream) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (!dP || !gbsum) return rs::set_error(pl->ctx, RS_ERR_INVALID, "delta buffers are NULL");
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : pl->ctx->stream;
        const int64_t n4 = static_cast<int64_t>(pl->P.n) / 4;
        hipLaunchKernelGGL(rs::svd_apply_delta_kernel, dim3(1024), dim3(256), 0, s,
                           reinterpret_cast<float4*>(pl->P.p), static_cast<const float4*>(dP), n4,
                           pl->gb.p, static_cast<const double*>(gbsum), inv_total_nnz);
        RS_HIP(hipGetLastError());
        pl->last_stream = s;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_mode(rs_svd_plan* pl, int32_t write_back, int32_t ring_depth) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (write_back < RS_SGD_WB_TILE || write_back > RS_SGD_WB_ATOMIC)
        return rs::set_error(pl->ctx, RS_ERR_INVALID, "unknown write-back mode");
    if (ring_depth != 4 && ring_depth != 8 && ring_depth != 16)
        return rs::set_error(pl->ctx, RS_ERR_INVALID, "ring depth must be 4, 8 or 16");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);  // n_blocks (the fold's partial count) follows the mode
        const bool was_tile = pl->write_back == RS_SGD_WB_TILE;
        pl->write_back = write_back;
        pl->ring_depth = ring_depth;
        if (write_back == RS_SGD_WB_TILE) {
            if (!pl->tiles_built) rs::tile_build(pl);
            pl->n_blocks = rs::tile_partials(pl);
        } else {
            rs::ensure_hybrid(pl);
            if (was_tile) {  // the tile epochs trained the item rows only: refresh their copies
                rs::sync_item_copies(pl, pl->ctx->stream, 1);
                RS_HIP(hipStreamSynchronize(pl->ctx->stream));
            }
            pl->n_blocks = rs::fast_blocks(pl);
        }
        return RS_OK;
    });
}

// Tile schedule parameters (RS_SGD_WB_TILE), include/rsgpu.h.
extern "C" int rs_svd_plan_set_tiles(rs_svd_plan* pl, int32_t workgroups, int32_t waves, int32_t target,
                                     int32_t run_cap, int32_t ring) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (workgroups < 0 || target < 0 || run_cap < 0 || ring < 0 ||
        (waves != 1 && waves != 2 && waves != 4 && waves != 8 && waves != 16))
        return rs::set_error(pl->ctx, RS_ERR_INVALID, "bad tile parameters");
    return rs_guard(pl->ctx, [&]() -> int {
        pl->tile_wg = workgroups;
        pl->tile_waves = waves;
        pl->tile_target = target;
        pl->tile_run_cap = run_cap;
        pl->tile_ring = ring;
        rs::tile_build(pl);
        if (pl->write_back == RS_SGD_WB_TILE) pl->n_blocks = rs::tile_partials(pl);
        return RS_OK;
    });
}

// Test hook (include/rsgpu.h): the hot-run damping with a chosen concurrency, so one wave -- whose runs never
// overlap -- runs the damped kernel on R = deg x kconc and the oracle's or_svd_fit_works_damped can check it.
extern "C" int rs_svd_plan_set_damp_concurrency(rs_svd_plan* pl, float kconc) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (!(kconc >= 0.f) || !std::isfinite(kconc)) return rs::set_error(pl->ctx, RS_ERR_INVALID, "bad concurrency");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        pl->damp_kconc = kconc;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_gb_fold(rs_svd_plan* pl, int32_t mode) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (mode != RS_GB_FOLD_MEAN && mode != RS_GB_FOLD_SMOOTH) return rs::set_error(pl->ctx, RS_ERR_INVALID, "bad GlobalBias fold");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        pl->gb_fold = mode;
        return RS_OK;
    });
}

// Cold runs (include/rsgpu.h, sgd_plan.hpp kRunCold): the items whose runs end in write-through stores.  Rebuilds
// the schedule.
extern "C" int rs_svd_plan_set_cold_store(rs_svd_plan* pl, double runs_in_flight) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (!(runs_in_flight >= 0.0) || !std::isfinite(runs_in_flight))
        return rs::set_error(pl->ctx, RS_ERR_INVALID, "bad cold-run threshold");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        pl->cold_runs = runs_in_flight;
        if (pl->tiles_built) rs::tile_build(pl);
        return RS_OK;
    });
}

// Claimed runs inside a tile (include/rsgpu.h): 0 = runs dealt to the waves on the host, 4 or 8 = runs
// per claim from the tile's run queue (the default 4).  Rebuilds the schedule.
extern "C" int rs_svd_plan_set_tile_claim(rs_svd_plan* pl, int32_t runs_per_claim) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (runs_per_claim != 0 && runs_per_claim != 4 && runs_per_claim != 8)
        return rs::set_error(pl->ctx, RS_ERR_INVALID, "runs per claim must be 0, 4 or 8");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        pl->tile_claim = runs_per_claim;
        rs::tile_build(pl);
        if (pl->write_back == RS_SGD_WB_TILE) pl->n_blocks = rs::tile_partials(pl);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_tile_rule(rs_svd_plan* pl, int32_t rule) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (rule < RS_TILE_RULE_LPT || rule > RS_TILE_RULE_FILL_DEVICE)
        return rs::set_error(pl->ctx, RS_ERR_INVALID, "tile rule must be RS_TILE_RULE_LPT, _SNAKE or _SNAKE_DEVICE");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        if (rule == RS_TILE_RULE_FILL) {  // the host fill rule: whole users only
            rs::ensure_host_csr(pl);
            const int64_t rec_cap = static_cast<int64_t>((rs::kTileLdsBudget - 16 - static_cast<size_t>(rs::tile_lds_row(pl)) * 4) / 16);
            for (int32_t u = 0; u < pl->n_users; ++u)
                if (pl->h_rowptr[u + 1] - pl->h_rowptr[u] > rec_cap)
                    return rs::set_error(pl->ctx, RS_ERR_UNSUPPORTED, "fill tile rule: a user above the LDS bound");
        }
        const int32_t old = pl->tile_rule;
        pl->tile_rule = rule;
        try {
            rs::tile_build(pl);
        } catch (...) {
            pl->tile_rule = old;
            throw;
        }
        if (pl->write_back == RS_SGD_WB_TILE) pl->n_blocks = rs::tile_partials(pl);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_guard(rs_svd_plan* pl, int32_t on) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        pl->guard = on != 0;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_refits(const rs_svd_plan* pl, int32_t* n) {
    if (!pl || !n) return rs::set_error(pl ? pl->ctx : nullptr, RS_ERR_INVALID, "bad arguments");
    *n = pl->refits;
    return RS_OK;
}

extern "C" int rs_svd_plan_fixed_point(const rs_svd_plan* pl, int32_t* shift) {
    if (!pl || !shift) return rs::set_error(pl ? pl->ctx : nullptr, RS_ERR_INVALID, "bad arguments");
    *shift = pl->fx_shift;
    return RS_OK;
}

extern "C" int rs_svd_plan_tile_rule(const rs_svd_plan* pl, int32_t* rule) {
    if (!pl || !rule) return rs::set_error(pl ? pl->ctx : nullptr, RS_ERR_INVALID, "bad arguments");
    *rule = pl->tile_rule;
    return RS_OK;
}

extern "C" int rs_svd_plan_schedule_digest(rs_svd_plan* pl, uint64_t* digest) {
    if (!pl || !digest) return rs::set_error(pl ? pl->ctx : nullptr, RS_ERR_INVALID, "bad arguments");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        if (!pl->tiles_built) rs::tile_build(pl);
        uint64_t h = 1469598103934665603ULL;  // FNV-1a 64
        auto mix = [&](const void* p, size_t n) {
            const unsigned char* b = static_cast<const unsigned char*>(p);
            for (size_t x = 0; x < n; ++x) h = (h ^ b[x]) * 1099511628211ULL;
        };
        const int64_t nt = pl->n_tiles, lds = static_cast<int64_t>(pl->tile_lds);
        mix(&nt, 8);
        mix(&lds, 8);
        hipStream_t s = pl->ctx->stream;
        auto add = [&](const auto& buf, size_t count) {
            using T = std::remove_reference_t<decltype(*buf.p)>;
            std::vector<T> v(count);
            buf.download(v.data(), count, s);
            RS_HIP(hipStreamSynchronize(s));
            mix(v.data(), count * sizeof(T));
        };
        add(pl->t_tiles, static_cast<size_t>(nt));
        add(pl->t_users, static_cast<size_t>(pl->t_n_users));
        add(pl->t_streams, static_cast<size_t>(nt) * (pl->tile_waves + 1));
        add(pl->t_runs, static_cast<size_t>(pl->t_n_runs));
        add(pl->t_recs, static_cast<size_t>(pl->nnz));
        *digest = h;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_tile_clocks(rs_svd_plan* pl, int64_t* out, int64_t n) {
    if (!pl || !out || n < 0) return rs::set_error(pl ? pl->ctx : nullptr, RS_ERR_INVALID, "bad arguments");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        const size_t m = std::min(static_cast<size_t>(n), pl->trace.n);
        pl->trace.download(out, m, pl->ctx->stream);
        RS_HIP(hipStreamSynchronize(pl->ctx->stream));
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_tile_order(rs_svd_plan* pl, int64_t* pos, int64_t* work_off, int32_t* n_works) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::tile_order(pl, pos, work_off, n_works);
        return RS_OK;
    });
}

// Diagnostic timeline of the last RS_SGD_WB_ATOMIC epoch: 3 int64 per work item (LPT order) --
// start, end of its SGD chain, end of its write-back -- in 100 MHz ticks; out NULL enables it.
extern "C" int rs_svd_plan_trace(rs_svd_plan* pl, int64_t* out, int32_t* user) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        hipStream_t s = pl->ctx->stream;
        rs::plan_sync_last(pl);
        if (!out) {
            pl->trace.alloc(std::max<size_t>(3, 3 * static_cast<size_t>(pl->n_work)));
            return RS_OK;
        }
        if (!pl->trace.n) return rs::set_error(pl->ctx, RS_ERR_INVALID, "trace not enabled");
        pl->trace.download(out, 3 * static_cast<size_t>(pl->n_work), s);
        if (user) pl->wk_user.download(user, pl->n_work, s);
        RS_HIP(hipStreamSynchronize(s));
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_schedule(rs_svd_plan* pl, int32_t heavy_min, int32_t light_blocks) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (heavy_min < 0) return rs::set_error(pl->ctx, RS_ERR_INVALID, "heavy_min must be >= 0");
        pl->heavy_min = heavy_min;
        pl->light_blocks = light_blocks < 0 ? rs::default_light_blocks(pl->ctx) : light_blocks;
        if (pl->hybrid_built) rs::build_work(pl);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_fixed_q(rs_svd_plan* pl, int32_t on) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        pl->fixed_q = on ? 1 : 0;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_split(rs_svd_plan* pl, int32_t split_cap) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (split_cap < 0 || (split_cap > 0 && split_cap < 16))
            return rs::set_error(pl->ctx, RS_ERR_INVALID, "split_cap must be 0 (never) or >= 16");
        pl->split_cap = split_cap;
        if (pl->hybrid_built) rs::build_work(pl);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_hot_replicas(rs_svd_plan* pl, int32_t n_hot, int32_t copies) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (n_hot < 0 || copies < 2 || copies > rs::kMaxLiveCopies)
            return rs::set_error(pl->ctx, RS_ERR_INVALID, "n_hot must be >= 0 and copies in [2, 8]");
        pl->live_req = n_hot;
        pl->live_copies = copies;
        if (pl->hybrid_built) rs::build_items(pl);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_item_split(rs_svd_plan* pl, int32_t item_cap) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (item_cap < 0 || (item_cap > 0 && item_cap < 16))
            return rs::set_error(pl->ctx, RS_ERR_INVALID, "item_cap must be 0 (never) or >= 16");
        pl->item_cap = item_cap;
        if (pl->hybrid_built) rs::build_items(pl);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_upload(rs_svd_plan* pl, const double* P, const double* Q,
                                  const double* bu, const double* bi, const double* gb) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_upload(pl, P, Q, bu, bi, gb);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_download(rs_svd_plan* pl, double* P, double* Q, double* bu, double* bi,
                                    double* gb) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_download(pl, P, Q, bu, bi, gb);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_epochs(rs_svd_plan* pl, int32_t n_epochs, float lr, float reg,
                                  void* stream) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (n_epochs < 0) return rs::set_error(pl->ctx, RS_ERR_INVALID, "n_epochs < 0");
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : pl->ctx->stream;
        rs::plan_epochs(pl, n_epochs, lr, reg, s);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_device_ptrs(rs_svd_plan* pl, void** P, void** Q, void** gb,
                                       int32_t* ld) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (P) *P = pl->P.p;
    if (Q) *Q = pl->Q.p;
    if (gb) *gb = pl->gb.p;
    if (ld) *ld = pl->ld;
    return RS_OK;
}

extern "C" int rs_svd_plan_set_timing(rs_svd_plan* pl, int32_t on) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);  // epochs in flight keep the timing mode they were enqueued with
        pl->timing = on != 0;
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_last_kernel_ms(rs_svd_plan* pl, double* ms, int32_t* n_launches) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (pl->last_ms < 0.0) {
            RS_HIP(hipEventSynchronize(pl->ev1));
            float t = 0.f;
            if (pl->timing) {
                double sum = 0.0;
                for (int32_t x = 0; x < pl->tev_used; x += 2) {
                    RS_HIP(hipEventElapsedTime(&t, pl->tev[x], pl->tev[x + 1]));
                    sum += t;
                }
                pl->last_ms = sum;
            } else {
                RS_HIP(hipEventElapsedTime(&t, pl->ev0, pl->ev1));
                pl->last_ms = t;
            }
        }
        if (ms) *ms = pl->last_ms;
        if (n_launches) *n_launches = pl->last_launches;
        return RS_OK;
    });
}

namespace rs {
// One-shot Fit keeps its plan (CSR, tile schedule, device buffers) for the next rs_svd_fit on the same
// ctx with the same ratings -- GridSearchCV (eval.go:78-230) and repeated CrossValidate runs refit the
// same folds -- verified by comparing the whole COO (no hash: an exact match or a rebuild).
struct SvdFitCache {
    int64_t nnz = -1;
    int32_t n_users = 0, n_items = 0, k = 0, write_back = 0;
    std::vector<int32_t> users, items;
    std::vector<double> ratings;
    std::unique_ptr<rs_svd_plan> plan;
    bool matches(const rs_ratings* r, int32_t k2, int32_t wb) const {
        if (!plan || nnz != r->nnz || n_users != r->n_users || n_items != r->n_items || k != k2 || write_back != wb)
            return false;
        // exact comparison of the COO (16 B per rating), on pooled threads
        std::atomic<bool> same{true};
        parallel_ranges(nnz, 16, [&](int64_t b, int64_t e) {
            const size_t o = static_cast<size_t>(b), n = static_cast<size_t>(e - b);
            if (std::memcmp(users.data() + o, r->users + o, n * 4) != 0 ||
                std::memcmp(items.data() + o, r->items + o, n * 4) != 0 ||
                std::memcmp(ratings.data() + o, r->ratings + o, n * 8) != 0)
                same = false;
        });
        return same;
    }
};

// Sets larger than this are not cached (the cache holds a 16-byte-per-rating host copy of the COO and the
// plan's device buffers): 2^26 ratings = 1 GiB of host memory at most.
constexpr int64_t kFitCacheMaxNnz = int64_t{1} << 26;
}  // namespace rs

extern "C" int rs_fit_refits(const rs_ctx* ctx, int32_t* n) {
    if (!ctx || !n) return rs::set_error(nullptr, RS_ERR_INVALID, "bad arguments");
    *n = ctx->fit_refits;
    return RS_OK;
}

extern "C" int rs_fit_schedule_digest(rs_ctx* ctx, uint64_t* digest, int32_t* rule) {
    if (!ctx || !digest || !rule) return rs::set_error(ctx, RS_ERR_INVALID, "bad arguments");
    auto cache = std::static_pointer_cast<rs::SvdFitCache>(ctx->svd_fit_cache);
    if (!cache || !cache->plan || cache->plan->write_back != RS_SGD_WB_TILE)
        return rs::set_error(ctx, RS_ERR_INVALID, "no cached FAST tile plan (no rs_svd_fit ran on this ctx)");
    *rule = cache->plan->tile_rule;
    return rs_svd_plan_schedule_digest(cache->plan.get(), digest);
}

extern "C" int rs_svd_fit(rs_ctx* ctx, const rs_ratings* r, const rs_sgd_params* p, double* P,
                          double* Q, double* bu, double* bi, double* gb) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        int st = rs::check_sgd(ctx, r, p);
        if (st != RS_OK) return st;
        if (!P || !Q || !bu || !bi || !gb)
            return rs::set_error(ctx, RS_ERR_INVALID, "output pointer is NULL");
        const float lr = static_cast<float>(p->lr), reg = static_cast<float>(p->reg);
        if (p->mode == RS_SGD_FAST) {
            // RSGPU_FIT_TRACE=1: host phase times of this one-shot Fit on stderr (end-to-end study)
            static const bool trace = std::getenv("RSGPU_FIT_TRACE") != nullptr;
            auto now = [] { return std::chrono::steady_clock::now(); };
            auto t = now();
            auto mark = [&](const char* what) {
                if (!trace) return;
                (void)hipStreamSynchronize(ctx->stream);
                const auto t1 = now();
                std::fprintf(stderr, "fit-trace %-10s %8.3f ms\n", what,
                             std::chrono::duration<double, std::milli>(t1 - t).count());
                t = t1;
            };
            const int32_t wb = p->write_back >= RS_SGD_WB_TILE && p->write_back <= RS_SGD_WB_ATOMIC ? p->write_back : RS_SGD_WB_TILE;
            auto cache = std::static_pointer_cast<rs::SvdFitCache>(ctx->svd_fit_cache);
            const bool hit = cache && cache->matches(r, p->n_factors, wb);
            mark(hit ? "cache-hit" : "cache-miss");
            bool prepared = false;  // warm start done and factors packed during the device build
            if (!hit) {
                const bool dev = wb == RS_SGD_WB_TILE && r->nnz > 0 && r->nnz <= rs::kDeviceBuildMaxNnz;
                auto old = dev ? cache : nullptr;  // the device path recycles the old plan's buffers
                ctx->svd_fit_cache.reset();          // (otherwise they are freed first)
                cache = std::make_shared<rs::SvdFitCache>();
                cache->plan = std::make_unique<rs_svd_plan>();
                cache->plan->write_back = wb;
                if (dev) {
                    if (old && old->plan) rs::plan_recycle(cache->plan.get(), old->plan.get(), r->n_users, r->n_items, p->n_factors);
                    if (old) {  // and the host COO copy's memory
                        cache->users = std::move(old->users);
                        cache->items = std::move(old->items);
                        cache->ratings = std::move(old->ratings);
                    }
                    old.reset();
                    rs_svd_plan* np = cache->plan.get();
                    np->build_overlap = [&, np] {  // under the device build's kernels
                        if (p->n_epochs > 0) *gb = rs::gb_warm_start(r, bu, bi);
                        prepared = rs::plan_pack_fit(np, P, Q, bu, bi);
                    };
                    rs::plan_build_coo_device(ctx, r, p->n_factors, np);
                    np->build_overlap = nullptr;
                } else {
                    rs::UserCSR csr;
                    rs::build_csr(r->nnz, r->n_users, r->users, r->items, r->ratings, csr);
                    mark("csr");
                    rs::plan_build_csr(ctx, r->n_users, r->n_items, std::move(csr), p->n_factors, cache->plan.get());
                }
                mark("plan");
            }
            // the cache's copy of the COO (compared by the next call) is made while the first epochs run
            auto keep_coo = [&] {
                if (hit || r->nnz > rs::kFitCacheMaxNnz) return;
                const size_t n = static_cast<size_t>(r->nnz);
                cache->nnz = r->nnz;
                cache->n_users = r->n_users;
                cache->n_items = r->n_items;
                cache->k = p->n_factors;
                cache->write_back = wb;
                cache->users.resize(n);
                cache->items.resize(n);
                cache->ratings.resize(n);
                rs::parallel_ranges(r->nnz, 16, [&](int64_t b, int64_t e) {  // the COO copy, pooled threads
                    const size_t o = static_cast<size_t>(b), m = static_cast<size_t>(e - b);
                    std::memcpy(cache->users.data() + o, r->users + o, m * 4);
                    std::memcpy(cache->items.data() + o, r->items + o, m * 4);
                    std::memcpy(cache->ratings.data() + o, r->ratings + o, m * 8);
                });
                ctx->svd_fit_cache = cache;
            };
            rs_svd_plan& pl = *cache->plan;
            // Divergence guard: plan_epochs redoes a call that left the fixed-point range or went non-finite on
            // a quarter of the workgroups (up to three times; the plan keeps the smaller grid), so a Go Fit that panics on
            // an error never gets a NaN model first; RS_ERR_NUMERIC only when every attempt failed.
            const int32_t refits0 = pl.refits;
            if (prepared) {
                rs::plan_dma_fit(&pl, gb);
            } else {
                if (p->n_epochs > 0) *gb = rs::gb_warm_start(r, bu, bi);
                mark("warm");
                if (!rs::plan_upload_fit(&pl, P, Q, bu, bi, gb)) rs::plan_upload(&pl, P, Q, bu, bi, gb);
            }
            mark("upload");
            // the results' download is enqueued behind the epochs (and the guard's check), so one wait covers both
            const bool staged = rs::fit_fits_staging(&pl);
            int32_t flag = 0;
            auto fetch = [&] {
                rs::kernel_span_record(ctx);  // the kernel span ends before the copies
                if (staged) rs::plan_fetch_enqueue(&pl);
            };
            rs::kernel_span_begin(ctx);
            rs::plan_epochs(&pl, p->n_epochs, lr, reg, ctx->stream, trace ? std::function<void()>() : std::function<void()>(keep_coo),
                            fetch);
            rs::kernel_span_wait(ctx);
            ctx->fit_refits = pl.refits - refits0;
            mark("epochs");
            if (trace) {
                keep_coo();
                mark("cache-copy");
            }
            if (staged) {
                RS_HIP(hipStreamSynchronize(ctx->stream));
                rs::plan_fetch_result(ctx, gb, &flag);
                rs::plan_finish_fit(&pl, P, Q, bu, bi, flag);
            } else {
                rs::plan_download(&pl, P, Q, bu, bi, gb);
            }
            mark("download");
            return RS_OK;
        }
        // ORDERED: COO in train-set order, conflict-free batches on one workgroup, all epochs in one launch (sgd_ordered.hip), rows in the
        // folded layout P [p, b_u, 1], Q [q, 1, b_i]
        rs::drop_fit_cache(ctx);
        hipStream_t s = ctx->stream;
        const int32_t k = p->n_factors, ld = rs::round_up4(k + 2);
        const int64_t nnz = r->nnz;
        const int64_t npad = rs::ordered_padded(nnz);  // whole blocks for the kernel's scalar id loads
        rs::DevBuf<int32_t> du(npad), di(npad);
        rs::DevBuf<float> dr(npad);
        std::vector<float> rf(static_cast<size_t>(npad), 0.f);
        for (int64_t t = 0; t < nnz; ++t) rf[t] = static_cast<float>(r->ratings[t]);
        RS_HIP(hipMemsetAsync(du.p, 0, npad * sizeof(int32_t), s));
        RS_HIP(hipMemsetAsync(di.p, 0, npad * sizeof(int32_t), s));
        du.upload(r->users, nnz, s);
        di.upload(r->items, nnz, s);
        dr.upload(rf.data(), npad, s);
        const int64_t pn = static_cast<int64_t>(std::max(1, r->n_users)) * ld, qn = static_cast<int64_t>(std::max(1, r->n_items)) * ld;
        rs::DevBuf<float> dP(pn), dQ(qn);
        rs::DevBuf<double> dgb(1);
        std::vector<float> hP(static_cast<size_t>(pn), 0.f), hQ(static_cast<size_t>(qn), 0.f);
        for (int32_t x = 0; x < r->n_users; ++x) {
            float* row = hP.data() + static_cast<int64_t>(x) * ld;
            for (int32_t f = 0; f < k; ++f) row[f] = static_cast<float>(P[static_cast<int64_t>(x) * k + f]);
            row[k] = static_cast<float>(bu[x]);
            row[k + 1] = 1.f;
        }
        for (int32_t x = 0; x < r->n_items; ++x) {
            float* row = hQ.data() + static_cast<int64_t>(x) * ld;
            for (int32_t f = 0; f < k; ++f) row[f] = static_cast<float>(Q[static_cast<int64_t>(x) * k + f]);
            row[k] = 1.f;
            row[k + 1] = static_cast<float>(bi[x]);
        }
        dP.upload(hP.data(), hP.size(), s);
        dQ.upload(hQ.data(), hQ.size(), s);
        dgb.upload(gb, 1, s);
        const rs::OrderedSchedule os = rs::ordered_batches(r->users, r->items, nnz, r->n_users, r->n_items,
                                                           rs::ordered_wmax(ld));
        const int64_t nbs = static_cast<int64_t>(os.start.size());
        rs::DevBuf<int64_t> dbs(nbs);
        rs::DevBuf<int32_t> dfw(npad);
        dbs.upload(os.start.data(), nbs, s);
        RS_HIP(hipMemsetAsync(dfw.p, 0, npad * sizeof(int32_t), s));
        dfw.upload(os.fwd.data(), nnz, s);
        rs::kernel_span_begin(ctx);
        if (nnz > 0 && p->n_epochs > 0)
            rs::ordered_epochs(du.p, di.p, dr.p, dfw.p, nnz, dbs.p, nbs - 1, dP.p, pn, dQ.p, qn, ld, k, dgb.p,
                               p->n_epochs, lr, reg, s);
        rs::kernel_span_end(ctx);
        dP.download(hP.data(), hP.size(), s);
        dQ.download(hQ.data(), hQ.size(), s);
        dgb.download(gb, 1, s);
        RS_HIP(hipStreamSynchronize(s));
        for (int32_t x = 0; x < r->n_users; ++x) {
            const float* row = hP.data() + static_cast<int64_t>(x) * ld;
            for (int32_t f = 0; f < k; ++f) P[static_cast<int64_t>(x) * k + f] = row[f];
            bu[x] = row[k];
        }
        for (int32_t x = 0; x < r->n_items; ++x) {
            const float* row = hQ.data() + static_cast<int64_t>(x) * ld;
            for (int32_t f = 0; f < k; ++f) Q[static_cast<int64_t>(x) * k + f] = row[f];
            bi[x] = row[k + 1];
        }
        return RS_OK;
    });
}

namespace rs {
// Upload the pairs, run svd_predict_kernel on the plan's factors; out and/or (rmse, mae).
static void plan_predict(rs_svd_plan* pl, int64_t n, const int32_t* users, const int32_t* items,
                         const double* ratings, double* out, double* rmse, double* mae) {
    plan_sync_last(pl);
    hipStream_t s = pl->ctx->stream;
    if (n == 0) {
        if (rmse) *rmse = std::nan("");  // utils.go:169: sqrt(0 / 0)
        if (mae) *mae = std::nan("");
        return;
    }
    DevBuf<int32_t> du(n), di(n);
    DevBuf<double> dr(ratings ? n : 0), dout(out ? n : 0);
    du.upload(users, n, s);
    di.upload(items, n, s);
    if (ratings) dr.upload(ratings, n, s);
    const int64_t blocks = (n + 15) / 16;
    DevBuf<double> part(ratings ? 2 * blocks : 0), sums(ratings ? 2 : 0);
    hipLaunchKernelGGL(svd_predict_kernel, dim3(blocks), dim3(256), 0, s, pl->P.p, pl->Q.p, pl->ld, pl->k,
                       pl->n_users, pl->n_items, pl->gb.p, n, du.p, di.p, dr.p, dout.p, part.p);
    RS_HIP(hipGetLastError());
    if (ratings) {
        hipLaunchKernelGGL(pair_sum_kernel, dim3(1), dim3(256), 0, s, part.p, blocks, sums.p);
        RS_HIP(hipGetLastError());
        double h[2];
        sums.download(h, 2, s);
        RS_HIP(hipStreamSynchronize(s));
        if (rmse) *rmse = std::sqrt(h[0] / static_cast<double>(n));
        if (mae) *mae = h[1] / static_cast<double>(n);
    }
    if (out) dout.download(out, n, s);
    RS_HIP(hipStreamSynchronize(s));
}
}  // namespace rs

extern "C" int rs_svd_plan_predict(rs_svd_plan* pl, int64_t n, const int32_t* users,
                                   const int32_t* items, double* out) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (n < 0 || (n > 0 && (!users || !items || !out)))
            return rs::set_error(pl->ctx, RS_ERR_INVALID, "bad predict arguments");
        rs::plan_predict(pl, n, users, items, nullptr, out, nullptr, nullptr);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_evaluate(rs_svd_plan* pl, int64_t n, const int32_t* users,
                                    const int32_t* items, const double* ratings, double* rmse,
                                    double* mae) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (n < 0 || (n > 0 && (!users || !items || !ratings)) || (!rmse && !mae))
            return rs::set_error(pl->ctx, RS_ERR_INVALID, "bad evaluate arguments");
        rs::plan_predict(pl, n, users, items, ratings, nullptr, rmse, mae);
        return RS_OK;
    });
}

extern "C" int rs_svd_predict(rs_ctx* ctx, int64_t n, const int32_t* users, const int32_t* items,
                              int32_t n_users, int32_t n_items, int32_t n_factors, const double* P,
                              const double* Q, const double* bu, const double* bi, double gb,
                              double* out) {
    // Host restatement of svd.go:32-51 (the reference's Predict stays on the host);
    // kept in the C-ABI so a cgo host can batch its test-set predictions in one call.
    return rs_guard(nullptr, [&]() -> int {
        if (n < 0 || (n > 0 && (!users || !items || !out)))
            return rs::set_error(ctx, RS_ERR_INVALID, "bad predict arguments");
        for (int64_t t = 0; t < n; ++t) {
            const int32_t u = users[t], i = items[t];
            const bool ku = u >= 0 && u < n_users, ki = i >= 0 && i < n_items;
            double ret = gb;
            if (ku) ret += bu[u];
            if (ki) ret += bi[i];
            if (ku && ki) {
                double s = 0.0;
                const double* pu = P + static_cast<int64_t>(u) * n_factors;
                const double* qi = Q + static_cast<int64_t>(i) * n_factors;
                for (int32_t f = 0; f < n_factors; ++f) s += pu[f] * qi[f];
                ret += s;
            }
            out[t] = ret;
        }
        return RS_OK;
    });
}
