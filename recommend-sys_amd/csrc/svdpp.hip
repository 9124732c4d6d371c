// svdpp.hip -- K2: SVD++ epoch (reference core/svd.go:259-427), gfx950.
//
// ORDERED  one workgroup walks the ratings in train-set order with the literal per-rating work of
//          the reference: e = (sum_{j in N(u)} y_j) / sqrt|N(u)| recomputed for every rating
//          (svd.go:271-282, called from 363), then b, p_u, q_i and every y_j of N(u) updated
//          (svd.go:366-422).  Thread f owns factor column f of every row, so the only cross-thread
//          step per rating is the prediction's dot product.  Parity target (SVD++ is unpinned by
//          the reference: core/base_test.go:38-40 is commented out) = the fp64 restatement.
// FAST     user-CSR, one wave per user, heaviest first.  Within a user row the y-update is the same
//          affine map for every j in N(u) (y <- a y - (lr diff / sqrt n) q_new, a = 1 - lr reg), so
//          the wave keeps S0 = sum y_j, the scale A and the offset vector C in registers,
//              e = (A S0 - n C) / sqrt n,
//          and applies y_j += (A - 1) y_j - C once per (u, j) at the end of the row (SURVEY §8a
//          A8: equal to the literal update in user-major order).  q_i and y_j deltas go to the
//          memory side as float atomics (cross-XCD coherent, no lost updates), like K1.
//
// FAST device layout: P, Q, Y are (rows x ld) float32, ld = 64 ceil((k + 1) / 64); the bias (b_u in
// P, b_i in Q) sits in column k, right after the factors (lane 63 of the last register), Y's column k
// stays 0.  Padding lanes of the last register (columns > k) are never loaded or written, and Y rows
// skip lane 63 as well, so whole 64-B lines past the row get no request: the memory-side atomic unit
// prices a row update per line (K1, scripts/experiments/exp_atomics2.hip).  k = 128: Q rows 9 lines of 12, Y 8.
// Algorithmic bytes per epoch: nnz*(16 + 8k) + U*(16 + 8k) + nnz*(4 + 12k).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "sgd_plan.hpp"
#include "wave.hpp"

namespace rs {

constexpr int32_t kPPOut = 0x7FFFFFF0;
constexpr int kPPAux = 16;  // sc1

__device__ __forceinline__ float pp_wave_sum(float x) {
    x = group_sum<16>(x);
    auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
    auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

// column of this lane's last register (E - 1), or -1: lane 63 holds the bias (column kf) in P and Q
// rows; Y rows have no bias, so there lane 63 is padding too
template <int E>
__device__ __forceinline__ int32_t pp_last_col(int lane, int32_t kf, bool bias) {
    if (lane == 63) return bias ? kf : -1;
    const int32_t c = lane + 64 * (E - 1);
    return c < kf ? c : -1;
}
template <int E>
__device__ __forceinline__ int32_t pp_roff(int32_t row, int x, int32_t lane4, int32_t lc) {
    return x < E - 1 ? row + lane4 + 256 * x : (lc >= 0 ? row + 4 * lc : kPPOut);
}

// Fixed-point Q and Y (FX, the default; RSGPU_PP_FX=0 keeps fp32): the FAST fit packs Q and Y as
// int32 round(v * 2^S) on the host and unpacks them after the last epoch; loads convert to fp32 and
// the q_i / y_j deltas become integer atomics (memory-side u32 adds at 1.69 TB/s against 1.32 for
// f32, K1).  S follows the ratings (fx_shift_for, sgd_plan.hpp): 24 on star scales (resolution 2^-24,
// the fp32 ulp at |v| in [0.5, 1), |v| < 128), fewer where the biases reach further (|v| < 2^(31-S)).
__device__ __forceinline__ float pp_ld(uint32_t bits, bool fx, float fx_inv) {
    return fx ? static_cast<float>(static_cast<int32_t>(bits)) * fx_inv : __uint_as_float(bits);
}
template <bool FX>
__device__ __forceinline__ void pp_atomic_add(float d, __amdgpu_buffer_rsrc_t r, int32_t off, float fx) {
    if constexpr (FX)
        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(__float2int_rn(d * fx), r, off, 0, 0);
    else
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(d, r, off, 0, 0);
}

__device__ __forceinline__ float pp_lane63(float x) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

// ---------------------------------------------------------------------------------------------
// FAST (lazy y) epoch kernel

// Pass 1 of one user over the y rows j = b + first, b + first + step, ... (batches of YB rows):
// the sum of the y_j (svd.go:276-278) in that order.
template <int E, int YB, bool FX>
__device__ __forceinline__ void pp_sum_y(__amdgpu_buffer_rsrc_t ry, const int32_t* __restrict__ items,
                                         int64_t b, int64_t e, int32_t first, int32_t step, int32_t lane4,
                                         int32_t lcy, float (&S0)[E], float fx) {
    constexpr int LD = 64 * E;
#pragma unroll
    for (int x = 0; x < E; ++x) S0[x] = 0.f;
    for (int64_t base = b + first; base < e; base += step) {
        const int32_t rem = static_cast<int32_t>(e - base);
        float yv[YB][E];
#pragma unroll
        for (int j = 0; j < YB; ++j) {
            const int32_t row = j < rem ? items[base + j] * (LD * 4) : kPPOut;
#pragma unroll
            for (int x = 0; x < E; ++x)
                yv[j][x] = pp_ld(__builtin_amdgcn_raw_buffer_load_b32(ry, pp_roff<E>(row, x, lane4, lcy), 0, kPPAux), FX, 1.f / fx);
        }
#pragma unroll
        for (int j = 0; j < YB; ++j)
#pragma unroll
            for (int x = 0; x < E; ++x) S0[x] += yv[j][x];
    }
}

// Pass 3 over the same row subset: y_j += (A - 1) y_j - C (the deferred svd.go:399-422), atomics.
template <int E, int YB, bool FX>
__device__ __forceinline__ void pp_update_y(__amdgpu_buffer_rsrc_t ry, const int32_t* __restrict__ items,
                                            int64_t b, int64_t e, int32_t first, int32_t step,
                                            int32_t lane4, int32_t lcy, float am1, const float (&Cv)[E], float fx) {
    constexpr int LD = 64 * E;
    for (int64_t base = b + first; base < e; base += step) {
        const int32_t rem = static_cast<int32_t>(e - base);
        float yv[YB][E];
        int32_t rows[YB];
#pragma unroll
        for (int j = 0; j < YB; ++j) {
            rows[j] = j < rem ? items[base + j] * (LD * 4) : kPPOut;
#pragma unroll
            for (int x = 0; x < E; ++x)
                yv[j][x] = pp_ld(__builtin_amdgcn_raw_buffer_load_b32(ry, pp_roff<E>(rows[j], x, lane4, lcy), 0, kPPAux), FX, 1.f / fx);
        }
#pragma unroll
        for (int j = 0; j < YB; ++j)
#pragma unroll
            for (int x = 0; x < E; ++x)
                pp_atomic_add<FX>(__builtin_fmaf(am1, yv[j][x], -Cv[x]), ry, pp_roff<E>(rows[j], x, lane4, lcy), fx);
    }
}

// Pass 2 of one user: the ratings in data order with the lazy y state (S0, A, Cv).  Every q_i update
// is handed to emit(row byte offset, q_new, q_old).  Returns with p (bias in lane 63), ub, gb, A, Cv
// advanced.
template <int E, int D, bool FX, class Emit>
__device__ __forceinline__ void pp_chain(__amdgpu_buffer_rsrc_t rq, const int32_t* __restrict__ items,
                                         const float* __restrict__ ratings, int64_t b, int64_t e,
                                         int32_t lane, int32_t lcq, float lr, float a, const float (&S0)[E], float (&p)[E],
                                         float& ub, float& gb, float& A, float (&Cv)[E], float fx, Emit&& emit) {
#pragma clang fp contract(fast)
    constexpr int LD = 64 * E, B = 16;
    static_assert(B % D == 0, "ring depth must divide the 16-rating batch");
    const int32_t lane4 = lane * 4;
    const bool bias_lane = lane == 63;
    const int32_t deg = static_cast<int32_t>(e - b);
    const float nf = static_cast<float>(deg);
    const float rsq = 1.f / sqrtf(nf);  // the chain multiplies by 1/sqrt|N(u)| (no divide per rating)
    const float fx_inv = 1.f / fx;
    auto load_rowq = [&](float (&q)[E], int32_t valid, int32_t item) {
        const int32_t row = valid ? item * (LD * 4) : kPPOut;
#pragma unroll
        for (int x = 0; x < E; ++x)
            q[x] = pp_ld(__builtin_amdgcn_raw_buffer_load_b32(rq, pp_roff<E>(row, x, lane4, lcq), 0, kPPAux), FX, fx_inv);
    };
    int32_t it_cur[B], it_nxt[B];
#pragma unroll
    for (int j = 0; j < B; ++j) it_cur[j] = items[b + j];
#pragma unroll
    for (int j = 0; j < B; ++j) it_nxt[j] = items[b + B + j];
    float ring[D][E];
#pragma unroll
    for (int s = 0; s < D; ++s) load_rowq(ring[s], s < deg, it_cur[s]);
    for (int64_t base = b; base < e; base += B) {
        const int32_t rem = static_cast<int32_t>(e - base);
        float rt[B];
#pragma unroll
        for (int j = 0; j < B; ++j) rt[j] = ratings[base + j];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            constexpr int kD = D;
            const int slot = j % kD;
            if (j < rem) {
                float (&q)[E] = ring[slot];
                const float bq = pp_lane63(q[E - 1]);
                float ev[E];
                float s = 0.f;
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    ev[x] = (A * S0[x] - nf * Cv[x]) * rsq;           // svd.go:271-282
                    const float qx = (x == E - 1 && bias_lane) ? 0.f : q[x];
                    s += (p[x] + ev[x]) * qx;                         // svd.go:302-305
                }
                s = pp_wave_sum(s);
                const float diff = ((gb + ub) + bq) + s - rt[j];      // svd.go:363-364
                const float c = lr * diff;
                gb -= c;                                              // svd.go:366-367
                ub = __builtin_fmaf(ub, a, -c);                       // svd.go:370-371
                const float bq_new = __builtin_fmaf(bq, a, -c);       // svd.go:374-375
                const float cy = c * rsq;                             // svd.go:410-412
                A *= a;                                               // svd.go:413-417 (lazy)
                float qw[E];
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    const float pn = __builtin_fmaf(-c, q[x], p[x] * a);           // 378-384
                    const float qn = __builtin_fmaf(-c, pn + ev[x], q[x] * a);     // 387-396
                    const bool bx = x == E - 1 && bias_lane;
                    p[x] = bx ? ub : pn;
                    qw[x] = bx ? bq_new : qn;
                    Cv[x] = bx ? 0.f : __builtin_fmaf(cy, qn, Cv[x] * a);
                }
                emit(it_cur[j] * (LD * 4), qw, q);
            }
            const int jn = j + D;
            load_rowq(ring[slot], jn < rem, jn < B ? it_cur[jn % B] : it_nxt[jn % B]);
        }
#pragma unroll
        for (int j = 0; j < B; ++j) it_cur[j] = it_nxt[j];
#pragma unroll
        for (int j = 0; j < B; ++j) it_nxt[j] = items[base + 2 * B + j];
    }
}

// FAST epoch.  Blocks [0, n_hblocks) stride over the heavy users (the first n_heavy work items, LPT
// order), one user at a time per block: pass 1 and pass 3 split over the block's four waves (rows
// j = 4 t YB + w YB ...), pass 2 on wave 0 with its q_i deltas written to an LDS ring that waves 1..3
// drain into the atomics (the K1 hybrid scheme: the chain's vmcnt then holds only its own loads, not
// the atomics' memory-side latency).  The other blocks' waves stride over the light users, each wave
// running all three passes itself with direct atomics.
template <int E>
struct PPRing {
    static constexpr int kRing = E <= 2 ? 32 : (E <= 4 ? 16 : 8);
    static constexpr int kBatch = E <= 2 ? 8 : (E <= 4 ? 4 : 2);
};

__device__ __forceinline__ int32_t pp_lds_load(const int32_t* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void pp_lds_store(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int E, int D, bool FX>
__global__ __launch_bounds__(256) void svdpp_epoch_fast_kernel(
    const int32_t* __restrict__ work, int32_t n_work, int32_t n_heavy, int32_t n_hblocks,
    const int64_t* __restrict__ rowptr,
    const int32_t* __restrict__ items, const float* __restrict__ ratings, float* __restrict__ P,
    float* Q, float* Y, int32_t row_bytes_q, int32_t row_bytes_y, const double* __restrict__ gb_in,
    double* __restrict__ gb_partial, float lr, float reg, int32_t kf, float fx) {
#pragma clang fp contract(fast)
    constexpr int LD = 64 * E;
    constexpr int YB = 8;  // y rows per pass-1/3 batch (24 was measured to break the FAST RMSE on ML-100K)
    constexpr int R = PPRing<E>::kRing, NB = PPRing<E>::kBatch, NW = 3;
    constexpr int DH = E <= 3 ? 16 : 8;  // heavy producer: its vmcnt holds only q loads
    __shared__ double s_contrib[4];
    __shared__ float s_red[4][LD];
    __shared__ float s_q[R][LD];
    __shared__ int32_t s_row[R];
    __shared__ int32_t s_tail, s_done, s_head[NW];
    __shared__ float s_A;
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const float gb0 = static_cast<float>(gb_in[0]);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, row_bytes_q, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(Y, 0, row_bytes_y, 0x00020000);
    const int32_t lane4 = lane * 4;
    const int32_t lcq = pp_last_col<E>(lane, kf, true), lcy = pp_last_col<E>(lane, kf, false);
    auto pcol = [&](int x) { return x < E - 1 ? lane + 64 * x : lcq; };  // P row column, or -1
    const float a = 1.f - lr * reg;
    const int blk = static_cast<int>(blockIdx.x);
    double contrib = 0.0;

    if (blk >= n_hblocks) {  // light blocks
        const int stride = (static_cast<int>(gridDim.x) - n_hblocks) * 4;
        for (int w = n_heavy + (blk - n_hblocks) * 4 + wib; w < n_work; w += stride) {
            const int32_t u = work[w];
            const int64_t b = rowptr[u], e = rowptr[u + 1];
            float p[E];
            float* prow = P + static_cast<int64_t>(u) * LD;
#pragma unroll
            for (int x = 0; x < E; ++x) p[x] = pcol(x) >= 0 ? prow[pcol(x)] : 0.f;
            float ub = pp_lane63(p[E - 1]);
            float gb = gb0, A = 1.f;
            float S0[E], Cv[E];
            pp_sum_y<E, YB, FX>(ry, items, b, e, 0, YB, lane4, lcy, S0, fx);
#pragma unroll
            for (int x = 0; x < E; ++x) Cv[x] = 0.f;
            pp_chain<E, D, FX>(rq, items, ratings, b, e, lane, lcq, lr, a, S0, p, ub, gb, A, Cv, fx,
                               [&](int32_t row, const float (&qw)[E], const float (&q)[E]) {
#pragma unroll
                                   for (int x = 0; x < E; ++x)
                                       pp_atomic_add<FX>(qw[x] - q[x], rq, pp_roff<E>(row, x, lane4, lcq), fx);
                               });
            pp_update_y<E, YB, FX>(ry, items, b, e, 0, YB, lane4, lcy, A - 1.f, Cv, fx);
#pragma unroll
            for (int x = 0; x < E; ++x)
                if (pcol(x) >= 0) prow[pcol(x)] = p[x];
            contrib += static_cast<double>(e - b) * (static_cast<double>(gb) - static_cast<double>(gb0));
        }
        if (lane == 0) s_contrib[wib] = contrib;
        __syncthreads();
        if (threadIdx.x == 0)
            gb_partial[blk] = ((s_contrib[0] + s_contrib[1]) + s_contrib[2]) + s_contrib[3];
        return;
    }

    // heavy block (block-uniform branch): users work[blk], work[blk + n_hblocks], ...
    for (int32_t hw = blk; hw < n_heavy; hw += n_hblocks) {
        const int32_t u = work[hw];
        const int64_t b = rowptr[u], e = rowptr[u + 1];
        if (threadIdx.x == 0) {
            s_tail = 0;
            s_done = 0;
        }
        if (threadIdx.x < NW) s_head[threadIdx.x] = static_cast<int32_t>(threadIdx.x);
        // pass 1 split over the four waves, the partial sums added in wave order (identical everywhere)
        {
            float S0w[E];
            pp_sum_y<E, YB, FX>(ry, items, b, e, wib * YB, 4 * YB, lane4, lcy, S0w, fx);
#pragma unroll
            for (int x = 0; x < E; ++x) s_red[wib][lane + 64 * x] = S0w[x];
        }
        __syncthreads();
        float Cv[E];
#pragma unroll
        for (int x = 0; x < E; ++x) Cv[x] = 0.f;
        if (wib == 0) {
            float S0[E], p[E];
#pragma unroll
            for (int x = 0; x < E; ++x)
                S0[x] = ((s_red[0][lane + 64 * x] + s_red[1][lane + 64 * x]) + s_red[2][lane + 64 * x]) +
                        s_red[3][lane + 64 * x];
            float* prow = P + static_cast<int64_t>(u) * LD;
#pragma unroll
            for (int x = 0; x < E; ++x) p[x] = pcol(x) >= 0 ? prow[pcol(x)] : 0.f;
            float ub = pp_lane63(p[E - 1]);
            float gb = gb0, A = 1.f;
            int32_t tail = 0, free_end = R;
            pp_chain<E, DH, FX>(rq, items, ratings, b, e, lane, lcq, lr, a, S0, p, ub, gb, A, Cv, fx,
                            [&](int32_t row, const float (&qw)[E], const float (&q)[E]) {
                                if (tail >= free_end) {  // ring full: wait for the writers
                                    for (;;) {
                                        const int32_t h = min(min(pp_lds_load(&s_head[0]), pp_lds_load(&s_head[1])),
                                                              pp_lds_load(&s_head[2]));
                                        free_end = h + R;
                                        if (tail < free_end) break;
                                        __builtin_amdgcn_s_sleep(1);
                                    }
                                }
                                const int slot = tail & (R - 1);
#pragma unroll
                                for (int x = 0; x < E; ++x) s_q[slot][lane + 64 * x] = qw[x] - q[x];
                                if (lane == 0) s_row[slot] = row;
                                __atomic_signal_fence(__ATOMIC_SEQ_CST);  // entry before tail, in issue order
                                ++tail;
                                if (lane == 0) pp_lds_store(&s_tail, tail);
                            });
#pragma unroll
            for (int x = 0; x < E; ++x) {
                if (pcol(x) >= 0) prow[pcol(x)] = p[x];
                s_red[0][lane + 64 * x] = Cv[x];  // pass 3 reads C and A from LDS
            }
            if (lane == 0) s_A = A;
            contrib += static_cast<double>(e - b) * (static_cast<double>(gb) - static_cast<double>(gb0));
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            if (lane == 0) pp_lds_store(&s_done, 1);
        } else {
            const int wr = wib - 1;
            int32_t next = wr;
            for (;;) {
                const int32_t done = pp_lds_load(&s_done);
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                const int32_t tail = pp_lds_load(&s_tail);
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                if (next < tail) {
                    while (next < tail) {
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
                                for (int x = 0; x < E; ++x)
                                    pp_atomic_add<FX>(v[j][x], rq, pp_roff<E>(row, x, lane4, lcq), fx);
                            }
                        }
                        next += NW * n;
                    }
                    __atomic_signal_fence(__ATOMIC_SEQ_CST);
                    if (lane == 0) pp_lds_store(&s_head[wr], next);
                } else if (done) {
                    break;
                } else {
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        }
        __syncthreads();  // A and C in LDS; every q delta issued
        {
            float C[E];
#pragma unroll
            for (int x = 0; x < E; ++x) C[x] = s_red[0][lane + 64 * x];
            pp_update_y<E, YB, FX>(ry, items, b, e, wib * YB, 4 * YB, lane4, lcy, s_A - 1.f, C, fx);
        }
        __syncthreads();  // s_red, s_A and the ring are reset by the next user
    }
    if (threadIdx.x == 0) gb_partial[blk] = contrib;
}

__global__ __launch_bounds__(256) void pp_gb_fold_kernel(const double* __restrict__ partial,
                                                         int64_t n, double* __restrict__ gb,
                                                         double inv_nnz) {
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

// ---------------------------------------------------------------------------------------------
// ORDERED (literal) kernel: one workgroup of NT threads, thread f = factor column f (k <= NT).

template <int NT>
__global__ __launch_bounds__(NT) void svdpp_ordered_kernel(
    int64_t nnz, const int32_t* __restrict__ users, const int32_t* __restrict__ items,
    const float* __restrict__ ratings, const int64_t* __restrict__ nrow,
    const int32_t* __restrict__ ncol, float* P, float* Q, float* Y, float* bu, float* bi,
    int32_t k, double* gb_io, int32_t epochs, float lr, float reg) {
#pragma clang fp contract(off)
    __shared__ float red[NT / 64];
    const int f = threadIdx.x;
    const bool act = f < k;
    const double lrd = lr, regd = reg;
    double gb = gb_io[0];
    for (int32_t epoch = 0; epoch < epochs; ++epoch) {       // svd.go:350
        for (int64_t n = 0; n < nnz; ++n) {                   // svd.go:352
            const int32_t u = users[n], i = items[n];
            const float r = ratings[n];
            const int64_t jb = nrow[u], je = nrow[u + 1];
            const float ub = bu[u], ib = bi[i];               // svd.go:358-359
            float p = act ? P[static_cast<int64_t>(u) * k + f] : 0.f;
            float q = act ? Q[static_cast<int64_t>(i) * k + f] : 0.f;
            // svd.go:271-282 ensembleImplFactors (column f, N(u) order)
            float e = 0.f;
            if (act)
                for (int64_t x = jb; x < je; ++x) e = e + Y[static_cast<int64_t>(ncol[x]) * k + f];
            const float sq = static_cast<float>(sqrt(static_cast<double>(je - jb)));
            e = e / sq;
            float tmp = 0.f;                                   // svd.go:302-305
            tmp = tmp + p;
            tmp = tmp + e;
            float s = tmp * q;
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            if ((f & 63) == 0) red[f >> 6] = s;
            __syncthreads();
            float dot = 0.f;
            for (int x = 0; x < NT / 64; ++x) dot += red[x];
            __syncthreads();
            double pred = gb;                                  // svd.go:290-305
            pred += static_cast<double>(ub);
            pred += static_cast<double>(ib);
            pred += static_cast<double>(dot);
            const double diff = pred - static_cast<double>(r);
            gb -= lrd * diff;                                  // svd.go:366-367
            const float ub_new = static_cast<float>(ub - lrd * (diff + regd * ub));
            const float ib_new = static_cast<float>(ib - lrd * (diff + regd * ib));
            const float df = static_cast<float>(diff);
            float av = (q * df + p * reg) * lr;                // svd.go:378-384 (old q)
            p = p - av;
            av = p;                                            // svd.go:387-396 (new p + e)
            av = av + e;
            av = av * df;
            av = (av + q * reg) * lr;
            q = q - av;
            if (act) {
                P[static_cast<int64_t>(u) * k + f] = p;
                Q[static_cast<int64_t>(i) * k + f] = q;
                for (int64_t x = jb; x < je; ++x) {            // svd.go:399-422
                    float* y = Y + static_cast<int64_t>(ncol[x]) * k + f;
                    float a2 = q * df;
                    a2 = a2 / sq;
                    a2 = (a2 + *y * reg) * lr;
                    *y = *y - a2;
                }
            }
            bu[u] = ub_new;  // every thread stores the same bits and re-reads its own write
            bi[i] = ib_new;
        }
    }
    if (f == 0) gb_io[0] = gb;
}

// fixed point (FX): the fp32 value v stored as int32 round(v * 2^shift), saturating like v_cvt_i32_f32
static float pp_host_fx(float v, int32_t shift) {
    const double t = std::nearbyint(static_cast<double>(v) * std::ldexp(1.0, shift));
    const int32_t i = t >= 2147483647.0 ? INT32_MAX : (t <= -2147483648.0 ? INT32_MIN : static_cast<int32_t>(t));
    float out;
    std::memcpy(&out, &i, 4);
    return out;
}
static float pp_host_unfx(float bits, int32_t shift) {
    int32_t i;
    std::memcpy(&i, &bits, 4);
    return static_cast<float>(i) * std::ldexp(1.f, -shift);
}
// a fixed-point word within 1/2 of the int32 range (integer atomics may have wrapped), or a non-finite float
static bool pp_out_of_range(const std::vector<float>& v, bool fx, int32_t shift) {
    const int32_t lim = static_cast<int32_t>(0x80000000u - (1u << (shift - 1)));
    for (float x : v) {
        if (fx) {
            int32_t i;
            std::memcpy(&i, &x, 4);
            if (i >= lim || i <= -lim) return true;
        } else if (!std::isfinite(x)) {
            return true;
        }
    }
    return false;
}

static void pack_bias_rows(const double* F, const double* bias, int64_t rows, int32_t k, int32_t ld,
                           std::vector<float>& dst, bool fx = false, int32_t shift = 24) {
    dst.assign(static_cast<size_t>(rows) * ld, 0.f);
    for (int64_t r = 0; r < rows; ++r) {
        for (int32_t f = 0; f < k; ++f) dst[r * ld + f] = static_cast<float>(F[r * k + f]);
        if (bias) dst[r * ld + k] = static_cast<float>(bias[r]);  // bias column k
    }
    if (fx)
        for (float& v : dst) v = pp_host_fx(v, shift);
}

static void unpack_bias_rows(const std::vector<float>& src, int64_t rows, int32_t k, int32_t ld,
                             double* F, double* bias, bool fx = false, int32_t shift = 24) {
    auto v = [&](int64_t x) { return fx ? pp_host_unfx(src[x], shift) : src[x]; };
    for (int64_t r = 0; r < rows; ++r) {
        for (int32_t f = 0; f < k; ++f) F[r * k + f] = v(r * ld + f);
        if (bias) bias[r] = v(r * ld + k);
    }
}

template <int E>
static void launch_pp_fast(int32_t n_blocks, const DevBuf<int32_t>& work, int32_t n_work, int32_t n_heavy, int32_t n_hblocks,
                           const DevBuf<int64_t>& rowptr, const DevBuf<int32_t>& items,
                           const DevBuf<float>& ratings, DevBuf<float>& P, DevBuf<float>& Q,
                           DevBuf<float>& Y, DevBuf<double>& gb, DevBuf<double>& partial, float lr,
                           float reg, int32_t kf, bool fx, int32_t shift, hipStream_t s) {
    // light ring depth 8: 16 and 32 measured slower (1.33 / 1.34 against 1.28 ms per ML-1M epoch, k = 128)
    auto kern = fx ? svdpp_epoch_fast_kernel<E, 8, true> : svdpp_epoch_fast_kernel<E, 8, false>;
    hipLaunchKernelGGL(kern, dim3(n_blocks), dim3(256), 0, s, work.p,
                       n_work, n_heavy, n_hblocks, rowptr.p, items.p, ratings.p, P.p, Q.p, Y.p,
                       rs::buffer_bytes32(Q.n, 4, "item factor matrix"), rs::buffer_bytes32(Y.n, 4, "implicit factor matrix"), gb.p,
                       partial.p, lr, reg, kf, std::ldexp(1.f, shift));
}

}  // namespace rs

extern "C" int rs_svdpp_fit(rs_ctx* ctx, const rs_ratings* r, const rs_sgd_params* p, double* P,
                            double* Q, double* Y, double* bu, double* bi, double* gb) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        rs::drop_fit_cache(ctx);
        int st = rs::check_ratings(ctx, r);
        if (st != RS_OK) return st;
        if (!p || !P || !Q || !Y || !bu || !bi || !gb)
            return rs::set_error(ctx, RS_ERR_INVALID, "NULL argument");
        const int32_t k = p->n_factors;
        if (k < 1 || k > 511) return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 511]");
        if (p->n_epochs < 0) return rs::set_error(ctx, RS_ERR_INVALID, "n_epochs < 0");
        hipStream_t s = ctx->stream;
        const float lr = static_cast<float>(p->lr), reg = static_cast<float>(p->reg);
        rs::UserCSR csr;  // N(u) = TrainSet.UserRatings() (data.go:185-199), data order
        rs::build_csr(r->nnz, r->n_users, r->users, r->items, r->ratings, csr);
        csr.cols.resize(csr.cols.size() + 64, 0);  // pp_chain reads ids up to 3 batches (<= 48) ahead
        csr.vals.resize(csr.vals.size() + 64, 0.f);
        rs::DevBuf<int64_t> drow(csr.rowptr.size());
        rs::DevBuf<int32_t> dcol(csr.cols.size());
        rs::DevBuf<float> dval(csr.vals.size());
        drow.upload(csr.rowptr.data(), csr.rowptr.size(), s);
        dcol.upload(csr.cols.data(), csr.cols.size(), s);
        dval.upload(csr.vals.data(), csr.vals.size(), s);
        rs::DevBuf<double> dgb(1);
        dgb.upload(gb, 1, s);
        if (p->mode == RS_SGD_ORDERED) {
            const int64_t nnz = r->nnz;
            rs::DevBuf<int32_t> du(std::max<int64_t>(1, nnz)), di(std::max<int64_t>(1, nnz));
            rs::DevBuf<float> dr(std::max<int64_t>(1, nnz));
            std::vector<float> rf(nnz);
            for (int64_t t = 0; t < nnz; ++t) rf[t] = static_cast<float>(r->ratings[t]);
            du.upload(r->users, nnz, s);
            di.upload(r->items, nnz, s);
            dr.upload(rf.data(), nnz, s);
            std::vector<float> hP, hQ, hY, hbu, hbi;
            rs::pack_rows_f32(P, r->n_users, k, k, hP);
            rs::pack_rows_f32(Q, r->n_items, k, k, hQ);
            rs::pack_rows_f32(Y, r->n_items, k, k, hY);
            rs::pack_rows_f32(bu, r->n_users, 1, 1, hbu);
            rs::pack_rows_f32(bi, r->n_items, 1, 1, hbi);
            rs::DevBuf<float> dP(std::max<size_t>(1, hP.size())), dQ(std::max<size_t>(1, hQ.size())),
                dY(std::max<size_t>(1, hY.size())), dbu(std::max<size_t>(1, hbu.size())),
                dbi(std::max<size_t>(1, hbi.size()));
            dP.upload(hP.data(), hP.size(), s);
            dQ.upload(hQ.data(), hQ.size(), s);
            dY.upload(hY.data(), hY.size(), s);
            dbu.upload(hbu.data(), hbu.size(), s);
            dbi.upload(hbi.data(), hbi.size(), s);
            rs::kernel_span_begin(ctx);
            if (nnz > 0 && p->n_epochs > 0) {
                if (k <= 256)
                    hipLaunchKernelGGL((rs::svdpp_ordered_kernel<256>), dim3(1), dim3(256), 0, s, nnz, du.p, di.p, dr.p, drow.p, dcol.p, dP.p, dQ.p, dY.p, dbu.p, dbi.p, k, dgb.p, p->n_epochs, lr, reg);
                else
                    hipLaunchKernelGGL((rs::svdpp_ordered_kernel<512>), dim3(1), dim3(512), 0, s, nnz, du.p, di.p, dr.p, drow.p, dcol.p, dP.p, dQ.p, dY.p, dbu.p, dbi.p, k, dgb.p, p->n_epochs, lr, reg);
                RS_HIP(hipGetLastError());
            }
            rs::kernel_span_end(ctx);
            dP.download(hP.data(), hP.size(), s);
            dQ.download(hQ.data(), hQ.size(), s);
            dY.download(hY.data(), hY.size(), s);
            dbu.download(hbu.data(), hbu.size(), s);
            dbi.download(hbi.data(), hbi.size(), s);
            dgb.download(gb, 1, s);
            RS_HIP(hipStreamSynchronize(s));
            rs::unpack_rows_f64(hP, r->n_users, k, k, P);
            rs::unpack_rows_f64(hQ, r->n_items, k, k, Q);
            rs::unpack_rows_f64(hY, r->n_items, k, k, Y);
            rs::unpack_rows_f64(hbu, r->n_users, 1, 1, bu);
            rs::unpack_rows_f64(hbi, r->n_items, 1, 1, bi);
            return RS_OK;
        }
        // FAST: heaviest user first; GlobalBias warm start (common.hpp)
        if (p->n_epochs > 0) {
            *gb = rs::gb_warm_start(r, bu, bi);
            dgb.upload(gb, 1, s);
        }
        std::vector<int32_t> order;
        for (int32_t x = 0; x < r->n_users; ++x)
            if (csr.rowptr[x + 1] > csr.rowptr[x]) order.push_back(x);
        std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
            return csr.rowptr[x + 1] - csr.rowptr[x] > csr.rowptr[y + 1] - csr.rowptr[y];
        });
        const int32_t E = (k + 1 + 63) / 64, ld = 64 * E;
        if (static_cast<int64_t>(std::max(1, r->n_items)) * ld * 4 >= (int64_t{1} << 31) - 64)
            return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "n_items * n_factors too large");
        const int32_t n_work = static_cast<int32_t>(order.size());
        // blocks of four waves striding over the LPT-ordered users: at most one block per CU.  The
        // number of users in flight sets the Hogwild error (every in-flight user trains on implicit
        // sums S0 read when its row started, while the others decay the same y_j): on the ML-1M shape
        // (k = 128, 20 epochs) 512 blocks give held-out RMSE 0.672-0.684, 384 give 0.649-0.656 run to
        // run, 128-320 give 0.6463-0.6475 on every run against the sequential restatement's 0.6470
        // (heaviest-first order) and 0.6493 (user-id order), at the same epoch time (1.27 ms: the
        // heaviest user's chain bounds it); profiles/r03_experiments/pp_accuracy.log.
        int cus = 256;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
            cus = 256;
        const int32_t cap = cus;
        // users with >= heavy_min ratings (LPT order: the first n_heavy work items) run on the heavy
        // blocks, n_hblocks of them striding over those users
        int32_t n_heavy = 0;
        int32_t heavy_min = 1024;
        if (const char* env = std::getenv("RSGPU_PP_HEAVY")) heavy_min = std::atoi(env);
        while (heavy_min > 0 && n_heavy < n_work &&
               csr.rowptr[order[n_heavy] + 1] - csr.rowptr[order[n_heavy]] >= heavy_min)
            ++n_heavy;
        // one block per heavy user: fewer blocks striding over them (or every user on the block path,
        // heavy_min = 1) measured slower at equal or worse RMSE (profiles/r03_experiments/pp_accuracy.log)
        // Users in flight set the Hogwild error, so a set with few users gets fewer light blocks: at least
        // kPPUsersPerWave light users per wave (round 5).  ML-100K (943 users) on 256 blocks of 4 waves had every
        // user in flight at once: 5-fold-0 held-out 4.75 / 4.70 on the -10..10 rescaled ratings against 4.54 /
        // 4.58 for the sequential restatement (0.922 against 0.920 on stars); 32 blocks: 4.54 / 4.57
        // (profiles/r05/svdpp_blocks_scales.log).  ML-1M (6040 users) keeps about one block per CU (250).
        constexpr int32_t kPPUsersPerWave = 6;
        const int32_t light_cap = std::max<int32_t>(1, (n_work - n_heavy + 4 * kPPUsersPerWave - 1) / (4 * kPPUsersPerWave));
        const int32_t n_hblocks = n_heavy;
        const int32_t n_light_blocks =
            n_work > n_heavy || n_hblocks == 0
                ? std::max<int32_t>(1, std::min<int32_t>({(n_work - n_heavy + 3) / 4, cap, light_cap}))
                : 0;
        const int32_t n_blocks = n_hblocks + n_light_blocks;
        rs::DevBuf<int32_t> dwork(std::max<size_t>(1, order.size()));
        dwork.upload(order.data(), order.size(), s);
        std::vector<float> hP, hQ, hY;
        const bool fx = true;  // fixed-point Q and Y (see pp_ld)
        // the fixed-point scale from the ratings' spread (fx_shift_for, sgd_plan.hpp: 2^-24 on star scales)
        double lo = 0.0, hi = 0.0, sum = 0.0;
        for (int64_t t = 0; t < r->nnz; ++t) {
            const double v = r->ratings[t];
            lo = t == 0 ? v : std::min(lo, v);
            hi = t == 0 ? v : std::max(hi, v);
            sum += v;
        }
        const int32_t shift = rs::fx_shift_for(lo, hi, r->nnz > 0 ? sum / static_cast<double>(r->nnz) : 0.0);
        rs::pack_bias_rows(P, bu, r->n_users, k, ld, hP);
        rs::pack_bias_rows(Q, bi, r->n_items, k, ld, hQ, fx, shift);
        rs::pack_bias_rows(Y, nullptr, r->n_items, k, ld, hY, fx, shift);
        rs::DevBuf<float> dP(std::max<size_t>(1, hP.size())), dQ(std::max<size_t>(1, hQ.size())),
            dY(std::max<size_t>(1, hY.size()));
        rs::DevBuf<double> dpart(n_blocks);
        dP.upload(hP.data(), hP.size(), s);
        dQ.upload(hQ.data(), hQ.size(), s);
        dY.upload(hY.data(), hY.size(), s);
        const double inv_nnz = r->nnz > 0 ? 1.0 / static_cast<double>(r->nnz) : 0.0;
        RS_HIP(hipStreamSynchronize(s));
        rs::kernel_span_begin(ctx);
        for (int32_t ep = 0; ep < p->n_epochs; ++ep) {
            switch (E) {
                case 1: rs::launch_pp_fast<1>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
                case 2: rs::launch_pp_fast<2>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
                case 3: rs::launch_pp_fast<3>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
                case 4: rs::launch_pp_fast<4>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
                case 5: rs::launch_pp_fast<5>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
                case 6: rs::launch_pp_fast<6>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
                case 7: rs::launch_pp_fast<7>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
                default: rs::launch_pp_fast<8>(n_blocks, dwork, n_work, n_heavy, n_hblocks, drow, dcol, dval, dP, dQ, dY, dgb, dpart, lr, reg, k, fx, shift, s); break;
            }
            RS_HIP(hipGetLastError());
            hipLaunchKernelGGL(rs::pp_gb_fold_kernel, dim3(1), dim3(256), 0, s, dpart.p,
                               static_cast<int64_t>(n_blocks), dgb.p, inv_nnz);
            RS_HIP(hipGetLastError());
        }
        rs::kernel_span_end(ctx);
        dP.download(hP.data(), hP.size(), s);
        dQ.download(hQ.data(), hQ.size(), s);
        dY.download(hY.data(), hY.size(), s);
        dgb.download(gb, 1, s);
        RS_HIP(hipStreamSynchronize(s));
        rs::unpack_bias_rows(hP, r->n_users, k, ld, P, bu);
        rs::unpack_bias_rows(hQ, r->n_items, k, ld, Q, bi, fx, shift);
        rs::unpack_bias_rows(hY, r->n_items, k, ld, Y, nullptr, fx, shift);
        if (rs::pp_out_of_range(hQ, fx, shift) || rs::pp_out_of_range(hY, fx, shift) || rs::pp_out_of_range(hP, false, shift) ||
            !std::isfinite(*gb))
            return rs::set_error(ctx, RS_ERR_NUMERIC, "SVD++ factors left the fixed-point range (or went non-finite) "
                                                      "during the fit; the returned model is not trustworthy");
        return RS_OK;
    });
}
