// sgd.hip -- K1: SGD epoch of the Funk-SVD model (reference core/svd.go:63-132), gfx950.
//
// Two schedules (SURVEY §8a parity contract):
//   FAST    user-CSR; one G-lane group per user; p_u and b_u live in VGPRs for the whole user row;
//           q_i / b_i are gathered (prefetched one rating ahead) and written back Hogwild-style;
//           GlobalBias (Q2) is a per-group local SGD copy folded at epoch end as
//           gb += sum_w n_w * (gb_w - gb) / nnz (deterministic fixed-order fold).
//           Users are dispatched heaviest-first (LPT) so the serial chain of the heaviest user starts
//           at t=0.  RMSE parity with the reference (P2).
//   ORDERED one group walks the ratings in train-set order with the exact update order of
//           svd.go:93-129 (aliasing Q1: q_i is updated with the NEW p_u) -- factor parity (P1).
//
// Algorithmic bytes per epoch: nnz*(16 + 8k) + U*(16 + 8k)  (fp32 factors).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "common.hpp"
#include "wave.hpp"

namespace rs {

// --------------------------------------------------------------------------------------------
// FAST epoch kernel

template <int G, int V>
__global__ __launch_bounds__(256) void svd_epoch_fast_kernel(
    const int32_t* __restrict__ work, int32_t n_work, const int64_t* __restrict__ rowptr,
    const int32_t* __restrict__ items, const float* __restrict__ ratings, float* __restrict__ P,
    float* Q, float* __restrict__ bu, float* bi, int32_t ld, const double* __restrict__ gb_in,
    double* __restrict__ gb_partial, float lr, float reg) {
#pragma clang fp contract(fast)
    constexpr int GPB = 256 / G;  // groups per block
    __shared__ double s_contrib[GPB];
    const int gl = threadIdx.x & (G - 1);
    const int grp = threadIdx.x / G;
    const int w = blockIdx.x * GPB + grp;
    const float gb0 = static_cast<float>(gb_in[0]);
    double contrib = 0.0;

    if (w < n_work) {
        const int32_t u = work[w];
        const int64_t b = rowptr[u], e = rowptr[u + 1];
        bool act[V];
        float4 p[V];
        const float* prow = P + static_cast<int64_t>(u) * ld;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int c = gl + G * v;
            act[v] = 4 * c < ld;
            p[v] = act[v] ? *reinterpret_cast<const float4*>(prow + 4 * c) : make_float4(0, 0, 0, 0);
        }
        float ub = bu[u];
        float gb = gb0;
        if (b < e) {
            int32_t it = items[b];
            float rr = ratings[b];
            float4 q[V];
            {
                const float* qrow = Q + static_cast<int64_t>(it) * ld;
#pragma unroll
                for (int v = 0; v < V; ++v)
                    q[v] = act[v] ? *reinterpret_cast<const float4*>(qrow + 4 * (gl + G * v))
                                  : make_float4(0, 0, 0, 0);
            }
            float bq = bi[it];
            int32_t itn = it;
            float rn = 0.f;
            if (b + 1 < e) {
                itn = items[b + 1];
                rn = ratings[b + 1];
            }
            for (int64_t pos = b; pos < e; ++pos) {
                // prefetch rating pos+1's item row and rating pos+2's (item, rating)
                const bool more = pos + 1 < e;
                float4 qn[V];
                float bqn = 0.f;
                if (more) {
                    const float* qrow = Q + static_cast<int64_t>(itn) * ld;
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        qn[v] = act[v] ? *reinterpret_cast<const float4*>(qrow + 4 * (gl + G * v))
                                       : make_float4(0, 0, 0, 0);
                    bqn = bi[itn];
                } else {
#pragma unroll
                    for (int v = 0; v < V; ++v) qn[v] = make_float4(0, 0, 0, 0);
                }
                int32_t itnn = 0;
                float rnn = 0.f;
                if (pos + 2 < e) {
                    itnn = items[pos + 2];
                    rnn = ratings[pos + 2];
                }
                // svd.go:102 -> Predict: ((gb + b_u) + b_i) + <p_u, q_i>
                float s = 0.f;
#pragma unroll
                for (int v = 0; v < V; ++v) s += dot4(p[v], q[v]);
                s = group_sum<G>(s);
                const float diff = ((gb + ub) + bq) + s - rr;
                gb -= lr * diff;                                   // svd.go:106 (local copy)
                const float ub_new = ub - lr * (diff + reg * ub);  // svd.go:108-109
                const float bq_new = bq - lr * (diff + reg * bq);  // svd.go:111-112
#pragma unroll
                for (int v = 0; v < V; ++v) {  // svd.go:114-120 then 122-128 with the new p (Q1)
                    p[v].x = p[v].x - (q[v].x * diff + p[v].x * reg) * lr;
                    p[v].y = p[v].y - (q[v].y * diff + p[v].y * reg) * lr;
                    p[v].z = p[v].z - (q[v].z * diff + p[v].z * reg) * lr;
                    p[v].w = p[v].w - (q[v].w * diff + p[v].w * reg) * lr;
                    q[v].x = q[v].x - (p[v].x * diff + q[v].x * reg) * lr;
                    q[v].y = q[v].y - (p[v].y * diff + q[v].y * reg) * lr;
                    q[v].z = q[v].z - (p[v].z * diff + q[v].z * reg) * lr;
                    q[v].w = q[v].w - (p[v].w * diff + q[v].w * reg) * lr;
                }
                {
                    float* qrow = Q + static_cast<int64_t>(it) * ld;
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (act[v]) *reinterpret_cast<float4*>(qrow + 4 * (gl + G * v)) = q[v];
                }
                bi[it] = bq_new;  // every lane of the group stores the same bits
                ub = ub_new;
                if (itn == it) {  // repeated (u, i): use the value just written, not the prefetch
#pragma unroll
                    for (int v = 0; v < V; ++v) qn[v] = q[v];
                    bqn = bq_new;
                }
#pragma unroll
                for (int v = 0; v < V; ++v) q[v] = qn[v];
                bq = bqn;
                it = itn;
                rr = rn;
                itn = itnn;
                rn = rnn;
            }
        }
        float* pw = P + static_cast<int64_t>(u) * ld;
#pragma unroll
        for (int v = 0; v < V; ++v)
            if (act[v]) *reinterpret_cast<float4*>(pw + 4 * (gl + G * v)) = p[v];
        bu[u] = ub;
        contrib = static_cast<double>(e - b) * (static_cast<double>(gb) - static_cast<double>(gb0));
    }
    if (gl == 0) s_contrib[grp] = contrib;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int g = 0; g < GPB; ++g) t += s_contrib[g];
        gb_partial[blockIdx.x] = t;
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

// --------------------------------------------------------------------------------------------
// ORDERED kernel: one 16-lane group, all epochs, reference visit and update order.

template <int V>
__global__ __launch_bounds__(64) void svd_ordered_kernel(
    int64_t nnz, const int32_t* __restrict__ users, const int32_t* __restrict__ items,
    const float* __restrict__ ratings, float* P, float* Q, float* bu, float* bi, int32_t ld,
    double* gb_io, int32_t epochs, float lr, float reg) {
#pragma clang fp contract(off)
    constexpr int G = 16;
    const int gl = threadIdx.x;
    if (gl >= G) return;
    const double lrd = lr, regd = reg;
    bool act[V];
#pragma unroll
    for (int v = 0; v < V; ++v) act[v] = 4 * (gl + G * v) < ld;
    double gb = gb_io[0];
    for (int32_t epoch = 0; epoch < epochs; ++epoch) {       // svd.go:92
        for (int64_t n = 0; n < nnz; ++n) {                   // svd.go:93
            const int32_t u = users[n], i = items[n];
            const float r = ratings[n];
            float* prow = P + static_cast<int64_t>(u) * ld;   // svd.go:99-100 aliases
            float* qrow = Q + static_cast<int64_t>(i) * ld;
            float4 p[V], q[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int c = 4 * (gl + G * v);
                p[v] = act[v] ? *reinterpret_cast<const float4*>(prow + c) : make_float4(0, 0, 0, 0);
                q[v] = act[v] ? *reinterpret_cast<const float4*>(qrow + c) : make_float4(0, 0, 0, 0);
            }
            const float ub = bu[u], ib = bi[i];               // svd.go:97-98
            float s = 0.f;
#pragma unroll
            for (int v = 0; v < V; ++v) s += dot4(p[v], q[v]);
            s = group_sum<G>(s);
            double pred = gb;                                 // Predict svd.go:35-48
            pred += static_cast<double>(ub);
            pred += static_cast<double>(ib);
            pred += static_cast<double>(s);
            const double diff = pred - static_cast<double>(r);
            gb -= lrd * diff;                                 // svd.go:105-106
            const float ub_new = static_cast<float>(ub - lrd * (diff + regd * ub));  // 108-109
            const float ib_new = static_cast<float>(ib - lrd * (diff + regd * ib));  // 111-112
            const float df = static_cast<float>(diff);
#pragma unroll
            for (int v = 0; v < V; ++v) {                     // svd.go:114-120
                float4 a;
                a.x = (q[v].x * df + p[v].x * reg) * lr;
                a.y = (q[v].y * df + p[v].y * reg) * lr;
                a.z = (q[v].z * df + p[v].z * reg) * lr;
                a.w = (q[v].w * df + p[v].w * reg) * lr;
                p[v].x -= a.x; p[v].y -= a.y; p[v].z -= a.z; p[v].w -= a.w;
            }
#pragma unroll
            for (int v = 0; v < V; ++v) {                     // svd.go:122-128 (new p: Q1)
                float4 a;
                a.x = (p[v].x * df + q[v].x * reg) * lr;
                a.y = (p[v].y * df + q[v].y * reg) * lr;
                a.z = (p[v].z * df + q[v].z * reg) * lr;
                a.w = (p[v].w * df + q[v].w * reg) * lr;
                q[v].x -= a.x; q[v].y -= a.y; q[v].z -= a.z; q[v].w -= a.w;
            }
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const int c = 4 * (gl + G * v);
                if (act[v]) {
                    *reinterpret_cast<float4*>(prow + c) = p[v];
                    *reinterpret_cast<float4*>(qrow + c) = q[v];
                }
            }
            bu[u] = ub_new;  // all 16 lanes store identical bits: each lane re-reads its own write
            bi[i] = ib_new;
        }
    }
    if (gl == 0) gb_io[0] = gb;
}

}  // namespace rs

// ------------------------------------------------------------------------------------------------
// Plan (device-resident CSR + factors)

struct rs_svd_plan {
    rs_ctx* ctx = nullptr;
    int32_t n_users = 0, n_items = 0, k = 0, ld = 0, n_work = 0;
    int64_t nnz = 0;
    rs::DevBuf<int64_t> rowptr;
    rs::DevBuf<int32_t> items;
    rs::DevBuf<float> ratings;
    rs::DevBuf<int32_t> work;
    rs::DevBuf<float> P, Q, bu, bi;
    rs::DevBuf<double> gb, partial;
    int32_t n_blocks = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0;
    int32_t last_launches = 0;
    bool timing = false;
    hipStream_t last_stream = nullptr;  // stream of the last enqueued epochs (synced before copies)
    std::vector<hipEvent_t> tev;  // timing mode: [2 * epoch] start, [2 * epoch + 1] end
    int32_t tev_used = 0;
    ~rs_svd_plan() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        for (hipEvent_t e : tev) (void)hipEventDestroy(e);
    }
};

namespace rs {

static int fast_groups(int32_t ld) { return ld <= 32 ? 8 : 16; }

template <int G, int V>
static void launch_fast_t(rs_svd_plan* pl, float lr, float reg, hipStream_t s) {
    hipLaunchKernelGGL((svd_epoch_fast_kernel<G, V>), dim3(pl->n_blocks), dim3(256), 0, s,
                       pl->work.p, pl->n_work, pl->rowptr.p, pl->items.p, pl->ratings.p, pl->P.p,
                       pl->Q.p, pl->bu.p, pl->bi.p, pl->ld, pl->gb.p, pl->partial.p, lr, reg);
}

static void launch_fast(rs_svd_plan* pl, float lr, float reg, hipStream_t s) {
    const int32_t ld = pl->ld;
    if (ld <= 32) launch_fast_t<8, 1>(pl, lr, reg, s);
    else if (ld <= 64) launch_fast_t<16, 1>(pl, lr, reg, s);
    else if (ld <= 128) launch_fast_t<16, 2>(pl, lr, reg, s);
    else if (ld <= 256) launch_fast_t<16, 4>(pl, lr, reg, s);
    else launch_fast_t<16, 8>(pl, lr, reg, s);
    RS_HIP(hipGetLastError());
}

static void launch_ordered(int64_t nnz, const int32_t* u, const int32_t* i, const float* r,
                           float* P, float* Q, float* bu, float* bi, int32_t ld, double* gb,
                           int32_t epochs, float lr, float reg, hipStream_t s) {
    if (ld <= 64)
        hipLaunchKernelGGL((svd_ordered_kernel<1>), dim3(1), dim3(16), 0, s, nnz, u, i, r, P, Q, bu, bi, ld, gb, epochs, lr, reg);
    else if (ld <= 128)
        hipLaunchKernelGGL((svd_ordered_kernel<2>), dim3(1), dim3(16), 0, s, nnz, u, i, r, P, Q, bu, bi, ld, gb, epochs, lr, reg);
    else if (ld <= 256)
        hipLaunchKernelGGL((svd_ordered_kernel<4>), dim3(1), dim3(16), 0, s, nnz, u, i, r, P, Q, bu, bi, ld, gb, epochs, lr, reg);
    else
        hipLaunchKernelGGL((svd_ordered_kernel<8>), dim3(1), dim3(16), 0, s, nnz, u, i, r, P, Q, bu, bi, ld, gb, epochs, lr, reg);
    RS_HIP(hipGetLastError());
}

constexpr int32_t kMaxFactors = 512;

static void plan_build(rs_ctx* ctx, const rs_ratings* r, int32_t k, rs_svd_plan* pl) {
    hipStream_t s = ctx->stream;
    pl->ctx = ctx;
    pl->n_users = r->n_users;
    pl->n_items = r->n_items;
    pl->k = k;
    pl->ld = round_up4(k);
    pl->nnz = r->nnz;
    UserCSR csr;
    build_csr(r->nnz, r->n_users, r->users, r->items, r->ratings, csr);
    // LPT dispatch order: heaviest user first (ties by user id), empty users dropped.
    std::vector<int32_t> order;
    order.reserve(r->n_users);
    for (int32_t x = 0; x < r->n_users; ++x)
        if (csr.rowptr[x + 1] > csr.rowptr[x]) order.push_back(x);
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        return csr.rowptr[a + 1] - csr.rowptr[a] > csr.rowptr[b + 1] - csr.rowptr[b];
    });
    pl->n_work = static_cast<int32_t>(order.size());
    const int gpb = 256 / fast_groups(pl->ld);
    pl->n_blocks = std::max<int32_t>(1, (pl->n_work + gpb - 1) / gpb);
    pl->rowptr.alloc(csr.rowptr.size());
    pl->items.alloc(std::max<size_t>(1, csr.cols.size()));
    pl->ratings.alloc(std::max<size_t>(1, csr.vals.size()));
    pl->work.alloc(std::max<size_t>(1, order.size()));
    pl->rowptr.upload(csr.rowptr.data(), csr.rowptr.size(), s);
    pl->items.upload(csr.cols.data(), csr.cols.size(), s);
    pl->ratings.upload(csr.vals.data(), csr.vals.size(), s);
    pl->work.upload(order.data(), order.size(), s);
    pl->P.alloc(static_cast<size_t>(std::max(1, r->n_users)) * pl->ld);
    pl->Q.alloc(static_cast<size_t>(std::max(1, r->n_items)) * pl->ld);
    pl->bu.alloc(std::max(1, r->n_users));
    pl->bi.alloc(std::max(1, r->n_items));
    pl->gb.alloc(1);
    pl->partial.alloc(pl->n_blocks);
    RS_HIP(hipMemsetAsync(pl->P.p, 0, pl->P.n * sizeof(float), s));
    RS_HIP(hipMemsetAsync(pl->Q.p, 0, pl->Q.n * sizeof(float), s));
    RS_HIP(hipMemsetAsync(pl->bu.p, 0, pl->bu.n * sizeof(float), s));
    RS_HIP(hipMemsetAsync(pl->bi.p, 0, pl->bi.n * sizeof(float), s));
    RS_HIP(hipMemsetAsync(pl->gb.p, 0, sizeof(double), s));
    RS_HIP(hipEventCreate(&pl->ev0));
    RS_HIP(hipEventCreate(&pl->ev1));
    RS_HIP(hipStreamSynchronize(s));  // host CSR vectors die with this scope
}

static void plan_sync_last(rs_svd_plan* pl) {
    if (pl->last_stream) RS_HIP(hipStreamSynchronize(pl->last_stream));
}

static void plan_upload(rs_svd_plan* pl, const double* P, const double* Q, const double* bu,
                        const double* bi, const double* gb) {
    plan_sync_last(pl);
    hipStream_t s = pl->ctx->stream;
    std::vector<float> tmp;
    if (P) {
        pack_rows_f32(P, pl->n_users, pl->k, pl->ld, tmp);
        pl->P.upload(tmp.data(), tmp.size(), s);
        RS_HIP(hipStreamSynchronize(s));
    }
    if (Q) {
        pack_rows_f32(Q, pl->n_items, pl->k, pl->ld, tmp);
        pl->Q.upload(tmp.data(), tmp.size(), s);
        RS_HIP(hipStreamSynchronize(s));
    }
    if (bu) {
        pack_rows_f32(bu, pl->n_users, 1, 1, tmp);
        pl->bu.upload(tmp.data(), tmp.size(), s);
        RS_HIP(hipStreamSynchronize(s));
    }
    if (bi) {
        pack_rows_f32(bi, pl->n_items, 1, 1, tmp);
        pl->bi.upload(tmp.data(), tmp.size(), s);
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
    auto get = [&](const DevBuf<float>& d, int64_t rows, int32_t k, int32_t ld, double* out) {
        tmp.resize(static_cast<size_t>(rows) * ld);
        d.download(tmp.data(), tmp.size(), s);
        RS_HIP(hipStreamSynchronize(s));
        unpack_rows_f64(tmp, rows, k, ld, out);
    };
    if (P) get(pl->P, pl->n_users, pl->k, pl->ld, P);
    if (Q) get(pl->Q, pl->n_items, pl->k, pl->ld, Q);
    if (bu) get(pl->bu, pl->n_users, 1, 1, bu);
    if (bi) get(pl->bi, pl->n_items, 1, 1, bi);
    if (gb) {
        pl->gb.download(gb, 1, s);
        RS_HIP(hipStreamSynchronize(s));
    }
}

static void plan_epochs(rs_svd_plan* pl, int32_t epochs, float lr, float reg, hipStream_t s) {
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
    for (int32_t e = 0; e < epochs; ++e) {
        if (pl->timing) RS_HIP(hipEventRecord(pl->tev[2 * e], s));
        launch_fast(pl, lr, reg, s);
        if (pl->timing) RS_HIP(hipEventRecord(pl->tev[2 * e + 1], s));
        hipLaunchKernelGGL(gb_fold_kernel, dim3(1), dim3(256), 0, s, pl->partial.p,
                           static_cast<int64_t>(pl->n_blocks), pl->gb.p, inv_nnz);
        RS_HIP(hipGetLastError());
    }
    RS_HIP(hipEventRecord(pl->ev1, s));
    pl->last_launches = pl->timing ? epochs : 2 * epochs;
    pl->last_stream = s;
    pl->last_ms = -1.0;  // resolved lazily by rs_svd_plan_last_kernel_ms
}

static int check_sgd(rs_ctx* ctx, const rs_ratings* r, const rs_sgd_params* p) {
    int st = check_ratings(ctx, r);
    if (st != RS_OK) return st;
    if (!p) return set_error(ctx, RS_ERR_INVALID, "params is NULL");
    if (p->n_factors < 1 || p->n_factors > kMaxFactors)
        return set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 512]");
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
            return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 512]");
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

extern "C" void rs_svd_plan_destroy(rs_svd_plan* pl) {
    if (!pl) return;
    (void)hipSetDevice(pl->ctx->device);
    if (pl->last_stream) (void)hipStreamSynchronize(pl->last_stream);
    (void)hipStreamSynchronize(pl->ctx->stream);
    delete pl;
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

extern "C" int rs_svd_plan_device_ptrs(rs_svd_plan* pl, void** P, void** Q, void** bu, void** bi,
                                       void** gb, int32_t* ld) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (P) *P = pl->P.p;
    if (Q) *Q = pl->Q.p;
    if (bu) *bu = pl->bu.p;
    if (bi) *bi = pl->bi.p;
    if (gb) *gb = pl->gb.p;
    if (ld) *ld = pl->ld;
    return RS_OK;
}

extern "C" int rs_svd_plan_set_timing(rs_svd_plan* pl, int32_t on) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    pl->timing = on != 0;
    return RS_OK;
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
            rs_svd_plan pl;
            rs::plan_build(ctx, r, p->n_factors, &pl);
            rs::plan_upload(&pl, P, Q, bu, bi, gb);
            rs::plan_epochs(&pl, p->n_epochs, lr, reg, ctx->stream);
            rs::plan_download(&pl, P, Q, bu, bi, gb);
            return RS_OK;
        }
        // ORDERED: COO in train-set order, one group, all epochs in one launch.
        hipStream_t s = ctx->stream;
        const int32_t k = p->n_factors, ld = rs::round_up4(k);
        const int64_t nnz = r->nnz;
        rs::DevBuf<int32_t> du(std::max<int64_t>(1, nnz)), di(std::max<int64_t>(1, nnz));
        rs::DevBuf<float> dr(std::max<int64_t>(1, nnz));
        std::vector<float> rf(static_cast<size_t>(nnz));
        for (int64_t t = 0; t < nnz; ++t) rf[t] = static_cast<float>(r->ratings[t]);
        du.upload(r->users, nnz, s);
        di.upload(r->items, nnz, s);
        dr.upload(rf.data(), nnz, s);
        rs::DevBuf<float> dP(static_cast<size_t>(std::max(1, r->n_users)) * ld);
        rs::DevBuf<float> dQ(static_cast<size_t>(std::max(1, r->n_items)) * ld);
        rs::DevBuf<float> dbu(std::max(1, r->n_users)), dbi(std::max(1, r->n_items));
        rs::DevBuf<double> dgb(1);
        std::vector<float> hP, hQ, hbu, hbi;
        rs::pack_rows_f32(P, r->n_users, k, ld, hP);
        rs::pack_rows_f32(Q, r->n_items, k, ld, hQ);
        rs::pack_rows_f32(bu, r->n_users, 1, 1, hbu);
        rs::pack_rows_f32(bi, r->n_items, 1, 1, hbi);
        dP.upload(hP.data(), hP.size(), s);
        dQ.upload(hQ.data(), hQ.size(), s);
        dbu.upload(hbu.data(), hbu.size(), s);
        dbi.upload(hbi.data(), hbi.size(), s);
        dgb.upload(gb, 1, s);
        if (nnz > 0 && p->n_epochs > 0)
            rs::launch_ordered(nnz, du.p, di.p, dr.p, dP.p, dQ.p, dbu.p, dbi.p, ld, dgb.p,
                               p->n_epochs, lr, reg, s);
        dP.download(hP.data(), hP.size(), s);
        dQ.download(hQ.data(), hQ.size(), s);
        dbu.download(hbu.data(), hbu.size(), s);
        dbi.download(hbi.data(), hbi.size(), s);
        dgb.download(gb, 1, s);
        RS_HIP(hipStreamSynchronize(s));
        rs::unpack_rows_f64(hP, r->n_users, k, ld, P);
        rs::unpack_rows_f64(hQ, r->n_items, k, ld, Q);
        rs::unpack_rows_f64(hbu, r->n_users, 1, 1, bu);
        rs::unpack_rows_f64(hbi, r->n_items, 1, 1, bi);
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
