// baseline.hip -- BaseLine.Fit (reference core/base.go:135-163), used by KNN-baseline
// (core/knn.go:179-187).  Bias-only SGD is one serial scalar chain (every rating updates the global
// bias, Q2), so the exact reference order is kept: one wave stages 64 (u, i, r) triples at a time
// into LDS and lane 0 walks them in train-set order with the biases resident in LDS (float64,
// -ffp-contract=off), bitwise equal to the fp64 restatement.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.hpp"

namespace rs {

constexpr int kBaselineLdsDoubles = 18 * 1024;  // 144 KiB of biases in LDS

template <bool IN_LDS>
__global__ __launch_bounds__(64) void baseline_fit_kernel(int64_t nnz, const int32_t* __restrict__ users,
                                                          const int32_t* __restrict__ items,
                                                          const double* __restrict__ ratings,
                                                          int32_t n_users, int32_t n_items,
                                                          double* bu_g, double* bi_g, double* gb_io,
                                                          int32_t epochs, double lr, double reg) {
#pragma clang fp contract(off)
    extern __shared__ double lds[];
    __shared__ int32_t su[64], si[64];
    __shared__ double sr[64];
    const int lane = threadIdx.x;
    double* bu = bu_g;
    double* bi = bi_g;
    if constexpr (IN_LDS) {
        bu = lds;
        bi = lds + n_users;
        for (int32_t x = lane; x < n_users; x += 64) bu[x] = bu_g[x];
        for (int32_t x = lane; x < n_items; x += 64) bi[x] = bi_g[x];
        __syncthreads();
    }
    double gb = gb_io[0];
    for (int32_t epoch = 0; epoch < epochs; ++epoch) {              // base.go:145
        for (int64_t base = 0; base < nnz; base += 64) {
            if (base + lane < nnz) {
                su[lane] = users[base + lane];
                si[lane] = items[base + lane];
                sr[lane] = ratings[base + lane];
            }
            __syncthreads();
            if (lane == 0) {
                const int32_t m = static_cast<int32_t>(nnz - base < 64 ? nnz - base : 64);
                for (int32_t t = 0; t < m; ++t) {                   // base.go:146
                    const int32_t u = su[t], i = si[t];
                    const double userBias = bu[u], itemBias = bi[i];  // base.go:150-151
                    double pred = gb;                               // Predict base.go:126-133
                    pred += bu[u];
                    pred += bi[i];
                    const double diff = pred - sr[t];               // base.go:153
                    gb -= lr * diff;                                // base.go:158
                    bu[u] -= lr * (diff + reg * userBias);          // base.go:159
                    bi[i] -= lr * (diff + reg * itemBias);          // base.go:160
                }
            }
            __syncthreads();
        }
    }
    if constexpr (IN_LDS) {
        for (int32_t x = lane; x < n_users; x += 64) bu_g[x] = bu[x];
        for (int32_t x = lane; x < n_items; x += 64) bi_g[x] = bi[x];
    }
    if (lane == 0) gb_io[0] = gb;
}

}  // namespace rs

extern "C" int rs_baseline_fit(rs_ctx* ctx, const rs_ratings* r, int32_t n_epochs, double lr,
                               double reg, double* bu, double* bi, double* gb) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        rs::drop_fit_cache(ctx);
        int st = rs::check_ratings(ctx, r);
        if (st != RS_OK) return st;
        if (n_epochs < 0 || !bu || !bi || !gb) return rs::set_error(ctx, RS_ERR_INVALID, "bad arguments");
        hipStream_t s = ctx->stream;
        const int64_t nnz = r->nnz;
        rs::DevBuf<int32_t> du(std::max<int64_t>(1, nnz)), di(std::max<int64_t>(1, nnz));
        rs::DevBuf<double> dr(std::max<int64_t>(1, nnz)), dbu(std::max(1, r->n_users)),
            dbi(std::max(1, r->n_items)), dgb(1);
        du.upload(r->users, nnz, s);
        di.upload(r->items, nnz, s);
        dr.upload(r->ratings, nnz, s);
        dbu.upload(bu, r->n_users, s);
        dbi.upload(bi, r->n_items, s);
        dgb.upload(gb, 1, s);
        const int64_t nb = static_cast<int64_t>(r->n_users) + r->n_items;
        rs::kernel_span_begin(ctx);
        if (nnz > 0 && n_epochs > 0) {
            if (nb <= rs::kBaselineLdsDoubles)
                hipLaunchKernelGGL(rs::baseline_fit_kernel<true>, dim3(1), dim3(64), nb * sizeof(double), s, nnz, du.p, di.p, dr.p, r->n_users, r->n_items, dbu.p, dbi.p, dgb.p, n_epochs, lr, reg);
            else
                hipLaunchKernelGGL(rs::baseline_fit_kernel<false>, dim3(1), dim3(64), 0, s, nnz, du.p, di.p, dr.p, r->n_users, r->n_items, dbu.p, dbi.p, dgb.p, n_epochs, lr, reg);
            RS_HIP(hipGetLastError());
        }
        rs::kernel_span_end(ctx);
        dbu.download(bu, r->n_users, s);
        dbi.download(bi, r->n_items, s);
        dgb.download(gb, 1, s);
        RS_HIP(hipStreamSynchronize(s));
        return RS_OK;
    });
}
