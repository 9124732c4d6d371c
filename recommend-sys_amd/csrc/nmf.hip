// nmf.hip -- K3: multiplicative-update NMF epoch (reference core/svd.go:158-251), gfx950.
//
// The reference accumulates userUp/userDown/itemUp/itemDown over all ratings with the factors of
// the START of the epoch (svd.go:186-233 never writes P or Q), then updates every row
// (svd.go:236-249).  Nothing inside an epoch depends on visit order except the summation order of
// each accumulator, which is the row's data order.  So one epoch is two passes without any
// accumulator array in memory and without atomics:
//   item pass  (item-CSR, one wave per item row i, data order):  itemUp/itemDown of i in VGPRs,
//              Q'[i] = Q[i] * itemUp/itemDown     (as written, Q5: Q'[i] = Q[i] * itemUp)
//   user pass  (user-CSR, one wave per user row u, data order):  userUp/userDown of u in VGPRs,
//              P[u] = P[u] * userUp/userDown      (reads Q, not Q')
// then Q <- Q'.  Both passes read the start-of-epoch P and Q, exactly as the reference does.
// The partner row of every rating is gathered D ratings ahead into a register ring; the prediction
// dot product is a 64-lane DPP + permlane reduction.
//
// Algorithmic bytes per epoch: nnz*(8 + 20k) + U*28k + I*24k (fp32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.hpp"
#include "wave.hpp"

namespace rs {

__device__ __forceinline__ float nmf_wave_sum(float x) {
    x = group_sum<16>(x);
    auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
    auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

// One pass.  own = the matrix whose rows this pass updates (rows of the CSR), partner = the other
// factor matrix.  out[row] = own[row] * up / down (or * up when UPONLY, the as-written item rule).
template <int E, int D, bool UPONLY>
__global__ __launch_bounds__(256) void nmf_pass_kernel(
    int32_t n_rows, const int64_t* __restrict__ rowptr, const int32_t* __restrict__ cols,
    const float* __restrict__ vals, const float* __restrict__ own,
    const float* __restrict__ partner, float* __restrict__ out, int32_t k, float reg) {
#pragma clang fp contract(off)
    constexpr int LD = 64 * E, B = 16;
    const int lane = threadIdx.x & 63;
    const int row = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + (threadIdx.x >> 6));
    if (row >= n_rows) return;
    const int64_t b = rowptr[row], e = rowptr[row + 1];
    float p[E], up[E], down[E];
    const float* orow = own + static_cast<int64_t>(row) * LD;
#pragma unroll
    for (int x = 0; x < E; ++x) {
        p[x] = orow[lane + 64 * x];
        up[x] = 0.f;
        down[x] = 0.f;
    }
    auto load = [&](float (&q)[E], int32_t valid, int32_t c) {
        const float* qr = partner + static_cast<int64_t>(valid ? c : 0) * LD;
#pragma unroll
        for (int x = 0; x < E; ++x) q[x] = valid ? qr[lane + 64 * x] : 0.f;
    };
    const int32_t deg = static_cast<int32_t>(e - b);
    float ring[D][E];
#pragma unroll
    for (int s = 0; s < D; ++s) load(ring[s], s < deg, cols[b + s]);  // cols padded by 64
    for (int64_t base = b; base < e; base += B) {
        const int32_t rem = static_cast<int32_t>(e - base);
        int32_t cn[B];
        float rt[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            cn[j] = cols[base + D + j];
            rt[j] = vals[base + j];
        }
#pragma unroll
        for (int j = 0; j < B; ++j) {
            constexpr int kD = D;
            const int slot = j % kD;
            if (j < rem) {
                const float* q = ring[slot];
                float s = 0.f;
#pragma unroll
                for (int x = 0; x < E; ++x) s += p[x] * q[x];
                const float pred = nmf_wave_sum(s);            // svd.go:190 (Predict -> Dot)
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    up[x] = up[x] + q[x] * rt[j];              // svd.go:193-197 / 214-218
                    down[x] = down[x] + q[x] * pred;           // svd.go:200-204 / 221-225
                    down[x] = down[x] + p[x] * reg;            // svd.go:206-210 / 227-231
                }
            }
            load(ring[slot], j + D < rem, cn[j]);
        }
    }
    float* w = out + static_cast<int64_t>(row) * LD;
#pragma unroll
    for (int x = 0; x < E; ++x) {
        // svd.go:236-241 (users, items intended): buffer = up / down; p *= buffer
        // svd.go:243-249 (items as written, Q5):   q *= up (the undivided copy)
        const float buffer = UPONLY ? up[x] : up[x] / down[x];
        w[lane + 64 * x] = lane + 64 * x < k ? p[x] * buffer : 0.f;  // padding stays 0 (0/0)
    }
}

template <int E, int D>
static void nmf_epoch_t(int32_t n_users, int32_t n_items, const DevBuf<int64_t>& urow,
                        const DevBuf<int32_t>& ucol, const DevBuf<float>& uval,
                        const DevBuf<int64_t>& irow, const DevBuf<int32_t>& icol,
                        const DevBuf<float>& ival, float* P, float*& Q, float*& Qn, int32_t k,
                        float reg, bool as_written, hipStream_t s) {
    const dim3 gi((n_items + 3) / 4), gu((n_users + 3) / 4);
    if (n_items > 0) {
        if (as_written)
            hipLaunchKernelGGL((nmf_pass_kernel<E, D, true>), gi, dim3(256), 0, s, n_items, irow.p, icol.p, ival.p, Q, P, Qn, k, reg);
        else
            hipLaunchKernelGGL((nmf_pass_kernel<E, D, false>), gi, dim3(256), 0, s, n_items, irow.p, icol.p, ival.p, Q, P, Qn, k, reg);
    }
    if (n_users > 0)
        hipLaunchKernelGGL((nmf_pass_kernel<E, D, false>), gu, dim3(256), 0, s, n_users, urow.p, ucol.p, uval.p, P, Q, P, k, reg);
    RS_HIP(hipGetLastError());
    std::swap(Q, Qn);
}

}  // namespace rs

extern "C" int rs_nmf_fit(rs_ctx* ctx, const rs_ratings* r, int32_t n_factors, int32_t n_epochs,
                          double reg, int32_t as_written, double* P, double* Q) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        int st = rs::check_ratings(ctx, r);
        if (st != RS_OK) return st;
        if (n_factors < 1 || n_factors > 512)
            return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 512]");
        if (n_epochs < 0 || !P || !Q) return rs::set_error(ctx, RS_ERR_INVALID, "bad NMF arguments");
        hipStream_t s = ctx->stream;
        const int32_t k = n_factors, E = k <= 64 ? 1 : k <= 128 ? 2 : k <= 256 ? 4 : 8, ld = 64 * E;
        rs::UserCSR ucsr, icsr;
        rs::build_csr(r->nnz, r->n_users, r->users, r->items, r->ratings, ucsr);
        rs::build_csr(r->nnz, r->n_items, r->items, r->users, r->ratings, icsr);
        for (auto* c : {&ucsr, &icsr}) {  // kernels read 16-entry batches D ahead
            c->cols.resize(c->cols.size() + 64, 0);
            c->vals.resize(c->vals.size() + 64, 0.f);
        }
        rs::DevBuf<int64_t> urow(ucsr.rowptr.size()), irow(icsr.rowptr.size());
        rs::DevBuf<int32_t> ucol(ucsr.cols.size()), icol(icsr.cols.size());
        rs::DevBuf<float> uval(ucsr.vals.size()), ival(icsr.vals.size());
        urow.upload(ucsr.rowptr.data(), ucsr.rowptr.size(), s);
        irow.upload(icsr.rowptr.data(), icsr.rowptr.size(), s);
        ucol.upload(ucsr.cols.data(), ucsr.cols.size(), s);
        icol.upload(icsr.cols.data(), icsr.cols.size(), s);
        uval.upload(ucsr.vals.data(), ucsr.vals.size(), s);
        ival.upload(icsr.vals.data(), icsr.vals.size(), s);
        std::vector<float> hP, hQ;
        rs::pack_rows_f32(P, r->n_users, k, ld, hP);
        rs::pack_rows_f32(Q, r->n_items, k, ld, hQ);
        rs::DevBuf<float> dP(std::max<size_t>(1, hP.size())), dQa(std::max<size_t>(1, hQ.size())),
            dQb(std::max<size_t>(1, hQ.size()));
        dP.upload(hP.data(), hP.size(), s);
        dQa.upload(hQ.data(), hQ.size(), s);
        float* q = dQa.p;
        float* qn = dQb.p;
        const float fr = static_cast<float>(reg);
        RS_HIP(hipStreamSynchronize(s));
        rs::kernel_span_begin(ctx);
        for (int32_t ep = 0; ep < n_epochs; ++ep) {
            switch (E) {
                case 1: rs::nmf_epoch_t<1, 8>(r->n_users, r->n_items, urow, ucol, uval, irow, icol, ival, dP.p, q, qn, k, fr, as_written != 0, s); break;
                case 2: rs::nmf_epoch_t<2, 8>(r->n_users, r->n_items, urow, ucol, uval, irow, icol, ival, dP.p, q, qn, k, fr, as_written != 0, s); break;
                case 4: rs::nmf_epoch_t<4, 8>(r->n_users, r->n_items, urow, ucol, uval, irow, icol, ival, dP.p, q, qn, k, fr, as_written != 0, s); break;
                default: rs::nmf_epoch_t<8, 4>(r->n_users, r->n_items, urow, ucol, uval, irow, icol, ival, dP.p, q, qn, k, fr, as_written != 0, s); break;
            }
        }
        rs::kernel_span_end(ctx);
        dP.download(hP.data(), hP.size(), s);
        RS_HIP(hipMemcpyAsync(hQ.data(), q, hQ.size() * sizeof(float), hipMemcpyDeviceToHost, s));
        RS_HIP(hipStreamSynchronize(s));
        rs::unpack_rows_f64(hP, r->n_users, k, ld, P);
        rs::unpack_rows_f64(hQ, r->n_items, k, ld, Q);
        return RS_OK;
    });
}
