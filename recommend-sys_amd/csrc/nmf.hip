// nmf.hip -- K3: multiplicative-update NMF epoch (reference core/svd.go:158-251), gfx950.
//
// The reference accumulates userUp/userDown/itemUp/itemDown over all ratings with the factors of
// the START of the epoch (svd.go:186-233 never writes P or Q), then updates every row
// (svd.go:236-249).  Nothing inside an epoch depends on visit order except the summation order of
// each accumulator, which is the row's data order.  So one epoch is two passes without any
// accumulator array in memory and without atomics:
//   item pass  (item-CSR, data order):  itemUp/itemDown of i in VGPRs,
//              Q'[i] = Q[i] * itemUp/itemDown     (as written, Q5: Q'[i] = Q[i] * itemUp)
//   user pass  (user-CSR, data order):  userUp/userDown of u in VGPRs,
//              P[u] = P[u] * userUp/userDown      (reads Q, not Q')
// then Q <- Q'.  Both passes read the start-of-epoch P and Q, exactly as the reference does.
// Since no rating's terms depend on another's, rows are cut into chunks of <= 64 ratings, one
// G-lane group (G = 16 for the default k = 15: 64-byte rows) per chunk, partials of long rows added
// in chunk order by a combine kernel: the epoch is no longer bound by the longest row's chain.
// The partner row of every rating is gathered D ratings ahead into a register ring; the prediction
// dot product is a G-lane DPP (+ permlane) reduction.
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

// Row sums of G lanes (G = 16, 32 or 64): DPP inside each 16-lane row, then the gfx950 permlane
// swaps; every lane of the group ends with the bitwise-identical total.
template <int G>
__device__ __forceinline__ float nmf_group_sum(float x) {
    x = group_sum<16>(x);
    if constexpr (G >= 32) {
        auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
    }
    if constexpr (G >= 64) {
        auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
    }
    return x;
}

// One pass over chunks of rows.  own = the matrix whose rows this pass updates (rows of the CSR),
// partner = the other factor matrix, rows of LD = G * E floats (lane l of a G-lane group owns
// columns l + G x).  Every rating's terms depend only on the start-of-epoch factors, so a row's
// ratings are independent: a row is cut into chunks of at most kNmfChunk ratings, one G-lane group
// per chunk (chunks longest first, so the groups of a wave run equal trip counts), each chunk summed
// in data order.  A single-chunk row writes out[row] = own[row] * up / down (or * up when UPONLY, the
// as-written item rule) directly; the chunks of a longer row write (up, down) partials, which
// nmf_combine_kernel adds in chunk order.  chunk = {row, begin, end, partial slot or -1}.
constexpr int kNmfChunk = 64;

template <int G, int E, int D, bool UPONLY>
__global__ __launch_bounds__(256) void nmf_chunk_kernel(
    int32_t n_chunks, const int4* __restrict__ chunks, const int64_t* __restrict__ rowptr,
    const int32_t* __restrict__ cols, const float* __restrict__ vals, const float* __restrict__ own,
    const float* __restrict__ partner, float* __restrict__ out, float* __restrict__ partial, int32_t k,
    float reg) {
#pragma clang fp contract(off)
    constexpr int LD = G * E, NG = 256 / G;
    const int gl = threadIdx.x & (G - 1);
    const int32_t ci = static_cast<int32_t>(blockIdx.x) * NG + static_cast<int32_t>(threadIdx.x) / G;
    if (ci >= n_chunks) return;
    const int4 c = chunks[ci];
    const int64_t b = rowptr[c.x] + c.y, e = rowptr[c.x] + c.z;
    float p[E], up[E], down[E];
    const float* orow = own + static_cast<int64_t>(c.x) * LD;
#pragma unroll
    for (int x = 0; x < E; ++x) {
        p[x] = orow[gl + G * x];
        up[x] = 0.f;
        down[x] = 0.f;
    }
    auto load = [&](float (&q)[E], bool valid, int32_t col) {
        const float* qr = partner + static_cast<int64_t>(valid ? col : 0) * LD;
#pragma unroll
        for (int x = 0; x < E; ++x) q[x] = valid ? qr[gl + G * x] : 0.f;
    };
    const int32_t n = static_cast<int32_t>(e - b);
    float ring[D][E];
#pragma unroll
    for (int s = 0; s < D; ++s) load(ring[s], s < n, cols[b + s]);  // cols padded by 64
    for (int32_t o = 0; o < n; o += 16) {
        int32_t cn[16];
        float rt[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            cn[j] = cols[b + o + D + j];
            rt[j] = vals[b + o + j];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            constexpr int kD = D;
            const int slot = j % kD;
            if (o + j < n) {
                const float* q = ring[slot];
                float s = 0.f;
#pragma unroll
                for (int x = 0; x < E; ++x) s += p[x] * q[x];
                const float pred = nmf_group_sum<G>(s);       // svd.go:190 (Predict -> Dot)
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    up[x] = up[x] + q[x] * rt[j];              // svd.go:193-197 / 214-218
                    down[x] = down[x] + q[x] * pred;           // svd.go:200-204 / 221-225
                    down[x] = down[x] + p[x] * reg;            // svd.go:206-210 / 227-231
                }
            }
            load(ring[slot], o + j + D < n, cn[j]);
        }
    }
    if (c.w >= 0) {  // one chunk of a longer row: partials for nmf_combine_kernel
        float* w = partial + static_cast<int64_t>(c.w) * 2 * LD;
#pragma unroll
        for (int x = 0; x < E; ++x) {
            w[gl + G * x] = up[x];
            w[LD + gl + G * x] = down[x];
        }
        return;
    }
    float* w = out + static_cast<int64_t>(c.x) * LD;
#pragma unroll
    for (int x = 0; x < E; ++x) {
        // svd.go:236-241 (users, items intended): buffer = up / down; p *= buffer
        // svd.go:243-249 (items as written, Q5):   q *= up (the undivided copy)
        const float buffer = UPONLY ? up[x] : up[x] / down[x];
        w[gl + G * x] = gl + G * x < k ? p[x] * buffer : 0.f;  // padding stays 0 (0/0)
    }
}

// Rows cut into several chunks: partials added in chunk order, then the row update.  One G-lane
// group per row; multi = {row, first partial slot, chunks, -}.
template <int G, int E, bool UPONLY>
__global__ __launch_bounds__(256) void nmf_combine_kernel(int32_t n_multi, const int4* __restrict__ multi,
                                                          const float* __restrict__ own,
                                                          const float* __restrict__ partial,
                                                          float* __restrict__ out, int32_t k) {
#pragma clang fp contract(off)
    constexpr int LD = G * E, NG = 256 / G;
    const int gl = threadIdx.x & (G - 1);
    const int32_t mi = static_cast<int32_t>(blockIdx.x) * NG + static_cast<int32_t>(threadIdx.x) / G;
    if (mi >= n_multi) return;
    const int4 m = multi[mi];
    float up[E], down[E];
#pragma unroll
    for (int x = 0; x < E; ++x) {
        up[x] = 0.f;
        down[x] = 0.f;
    }
    for (int32_t t = 0; t < m.z; ++t) {
        const float* w = partial + static_cast<int64_t>(m.y + t) * 2 * LD;
#pragma unroll
        for (int x = 0; x < E; ++x) {
            up[x] = up[x] + w[gl + G * x];
            down[x] = down[x] + w[LD + gl + G * x];
        }
    }
    const float* orow = own + static_cast<int64_t>(m.x) * LD;
    float* w = out + static_cast<int64_t>(m.x) * LD;
#pragma unroll
    for (int x = 0; x < E; ++x) {
        const float buffer = UPONLY ? up[x] : up[x] / down[x];
        w[gl + G * x] = gl + G * x < k ? orow[gl + G * x] * buffer : 0.f;
    }
}

// The chunk list of one pass (host-built once per fit): chunks longest first; multi-chunk rows.
struct NmfChunks {
    DevBuf<int4> chunks, multi;
    int32_t n_chunks = 0, n_multi = 0, n_partial = 0;
    void build(const std::vector<int64_t>& rowptr, hipStream_t s) {
        std::vector<int4> ch, mu;
        const int32_t n_rows = static_cast<int32_t>(rowptr.size()) - 1;
        int32_t slot = 0;
        for (int32_t r = 0; r < n_rows; ++r) {
            const int64_t d = rowptr[r + 1] - rowptr[r];
            if (d <= kNmfChunk) {  // one chunk (empty rows too: they write 0 / 0 like the reference)
                ch.push_back(make_int4(r, 0, static_cast<int32_t>(d), -1));
                continue;
            }
            const int32_t nc = static_cast<int32_t>((d + kNmfChunk - 1) / kNmfChunk);
            mu.push_back(make_int4(r, slot, nc, 0));
            for (int32_t t = 0; t < nc; ++t)
                ch.push_back(make_int4(r, t * kNmfChunk, static_cast<int32_t>(std::min<int64_t>(d, (t + 1) * kNmfChunk)), slot + t));
            slot += nc;
        }
        std::stable_sort(ch.begin(), ch.end(), [](const int4& a, const int4& b) { return a.z - a.y > b.z - b.y; });
        n_chunks = static_cast<int32_t>(ch.size());
        n_multi = static_cast<int32_t>(mu.size());
        n_partial = slot;
        chunks.alloc(std::max<size_t>(1, ch.size()));
        multi.alloc(std::max<size_t>(1, mu.size()));
        chunks.upload(ch.data(), ch.size(), s);
        multi.upload(mu.data(), mu.size(), s);
    }
};

template <int G, int E, bool UPONLY>
static void nmf_pass(const NmfChunks& c, const DevBuf<int64_t>& row, const DevBuf<int32_t>& col,
                     const DevBuf<float>& val, const float* own, const float* partner, float* out,
                     float* partial, int32_t k, float reg, hipStream_t s) {
    constexpr int NG = 256 / G;
    if (c.n_chunks > 0)
        hipLaunchKernelGGL((nmf_chunk_kernel<G, E, 8, UPONLY>), dim3((c.n_chunks + NG - 1) / NG), dim3(256), 0, s,
                           c.n_chunks, c.chunks.p, row.p, col.p, val.p, own, partner, out, partial, k, reg);
    if (c.n_multi > 0)
        hipLaunchKernelGGL((nmf_combine_kernel<G, E, UPONLY>), dim3((c.n_multi + NG - 1) / NG), dim3(256), 0, s,
                           c.n_multi, c.multi.p, own, partial, out, k);
}

template <int G, int E>
static void nmf_epoch_t(const NmfChunks& uc, const NmfChunks& ic, const DevBuf<int64_t>& urow,
                        const DevBuf<int32_t>& ucol, const DevBuf<float>& uval,
                        const DevBuf<int64_t>& irow, const DevBuf<int32_t>& icol,
                        const DevBuf<float>& ival, float* P, float*& Q, float*& Qn, float* partial,
                        int32_t k, float reg, bool as_written, hipStream_t s) {
    // item pass (start-of-epoch P and Q) -> Qn; then the user pass (start-of-epoch Q) writes P in
    // place: a user row is read only by its own chunks, and a multi-chunk row is written only by the
    // combine kernel after all of them
    if (as_written)
        nmf_pass<G, E, true>(ic, irow, icol, ival, Q, P, Qn, partial, k, reg, s);
    else
        nmf_pass<G, E, false>(ic, irow, icol, ival, Q, P, Qn, partial, k, reg, s);
    nmf_pass<G, E, false>(uc, urow, ucol, uval, P, Q, P, partial, k, reg, s);
    RS_HIP(hipGetLastError());
    std::swap(Q, Qn);
}

}  // namespace rs

extern "C" int rs_nmf_fit(rs_ctx* ctx, const rs_ratings* r, int32_t n_factors, int32_t n_epochs,
                          double reg, int32_t as_written, double* P, double* Q) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        rs::drop_fit_cache(ctx);
        int st = rs::check_ratings(ctx, r);
        if (st != RS_OK) return st;
        if (n_factors < 1 || n_factors > 512)
            return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "n_factors must be in [1, 512]");
        if (n_epochs < 0 || !P || !Q) return rs::set_error(ctx, RS_ERR_INVALID, "bad NMF arguments");
        hipStream_t s = ctx->stream;
        // row layout: G-lane groups x E columns per lane (k = 15, the NMF default: 16 x 1, 64-byte rows)
        const int32_t k = n_factors;
        const int32_t G = k <= 16 ? 16 : k <= 32 ? 32 : 64;
        const int32_t E = k <= 64 ? 1 : k <= 128 ? 2 : k <= 256 ? 4 : 8, ld = G * E;
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
        rs::NmfChunks uc, ic;
        uc.build(ucsr.rowptr, s);
        ic.build(icsr.rowptr, s);
        std::vector<float> hP, hQ;
        rs::pack_rows_f32(P, r->n_users, k, ld, hP);
        rs::pack_rows_f32(Q, r->n_items, k, ld, hQ);
        rs::DevBuf<float> dP(std::max<size_t>(1, hP.size())), dQa(std::max<size_t>(1, hQ.size())),
            dQb(std::max<size_t>(1, hQ.size()));
        rs::DevBuf<float> partial(static_cast<size_t>(std::max({1, uc.n_partial, ic.n_partial})) * 2 * ld);
        dP.upload(hP.data(), hP.size(), s);
        dQa.upload(hQ.data(), hQ.size(), s);
        float* q = dQa.p;
        float* qn = dQb.p;
        const float fr = static_cast<float>(reg);
        const bool aw = as_written != 0;
        RS_HIP(hipStreamSynchronize(s));
        rs::kernel_span_begin(ctx);
        for (int32_t ep = 0; ep < n_epochs; ++ep) {
#define RS_NMF_EPOCH(g, e) rs::nmf_epoch_t<g, e>(uc, ic, urow, ucol, uval, irow, icol, ival, dP.p, q, qn, partial.p, k, fr, aw, s)
            if (G == 16) RS_NMF_EPOCH(16, 1);
            else if (G == 32) RS_NMF_EPOCH(32, 1);
            else if (E == 1) RS_NMF_EPOCH(64, 1);
            else if (E == 2) RS_NMF_EPOCH(64, 2);
            else if (E == 4) RS_NMF_EPOCH(64, 4);
            else RS_NMF_EPOCH(64, 8);
#undef RS_NMF_EPOCH
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
