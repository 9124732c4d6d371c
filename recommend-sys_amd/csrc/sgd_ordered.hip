// sgd_ordered.hip -- the ORDERED SVD epoch (RS_SGD_ORDERED, north_star's "factor values within 1e-5 of
// the reference after one epoch"): core/svd.go:92-130 in the train-set order with the reference's update
// order and aliasing (p_u first, then q_i with the NEW p_u, Q1), every rating after the previous one.
//
// The serial dependence of that loop is narrower than it looks: rating t needs the rows rating t - d
// wrote only when it shares the user or the item, and the only state EVERY rating shares is the scalar
// GlobalBias chain gb <- gb - lr ((gb + b_u + b_i + p.q) - r) (svd.go:102-106).  So one wave walks the
// ratings with
//   * the rows of rating t + D loaded while rating t computes (a D-deep register ring), ids read by
//     scalar loads two blocks of D ahead;
//   * a prefetched row that one of the last D ratings rewrote after its load was issued loaded again
//     (a uniform branch that rarely runs);
//   * the biases folded into the rows -- P row [p_0 .. p_{k-1}, b_u, 1], Q row [q_0 .. q_{k-1}, 1, b_i]
//     -- so p.q over all columns is the prediction minus gb, and the one update p <- a p - c q,
//     q <- a q - c p_new also performs svd.go:108-112 (the constant columns are held at 1);
//   * gb, the prediction and diff in float64 (the chain), the row arithmetic in float32.
// The result is the sequential epoch exactly (no reordering), within float32 rounding of the fp64
// restatement (tests/test_svd_gpu.py::test_ordered_matches_oracle, 1e-5).  One rating costs about 85
// instructions, most of them on its own dependency chain (DPP reduction, the f64 chain, the updates):
// 222 ms per ML-1M epoch (4.5e6 updates/s) against 515 ms for round 2's 16-lane group.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <type_traits>

#include "common.hpp"
#include "sgd_plan.hpp"

namespace rs {

namespace {

// sum over the wave, valid in lane 63 (DPP row sums, then row_bcast:15 / row_bcast:31)
__device__ __forceinline__ float ordered_wave_sum(float x) {
    x = group_sum<16>(x);
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xA, 0xF, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xC, 0xF, false));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

}  // namespace

// One wave; lane l holds the column pairs (128 h + 2 l, 128 h + 2 l + 1), h < H, of a row: one 8-byte
// load / store and one packed-math op per pair.  Rows are ld floats (ld even, ld >= k + 2,
// ld <= 128 H); the id and rating arrays hold whole blocks of D entries (padded).  All epochs in one
// launch.
//
// Rating t's rows are loaded when rating t - D ends (ring slot t mod D).  If one of the ratings in
// between wrote the same user or item row (a rare, uniform branch: about one rating in seventy on the
// ML-1M shape), the row is loaded again.  The loop body is D ratings with every slot issuing the same
// loads and stores (an empty slot's go to out-of-range offsets), so the compiler's vmcnt waits keep the
// whole ring in flight.  Measured alternatives (DESIGN.md K1 ORDERED): a float4-per-lane layout with the
// rewritten rows forwarded from registers (277 ms per ML-1M epoch), blocks of 4 ratings run as one
// group with interleaved reductions (288-309 ms), against 222 ms for this loop.
template <int H, int D>
__global__ __launch_bounds__(64) void svd_ordered_wave_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, const float* __restrict__ ratings,
    int64_t nnz, int64_t n_blocks /* per epoch, of D ratings */, float* P, int32_t p_bytes, float* Q,
    int32_t q_bytes, int32_t ld, int32_t kf, double* gb_io, int32_t epochs, float lr, float reg) {
#pragma clang fp contract(fast)
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int lane = static_cast<int>(threadIdx.x);
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(P, 0, p_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    // per pair: byte offset inside a row (kOutOfRange past it: 2^31 lies past every buffer) and the update's
    // multipliers, which hold the constant columns at 1 (P: k + 1, Q: k): x <- x * am - y * (c * cm)
    int32_t coff[H];
    f2 amp[H], cmp[H], amq[H], cmq[H];
    const float a = 1.f - lr * reg;
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int32_t c = 128 * h + 2 * lane;
        coff[h] = c < ld ? 4 * c : kOutOfRange;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const bool kp = c + e == kf + 1, kq = c + e == kf;
            amp[h][e] = kp ? 1.f : a;
            cmp[h][e] = kp ? 0.f : 1.f;
            amq[h][e] = kq ? 1.f : a;
            cmq[h][e] = kq ? 0.f : 1.f;
        }
    }
    const double lrd = lr;
    double gb = gb_io[0];
    const int64_t total = n_blocks * static_cast<int64_t>(epochs);
    auto rl = [](int32_t x, int j) { return __builtin_amdgcn_readlane(x, j); };
    // byte offset of pair h of `row`: no branch on the row (a uniform condition would become a branch
    // around the memory operation and the vmcnt waits would lose count); row -1 and the pairs past the
    // row wrap to offsets past the buffer's end, which load 0 and drop the store
    auto off = [&](int32_t row, int h) {
        return static_cast<int32_t>(static_cast<uint32_t>(row) * static_cast<uint32_t>(ld * 4) + static_cast<uint32_t>(coff[h]));
    };
    auto load_row = [&](__amdgpu_buffer_rsrc_t r, int32_t row, f2 (&dst)[H]) {
#pragma unroll
        for (int h = 0; h < H; ++h)
            dst[h] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, off(row, h), 0, kSgdAux));
    };
    auto store_row = [&](__amdgpu_buffer_rsrc_t r, int32_t row, const f2 (&src)[H]) {
#pragma unroll
        for (int h = 0; h < H; ++h)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) uint32_t, src[h]),
                                                  r, off(row, h), 0, 0);
    };

    auto dot = [&](const f2 (&p)[H], const f2 (&q)[H]) {  // p.q over all columns: the prediction minus gb
        f2 acc = p[0] * q[0];
#pragma unroll
        for (int h = 1; h < H; ++h) acc = __builtin_elementwise_fma(p[h], q[h], acc);
        return acc.x + acc.y;
    };
    // svd.go:114-128: p <- p - (q diff + p reg) lr, then q with the NEW p (Q1); c = lr diff
    auto update = [&](f2 (&p)[H], f2 (&q)[H], float c) {
        const f2 cc = {c, c};
#pragma unroll
        for (int h = 0; h < H; ++h) {
            p[h] = __builtin_elementwise_fma(-q[h], cc * cmp[h], p[h] * amp[h]);
            q[h] = __builtin_elementwise_fma(-p[h], cc * cmq[h], q[h] * amq[h]);
        }
    };
    // ids of block B, lane j < D holding rating j of the block (-1: none, also for B < 0 or past the
    // last epoch); rating index base (B mod n_blocks) D.  Scalar loads (lgkmcnt: the ids never stall the
    // row ring's vmcnt), then spread over the lanes; the arrays are padded to whole blocks.
    auto ids = [&](int64_t B, int32_t& u, int32_t& i, float& r) {
        const int64_t Bc = B < 0 ? 0 : B;
        const int64_t base = (Bc % n_blocks) * D;
        const int32_t ok_n = (B >= 0 && B < total) ? static_cast<int32_t>(min(static_cast<int64_t>(D), nnz - base)) : 0;
        u = -1;
        i = -1;
        r = 0.f;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int32_t uj = users[base + j], ij = items[base + j];
            const float rj = ratings[base + j];
            u = (lane == j && j < ok_n) ? uj : u;
            i = (lane == j && j < ok_n) ? ij : i;
            r = (lane == j && j < ok_n) ? rj : r;
        }
    };
    int32_t cu, ci, nu, ni;  // this block's and the next block's ids (lane j: slot j)
    float cr, nr;
    int32_t ou = -1, oi = -1;  // lane s < D: ids of the rating slot s last processed
    f2 lp[D][H], lq[D][H];     // the ring: rows of the next D ratings
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
        for (int h = 0; h < H; ++h) lp[j][h] = lq[j][h] = f2{0.f, 0.f};
    ids(-1, cu, ci, cr);
    ids(0, nu, ni, nr);
    // The loop starts at an empty block -1 (nothing updated, its stores dropped) whose slots issue block
    // 0's loads in the loop's own order.
    for (int64_t B = -1; B < total; ++B) {
        int32_t fu, fi;
        float fr;
        ids(B + 2, fu, fi, fr);  // two blocks ahead
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int32_t u = rl(cu, j), i = rl(ci, j);
            f2 p[H], q[H];
#pragma unroll
            for (int h = 0; h < H; ++h)  // real copies: the refill below lands in the ring's own registers
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    asm volatile("v_mov_b32 %0, %1" : "=v"(p[h][e]) : "v"(lp[j][h][e]));
                    asm volatile("v_mov_b32 %0, %1" : "=v"(q[h][e]) : "v"(lq[j][h][e]));
                }
            // a row one of the last D ratings rewrote after this load was issued: load it again
            const bool su = __ballot(lane < D && ou == u) != 0, si = __ballot(lane < D && oi == i) != 0;
            if (u >= 0 && (su || si)) {  // (a load after this lane's own store of the address sees it)
                if (su) load_row(rp, u, p);
                if (si) load_row(rq, i, q);
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), as the compiler's wait tracking knows
            }
            const float sp = ordered_wave_sum(dot(p, q));
            const float rt = __int_as_float(rl(__float_as_int(cr), j));
            const double diff = gb + (static_cast<double>(sp) - static_cast<double>(rt));  // svd.go:102
            gb = u >= 0 ? gb - lrd * diff : gb;                                             // svd.go:105-106
            update(p, q, static_cast<float>(lrd * diff));
            store_row(rp, u, p);  // (an empty slot's stores go to out-of-range offsets and are dropped)
            store_row(rq, i, q);
            ou = lane == j ? u : ou;
            oi = lane == j ? i : oi;
            load_row(rp, rl(nu, j), lp[j]);  // rating D ahead into the freed slot
            load_row(rq, rl(ni, j), lq[j]);
        }
        cu = nu;
        ci = ni;
        cr = nr;
        nu = fu;
        ni = fi;
        nr = fr;
    }
    if (lane == 0) gb_io[0] = gb;
}

// ORDERED epochs on the folded layout (rows of ld floats: P [p, b_u, 1], Q [q, 1, b_i]); users / items /
// ratings in train-set order, allocated for ordered_padded(nnz) entries.
int64_t ordered_padded(int64_t nnz) { return (nnz + 7) / 8 * 8 + 16; }

void ordered_epochs(const int32_t* users, const int32_t* items, const float* ratings, int64_t nnz, float* P,
                    int64_t p_floats, float* Q, int64_t q_floats, int32_t ld, int32_t kf, double* gb,
                    int32_t epochs, float lr, float reg, hipStream_t s) {
    if (nnz == 0 || epochs <= 0) return;
    if (p_floats * 4 >= (int64_t{1} << 31) || q_floats * 4 >= (int64_t{1} << 31))
        throw std::invalid_argument("ORDERED mode: factor matrices of 2 GiB or more");
    const int32_t pb = static_cast<int32_t>(p_floats * 4), qb = static_cast<int32_t>(q_floats * 4);
    // ring depth: every slot keeps 4 H memory operations in flight, the vmcnt counter holds 63
    auto go = [&](auto h_c, auto d_c) {
        constexpr int H = decltype(h_c)::value, D = decltype(d_c)::value;
        hipLaunchKernelGGL((svd_ordered_wave_kernel<H, D>), dim3(1), dim3(64), 0, s, users, items, ratings, nnz,
                           (nnz + D - 1) / D, P, pb, Q, qb, ld, kf, gb, epochs, lr, reg);
    };
    using std::integral_constant;
    if (ld <= 128) go(integral_constant<int, 1>{}, integral_constant<int, 14>{});
    else if (ld <= 256) go(integral_constant<int, 2>{}, integral_constant<int, 7>{});
    else go(integral_constant<int, 4>{}, integral_constant<int, 3>{});
    RS_HIP(hipGetLastError());
}

}  // namespace rs
