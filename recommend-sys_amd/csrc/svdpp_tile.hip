// svdpp_tile.hip -- K2 on the tile schedule: the SVD++ epoch of core/svd.go:316-427 (FAST) with the
// users' rows in LDS and the item rows combined per (item, tile) run, gfx950.  The schedule is K1's
// (sgd_tile.hip: user tiles, per-item runs dealt to 16 waves, q_i in registers along a run, one
// memory-side integer atomic per run and row line); this file adds the implicit-feedback state.
//
// The lazy y update of the user-major kernel (svdpp.hip) keeps, per user row, the scale A = a^m and
// the offset C of the affine map every y_j of N(u) goes through (y_j <- A y_j - C at the row end), and
// the implicit factor e = (A S0 - n C) / sqrt(n) with S0 = sum_j y_j.  In a tile the ratings of a user
// are reached by several waves in run order, so that state is made order-free:
//   * W = S0 / sqrt(n) - sqrt(n) C / A, so e = A W, and a rating that is the user's m-th changes W by
//     -c q_i(new) a^-(m+1) (c = lr * diff) -- an integer LDS atomic add, whatever the order;
//   * m is the rating's rank among its user's ratings in the schedule (host-assigned: its progress
//     through its wave's stream), so A = a^m needs no counter.
// After the runs, C_u = a^n (W_init - W) / sqrt(n), and every y_j gets the sum over the tile's users
// of (a^n - 1) y_j - C_u in one integer atomic per (item, tile) run (svd.go:399-422, deferred to the
// tile's end; with one workgroup of one wave this is or_svdpp_fit_tiles exactly).
//
// LDS per user: P row [p, b_u, 1], W row, W_init row (then C), as int32 2^-24 fixed point (C as fp32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "sgd_plan.hpp"
#include "wave.hpp"

namespace rs {

namespace {

__device__ __forceinline__ float wave_sum_pp(float x) {  // the K1 row-broadcast sum ending in lane 63
    x = group_sum<16>(x);
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xA, 0xF, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xC, 0xF, false));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

__device__ __forceinline__ int32_t cvt_rpi_pp(float x) {
    int32_t r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

}  // namespace

template <int E, int NW, int RQ>
__global__ __launch_bounds__(NW * 64) void svdpp_epoch_tile_kernel(
    const int4* __restrict__ tiles, int32_t n_tiles, const int2* __restrict__ tile_users,
    const int32_t* __restrict__ streams, const int2* __restrict__ runs, const int2* __restrict__ recs,
    float* __restrict__ P, int32_t* Q, int32_t q_bytes, int32_t* Y, int32_t y_bytes,
    const double* __restrict__ gb_in, double* __restrict__ gb_partial, float lr, float reg, float la,
    int32_t kf, int32_t ldm) {
#pragma clang fp contract(fast)
    constexpr int LD = 64 * E, NT = NW * 64;
    static_assert(2 * E * RQ <= 60, "ring loads and atomics must fit the 63-op vmcnt");
    extern __shared__ __align__(16) int32_t lds[];
    const int tid = static_cast<int>(threadIdx.x), lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(Y, 0, y_bytes, 0x00020000);
    const double gb0 = gb_in[0];
    const float a = 1.f - lr * reg, am1 = -lr * reg;  // la = log2(a), from the host in double
    int32_t qoff[E], yoff[E];
    bool qone[E], pone[E], fac[E];
#pragma unroll
    for (int x = 0; x < E; ++x) {
        const int32_t c = lane + 64 * x;
        qoff[x] = c < kf ? 4 * c : (c == kf + 1 ? 4 * kf : -1);
        yoff[x] = c < kf ? 4 * c : -1;
        qone[x] = c == kf;
        pone[x] = c == kf + 1;
        fac[x] = c < kf;
    }
    auto addr = [&](int32_t row, int32_t off) { return (row >= 0 && off >= 0) ? row + off : kOutOfRange; };
    double contrib = 0.0;

    for (int32_t t = static_cast<int32_t>(blockIdx.x); t < n_tiles; t += static_cast<int32_t>(gridDim.x)) {
        const int4 tm = tiles[t];  // {first user entry, users, first run, first record}
        const int32_t nu = tm.y;
        const int32_t* sp = streams + static_cast<int64_t>(t) * (NW + 1);
        const int32_t n_runs = sp[NW];
        const int2* tr = runs + tm.z;
        const int32_t n_rec = tr[n_runs].y;
        int32_t* Pl = lds;                 // nu x LD
        int32_t* Wl = Pl + nu * LD;        // nu x LD
        int32_t* Vl = Wl + nu * LD;        // nu x LD: W_init, then C (fp32 bits)
        float* Sl = reinterpret_cast<float*>(Vl + nu * LD);  // nu: 1/sqrt(n), then a^n - 1
        int2* Rl = reinterpret_cast<int2*>(Sl + ((nu + 1) & ~1));
        int2* Ul = Rl + n_rec;
        for (int32_t x = tid; x < nu * LD; x += NT) {
            const int32_t ul = x / LD, c = x - ul * LD;
            int32_t v = 0;
            if (c <= kf) v = __float2int_rn(P[static_cast<int64_t>(tile_users[tm.x + ul].x) * ldm + c] * kFx);
            else if (c == kf + 1) v = 1 << 24;
            Pl[x] = v;
            Vl[x] = 0;
        }
        for (int32_t x = tid; x < nu; x += NT) Sl[x] = rsqrtf(static_cast<float>(tile_users[tm.x + x].y));
        for (int32_t x = tid; x < n_rec; x += NT) Rl[x] = recs[tm.w + x];
        for (int32_t x = tid; x <= n_runs; x += NT) Ul[x] = tr[x];
        __syncthreads();

        const int32_t r0 = sp[w], r1 = sp[w + 1];
        // S0 pass: W_init[u] = sum over N(u) of y_j / sqrt(n_u) (integer LDS adds: order-free)
        for (int32_t r = r0; r < r1; ++r) {
            const int2 h = Ul[r], h1 = Ul[r + 1];
            const int32_t row = __builtin_amdgcn_readfirstlane(h.x) * (ldm * 4);
            float y[E];
#pragma unroll
            for (int x = 0; x < E; ++x)
                y[x] = static_cast<float>(static_cast<int32_t>(
                    __builtin_amdgcn_raw_buffer_load_b32(ry, addr(row, yoff[x]), 0, kSgdAux)));
            const int32_t jb = __builtin_amdgcn_readfirstlane(h.y), je = __builtin_amdgcn_readfirstlane(h1.y);
            for (int32_t j = jb; j < je; ++j) {
                const int32_t ul = __builtin_amdgcn_readfirstlane(Rl[j].x) & 0xffff;
                const float is = Sl[ul];
#pragma unroll
                for (int x = 0; x < E; ++x)
                    if (fac[x])
                        __hip_atomic_fetch_add(Vl + ul * LD + lane + 64 * x, cvt_rpi_pp(y[x] * is), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        for (int32_t x = tid; x < nu * LD; x += NT) Wl[x] = Vl[x];
        __syncthreads();

        // main pass: the K1 run loop with the implicit factor e = a^m W
        auto load_q = [&](int32_t (&q)[E], int32_t item) {
            const int32_t row = item >= 0 ? item * (ldm * 4) : -1;
#pragma unroll
            for (int x = 0; x < E; ++x)
                q[x] = static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(rq, addr(row, qoff[x]), 0, kSgdAux));
        };
        auto item_of = [&](int32_t r) -> int32_t { return r < r1 ? __builtin_amdgcn_readfirstlane(Ul[r].x) : -1; };
        int32_t ring[RQ][E];
#pragma unroll
        for (int s = 0; s < RQ; ++s) {
            load_q(ring[s], item_of(r0 + s));
#pragma unroll
            for (int x = 0; x < E; ++x) {
                int32_t z;
                asm volatile("v_mov_b32 %0, 0" : "=v"(z));
                __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(z, rq, kOutOfRange + lane * 4 + 256 * x, 0, 0);
            }
        }
        double gb = gb0;
        const float klr = lr * kFxInv * kFxInv;
        for (int32_t r = r0; r < r1; r += RQ) {
#pragma unroll
            for (int s = 0; s < RQ; ++s) {
                const int32_t rr = r + s;
                const bool live = rr < r1;
                int32_t q0[E];
                float q[E];
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    asm volatile("v_mov_b32 %0, %1" : "=v"(q0[x]) : "v"(ring[s][x]));
                    q[x] = qone[x] ? kFx : static_cast<float>(q0[x]);
                }
                const int2 h = Ul[min(rr, n_runs)];
                const int32_t item = __builtin_amdgcn_readfirstlane(h.x);
                const int32_t jb = live ? __builtin_amdgcn_readfirstlane(h.y) : 0;
                const int32_t je = live ? __builtin_amdgcn_readfirstlane(Ul[min(rr + 1, n_runs)].y) : 0;
                load_q(ring[s], item_of(rr + RQ));
                const float gbf = static_cast<float>(gb);
                float cs = 0.f;
                for (int32_t j = jb; j < je; ++j) {
                    const int2 rec = Rl[j];
                    const int32_t ux = __builtin_amdgcn_readfirstlane(rec.x);
                    const int32_t ul = ux & 0xffff, m = ux >> 16;
                    const float rt = __int_as_float(__builtin_amdgcn_readfirstlane(rec.y));
                    const float Ab = exp2f(la * static_cast<float>(m));
                    const float Ainv = exp2f(-la * static_cast<float>(m + 1));
                    int32_t* prow = Pl + ul * LD + lane;
                    int32_t* wrow = Wl + ul * LD + lane;
                    float pu[E], e[E];
#pragma unroll
                    for (int x = 0; x < E; ++x) {
                        pu[x] = static_cast<float>(prow[64 * x]);
                        e[x] = Ab * static_cast<float>(wrow[64 * x]);  // 0 past the factors
                    }
                    float sd = 0.f;
#pragma unroll
                    for (int x = 0; x < E; ++x) sd = __builtin_fmaf(pu[x] + e[x], q[x], sd);
                    sd = wave_sum_pp(sd);
                    // svd.go:381-398: diff = pred - r; c = lr diff; p <- a p - c q; q <- a q - c (p_new + e)
                    const float c = __builtin_fmaf(sd, klr, lr * ((gbf - cs) - rt));
                    cs += c;
#pragma unroll
                    for (int x = 0; x < E; ++x) {
                        const float d = pone[x] ? 0.f : __builtin_fmaf(q[x], -c, pu[x] * am1);
                        const float qn = qone[x] ? kFx : __builtin_fmaf(pu[x] + d + e[x], -c, q[x] * a);
                        q[x] = qn;
                        __hip_atomic_fetch_add(prow + 64 * x, cvt_rpi_pp(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (fac[x])  // W -= c q_new a^-(m+1)
                            __hip_atomic_fetch_add(wrow + 64 * x, cvt_rpi_pp(-c * Ainv * qn), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                gb -= static_cast<double>(cs);
                const int32_t row = live ? item * (ldm * 4) : -1;
#pragma unroll
                for (int x = 0; x < E; ++x)
                    __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(cvt_rpi_pp(q[x]) - q0[x], rq, addr(row, qoff[x]), 0, 0);
            }
        }
        const int32_t s_begin = r0 < r1 ? __builtin_amdgcn_readfirstlane(Ul[r0].y) : 0;
        const int32_t s_end = r0 < r1 ? __builtin_amdgcn_readfirstlane(Ul[r1].y) : 0;
        contrib += static_cast<double>(s_end - s_begin) * (gb - gb0);
        __syncthreads();
        // users: P back to HBM; C_u = a^n (W_init - W) / sqrt(n) (fp32 bits into Vl); a^n - 1 into Sl
        for (int32_t x = tid; x < nu * LD; x += NT) {
            const int32_t ul = x / LD, c = x - ul * LD;
            const int32_t n = tile_users[tm.x + ul].y;
            const float An = exp2f(la * static_cast<float>(n));
            if (c <= kf) P[static_cast<int64_t>(tile_users[tm.x + ul].x) * ldm + c] = fx_to_f(static_cast<uint32_t>(Pl[x]));
            const float Cv = c < kf ? An * static_cast<float>(Vl[x] - Wl[x]) * Sl[ul] : 0.f;  // 2^-24 units
            Vl[x] = __float_as_int(Cv);
        }
        __syncthreads();
        for (int32_t x = tid; x < nu; x += NT) Sl[x] = exp2f(la * static_cast<float>(tile_users[tm.x + x].y)) - 1.f;
        __syncthreads();
        // Y pass: y_j += sum over the run's users of (a^n - 1) y_j - C_u, one atomic per (item, tile)
        for (int32_t r = r0; r < r1; ++r) {
            const int2 h = Ul[r], h1 = Ul[r + 1];
            const int32_t row = __builtin_amdgcn_readfirstlane(h.x) * (ldm * 4);
            int32_t y0[E];
#pragma unroll
            for (int x = 0; x < E; ++x)
                y0[x] = static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(ry, addr(row, yoff[x]), 0, kSgdAux));
            float sa = 0.f, sc[E];
#pragma unroll
            for (int x = 0; x < E; ++x) sc[x] = 0.f;
            const int32_t jb = __builtin_amdgcn_readfirstlane(h.y), je = __builtin_amdgcn_readfirstlane(h1.y);
            for (int32_t j = jb; j < je; ++j) {
                const int32_t ul = __builtin_amdgcn_readfirstlane(Rl[j].x) & 0xffff;
                sa += Sl[ul];
#pragma unroll
                for (int x = 0; x < E; ++x) sc[x] += __int_as_float(Vl[ul * LD + lane + 64 * x]);
            }
#pragma unroll
            for (int x = 0; x < E; ++x)
                __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(
                    cvt_rpi_pp(__builtin_fmaf(sa, static_cast<float>(y0[x]), -sc[x])), ry, addr(row, yoff[x]), 0, 0);
        }
        __syncthreads();  // the next tile's staging overwrites the LDS
    }
    if (lane == 0) gb_partial[static_cast<int64_t>(blockIdx.x) * NW + w] = contrib;
}

namespace {

template <int E, int NW>
void pp_tile_launch_e(const rs_svd_plan& sh, int32_t* Q, int32_t q_bytes, int32_t* Y, int32_t y_bytes, float* P,
                      const double* gb, double* partial, float lr, float reg, int32_t kf, int32_t ldm, hipStream_t s) {
    auto kern = svdpp_epoch_tile_kernel<E, NW, 2>;
    static bool attr = false;
    if (!attr) {
        RS_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   static_cast<int>(160 * 1024 - 512)));
        attr = true;
    }
    const float la = static_cast<float>(std::log2(1.0 - static_cast<double>(lr) * static_cast<double>(reg)));
    hipLaunchKernelGGL(kern, dim3(sh.tile_grid), dim3(NW * 64), sh.tile_lds, s, sh.t_tiles.p, sh.n_tiles, sh.t_users.p,
                       sh.t_streams.p, sh.t_runs.p, sh.t_recs.p, P, Q, q_bytes, Y, y_bytes, gb, partial, lr, reg, la,
                       kf, ldm);
}

}  // namespace

int32_t pp_tile_user_lds(int32_t k) {
    const int32_t LD = 64 * ((k + 2 + 63) / 64);
    return 3 * LD + 2;  // + 1/sqrt(n) and the alignment pad of the records
}

void pp_tile_launch(const rs_svd_plan& sh, int32_t* Q, int32_t q_bytes, int32_t* Y, int32_t y_bytes, float* P,
                    const double* gb, double* partial, float lr, float reg, int32_t kf, int32_t ldm, hipStream_t s) {
    if (sh.n_tiles == 0) {
        RS_HIP(hipMemsetAsync(partial, 0, static_cast<size_t>(sh.tile_grid) * sh.tile_waves * sizeof(double), s));
        return;
    }
    auto launch = [&](auto e_tag) {
        constexpr int E = decltype(e_tag)::value;
        switch (sh.tile_waves) {
            case 1: pp_tile_launch_e<E, 1>(sh, Q, q_bytes, Y, y_bytes, P, gb, partial, lr, reg, kf, ldm, s); break;
            case 4: pp_tile_launch_e<E, 4>(sh, Q, q_bytes, Y, y_bytes, P, gb, partial, lr, reg, kf, ldm, s); break;
            case 8: pp_tile_launch_e<E, 8>(sh, Q, q_bytes, Y, y_bytes, P, gb, partial, lr, reg, kf, ldm, s); break;
            default: pp_tile_launch_e<E, 16>(sh, Q, q_bytes, Y, y_bytes, P, gb, partial, lr, reg, kf, ldm, s); break;
        }
    };
    switch ((kf + 2 + 63) / 64) {
        case 1: launch(std::integral_constant<int, 1>{}); break;
        case 2: launch(std::integral_constant<int, 2>{}); break;
        case 3: launch(std::integral_constant<int, 3>{}); break;
        case 4: launch(std::integral_constant<int, 4>{}); break;
        default: throw std::invalid_argument("SVD++ tile schedule: n_factors <= 254");
    }
    RS_HIP(hipGetLastError());
}

}  // namespace rs
