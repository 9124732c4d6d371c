// svdpp_tile.hip -- K2 on K1's user tiles (round 5): the SVD++ FAST epoch (reference core/svd.go:316-427) with
// the users of a tile in LDS and the item rows combined per (item, tile) run, gfx950.
//
// The user-major kernel (svdpp.hip) issues one memory-side atomic row per rating for q_i and one per (u, j) for
// y_j: 17M line requests per ML-1M epoch at k = 128, which bound it at 0.23 of HBM.  Here:
//
//   * S pass (pp_tile_sum_kernel): S_u = sum_{j in N(u)} y_j from the epoch-start Y, one wave per user.  Y is
//     read-only during the epoch, so every user's implicit sum is S_u scaled by its own lazy state.
//   * Tile pass (svdpp_tile_kernel): a tile's users hold three LDS rows -- p_u (int32 fixed point, as K1), S_u
//     (fp32) and C~_u (int32 fixed point) -- and a count m_u.  A run (one item's ratings by the tile's users)
//     loads q_i once, trains its ratings with q_i in registers and adds its delta with one atomic row (K1).  A
//     rating of user u is the reference's update with the lazy y state of svd.go:399-422: after m of the user's
//     ratings the scale is A = a^m (a = 1 - lr reg) and the offset C = A C~, C~ = sum_s cy_s q_s a^-(s+1)
//     (cy = lr diff / sqrt n), so e = A (S_u - n C~_u) / sqrt n, and C~_u takes cy q_new a^-(m+1) -- an add,
//     so the waves of a tile share it through LDS atomics like p_u.
//   * Map pass (same kernel, after the tile's ratings): every user u of the tile moves each y_j of N(u) by the
//     affine map y <- a^n y - a^n C~_u (n = |N(u)|: all of u's ratings are in the tile).  A run composes its
//     users' maps in order into one (A, B) per (item, tile) and stores it (plain stores, no atomics).
//   * Y pass (pp_tile_ymap_kernel): each item applies its runs' maps in run order (tile order).
//
// So per epoch the memory side sees one q_i atomic row per run (as K1) instead of one per rating plus one per
// (u, j), and the y traffic is the S pass's reads plus one map row per run.  Within an epoch a user reads the
// epoch-start y_j (the user-major kernel reads them at its row start, as concurrent users decay them); the
// visit order is K1's (tile by tile, a tile's runs in their dealt order, a run's ratings in user order).  With
// one workgroup of one wave the epoch is exactly tests/test_svdpp_tile_gpu.py's restatement of that order.
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
namespace {

// S_u = sum_{j in N(u)} y_j over the first kf columns (rows of LD floats), one wave per user, 8 rows in flight
template <int E>
__global__ __launch_bounds__(256) void pp_tile_sum_kernel(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ items,
                                                          int32_t n_users, const float* __restrict__ Y,
                                                          float* __restrict__ S, int32_t kf) {
    constexpr int LD = 64 * E;
    const int lane = threadIdx.x & 63;
    const int32_t u = static_cast<int32_t>(blockIdx.x) * 4 + static_cast<int32_t>(threadIdx.x >> 6);
    if (u >= n_users) return;
    const int64_t b = rowptr[u], e = rowptr[u + 1];
    float acc[E];
#pragma unroll
    for (int x = 0; x < E; ++x) acc[x] = 0.f;
    for (int64_t t = b; t < e; t += 8) {
        float v[8][E];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int32_t it = t + j < e ? items[t + j] : -1;
#pragma unroll
            for (int x = 0; x < E; ++x) {
                const int32_t c = lane + 64 * x;
                v[j][x] = (it >= 0 && c < kf) ? Y[static_cast<int64_t>(it) * LD + c] : 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int x = 0; x < E; ++x) acc[x] += v[j][x];
    }
#pragma unroll
    for (int x = 0; x < E; ++x) S[static_cast<int64_t>(u) * LD + lane + 64 * x] = acc[x];
}

// The tile pass.  LDS: per user LU = 3 LD ints (p fixed point, S fp32 bits, C~ fixed point), then per user m_u,
// n_u, 1 / sqrt(n_u); the records; the run headers.  Runs dealt to the waves on the host (streams, CH = 0).
template <int E, int NW, int RQ>
__global__ __launch_bounds__(NW * 64) void svdpp_tile_kernel(
    const int4* __restrict__ tiles, int32_t n_tiles, const int2* __restrict__ tile_users,
    const int32_t* __restrict__ streams, const int2* __restrict__ runs, const int2* __restrict__ recs,
    const int64_t* __restrict__ rowptr, float* __restrict__ P, int32_t* Q, int32_t q_bytes,
    const float* __restrict__ S, float* __restrict__ maps, const double* __restrict__ gb_in,
    double* __restrict__ gb_partial, float lr, float reg, float fx, int32_t kf, float log2a) {
#pragma clang fp contract(fast)
    constexpr int LD = 64 * E, NT = NW * 64, LU = 3 * LD;
    static_assert(2 * E * RQ <= 60, "ring loads and atomics must fit the 63-op vmcnt");
    typedef float f2 __attribute__((ext_vector_type(2)));
    extern __shared__ __align__(16) int32_t lds[];
    const int tid = static_cast<int>(threadIdx.x), lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    const double gb0 = gb_in[0];
    const float a = 1.f - lr * reg, am1 = -lr * reg, fx_inv = 1.f / fx;
    int32_t qoff[E];
    bool qone[E], pone[E], pfac[E];
#pragma unroll
    for (int x = 0; x < E; ++x) {
        const int32_t c = lane + 64 * x;
        qoff[x] = c < kf ? 4 * c : (c == kf + 1 ? 4 * kf : -1);
        qone[x] = c == kf;      // Q's constant 1 (partner of b_u)
        pone[x] = c == kf + 1;  // P's constant 1 (partner of b_i)
        pfac[x] = c < kf;
    }
    auto qaddr = [&](int32_t row, int x) { return (row >= 0 && qoff[x] >= 0) ? row + qoff[x] : kOutOfRange; };
    double contrib = 0.0;

    for (int32_t t = static_cast<int32_t>(blockIdx.x); t < n_tiles; t += static_cast<int32_t>(gridDim.x)) {
        const int4 tm = tiles[t];  // {first user entry, entries, first run, first record}
        const int32_t nu = tm.y;
        const int32_t* sp = streams + static_cast<int64_t>(t) * (NW + 1);
        const int32_t n_runs = sp[NW];
        const int2* tr = runs + tm.z;
        const int32_t n_rec = tr[n_runs].y;
        int32_t* Ul = lds;
        int32_t* Ml = Ul + nu * LU;
        int32_t* Nl = Ml + nu;
        float* Rs = reinterpret_cast<float*>(Nl + nu);
        int2* Rl = reinterpret_cast<int2*>(Rs + nu + (nu & 1));  // 8-byte aligned (3 nu ints + pad)
        int2* Hl = Rl + n_rec;
        for (int32_t x = tid; x < nu * LU; x += NT) {
            const int32_t ul = x / LU, cc = x - ul * LU;
            const int64_t g = static_cast<int64_t>(tile_users[tm.x + ul].x) * LD;
            int32_t v = 0;
            if (cc < LD) {
                if (cc <= kf) v = __float2int_rn(P[g + cc] * fx);
                else if (cc == kf + 1) v = static_cast<int32_t>(fx);
            } else if (cc < 2 * LD) {
                const int32_t c = cc - LD;
                v = __float_as_int(c < kf ? S[g + c] : 0.f);
            }
            Ul[x] = v;
        }
        for (int32_t x = tid; x < nu; x += NT) {
            const int32_t u = tile_users[tm.x + x].x;
            const int32_t n = static_cast<int32_t>(rowptr[u + 1] - rowptr[u]);
            Ml[x] = 0;
            Nl[x] = n;
            Rs[x] = 1.f / sqrtf(static_cast<float>(n));
        }
        for (int32_t x = tid; x < n_rec; x += NT) Rl[x] = recs[tm.w + x];
        for (int32_t x = tid; x <= n_runs; x += NT) Hl[x] = tr[x];
        __syncthreads();

        const int32_t r0 = sp[w], r1 = sp[w + 1];
        auto item_of = [&](int32_t r) -> int32_t { return r < r1 ? __builtin_amdgcn_readfirstlane(Hl[r].x) : -1; };
        auto load_q = [&](int32_t (&q)[E], int32_t item) {
            const int32_t row = item >= 0 ? item * (LD * 4) : -1;
#pragma unroll
            for (int x = 0; x < E; ++x)
                q[x] = static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(rq, qaddr(row, x), 0, kSgdAux));
        };
        int32_t ring[RQ][E];
#pragma unroll
        for (int s = 0; s < RQ; ++s) load_q(ring[s], item_of(r0 + s));
        double gb = gb0;
        const float klr = lr * fx_inv * fx_inv;
        int32_t nr = 0;
        for (int32_t r = r0; r < r1; r += RQ) {
#pragma unroll
            for (int s = 0; s < RQ; ++s) {
                const int32_t rr = r + s;
                const bool live = rr < r1;  // wave-uniform
                const int32_t item = live ? __builtin_amdgcn_readfirstlane(Hl[rr].x) : -1;
                const int32_t jb = live ? __builtin_amdgcn_readfirstlane(Hl[rr].y) : 0;
                const int32_t je = live ? __builtin_amdgcn_readfirstlane(Hl[rr + 1].y) : 0;
                int32_t q0[E];
                float q[E];
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    asm volatile("v_mov_b32 %0, %1" : "=v"(q0[x]) : "v"(ring[s][x]));
                    q[x] = qone[x] ? fx : static_cast<float>(q0[x]);
                }
                load_q(ring[s], item_of(rr + RQ));
                const float gbf = static_cast<float>(gb);
                float cs = 0.f;
                for (int32_t jj = jb; jj < je; ++jj) {
                    const int2 rec = Rl[jj];
                    const int32_t ul = __builtin_amdgcn_readfirstlane(rec.x);
                    const float rt = __int_as_float(__builtin_amdgcn_readfirstlane(rec.y));
                    int32_t* urow = Ul + ul * LU + lane;
                    const int32_t m = __builtin_amdgcn_readfirstlane(Ml[ul]);
                    const float nf = static_cast<float>(__builtin_amdgcn_readfirstlane(Nl[ul]));
                    const float rsq = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(Rs[ul])));
                    const float A = exp2f(static_cast<float>(m) * log2a);
                    float pu[E], ev[E];
#pragma unroll
                    for (int x = 0; x < E; ++x) {
                        pu[x] = static_cast<float>(urow[64 * x]);
                        const float sv = __int_as_float(urow[LD + 64 * x]);
                        const float cv = static_cast<float>(urow[2 * LD + 64 * x]);
                        ev[x] = pfac[x] ? A * (sv * fx - nf * cv) * rsq : 0.f;  // e in 2^-S units (svd.go:271-282)
                    }
                    float sd;
                    {
                        f2 acc = {0.f, 0.f};
#pragma unroll
                        for (int x = 0; x + 1 < E; x += 2) {
                            const f2 pv = {pu[x] + ev[x], pu[x + 1] + ev[x + 1]}, qv = {q[x], q[x + 1]};
                            acc = __builtin_elementwise_fma(pv, qv, acc);
                        }
                        sd = acc.x + acc.y;
                        if constexpr (E & 1) sd = __builtin_fmaf(pu[E - 1] + ev[E - 1], q[E - 1], sd);
                    }
                    sd = wave_sum_l63(sd);
                    // svd.go:363-396: diff = (gb + b_u + b_i + (p + e).q) - r, c = lr diff; p <- a p - c q;
                    // q <- a q - c (p_new + e); the biases through their constant partners (K1)
                    const float c = __builtin_fmaf(sd, klr, lr * ((gbf - cs) - rt));
                    cs += c;
                    const float sc = c * rsq * exp2f(-static_cast<float>(m + 1) * log2a);  // cy a^-(m+1)
#pragma unroll
                    for (int x = 0; x < E; ++x) {
                        float d = pone[x] ? 0.f : __builtin_fmaf(q[x], -c, pu[x] * am1);
                        const float np = pu[x] + d;
                        q[x] = qone[x] ? fx : __builtin_fmaf(np + ev[x], -c, q[x] * a);
                        __hip_atomic_fetch_add(urow + 64 * x, cvt_rpi(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (pfac[x])  // svd.go:408-418, lazily: C~_u += cy q_new a^-(m+1)
                            __hip_atomic_fetch_add(urow + 2 * LD + 64 * x, cvt_rpi(sc * q[x]), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    if (lane == 0) __hip_atomic_fetch_add(Ml + ul, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                gb -= static_cast<double>(cs);
                nr += je - jb;
                const int32_t row = item >= 0 ? item * (LD * 4) : -1;
#pragma unroll
                for (int x = 0; x < E; ++x)
                    __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(cvt_rpi(q[x]) - q0[x], rq, qaddr(row, x), 0, 0);
            }
        }
        contrib += static_cast<double>(nr) * (gb - gb0);
        __syncthreads();  // every rating of the tile trained: C~_u final (m_u = n_u)
        // map pass: per run, its users' maps y <- a^n y - a^n C~_u composed in order into (A, B), stored at the
        // run's slot (B in the first kf columns, A in column kf)
        for (int32_t r = r0; r < r1; ++r) {
            const int32_t jb = __builtin_amdgcn_readfirstlane(Hl[r].y), je = __builtin_amdgcn_readfirstlane(Hl[r + 1].y);
            float B[E];
#pragma unroll
            for (int x = 0; x < E; ++x) B[x] = 0.f;
            float Af = 1.f;
            for (int32_t jj = jb; jj < je; ++jj) {
                const int32_t ul = __builtin_amdgcn_readfirstlane(Rl[jj].x);
                const float al = exp2f(static_cast<float>(__builtin_amdgcn_readfirstlane(Nl[ul])) * log2a);
                const int32_t* urow = Ul + ul * LU + 2 * LD + lane;
#pragma unroll
                for (int x = 0; x < E; ++x) B[x] = al * (B[x] - static_cast<float>(urow[64 * x]) * fx_inv);
                Af *= al;
            }
            float* mrow = maps + static_cast<int64_t>(tm.z + r) * LD + lane;
#pragma unroll
            for (int x = 0; x < E; ++x) {
                const int32_t c = lane + 64 * x;
                mrow[64 * x] = c < kf ? B[x] : (c == kf ? Af : 0.f);
            }
        }
        __syncthreads();  // the maps read C~ before the next tile's staging overwrites it
        for (int32_t x = tid; x < nu * LD; x += NT) {  // P rows back (whole users: the schedule has no pieces)
            const int32_t ul = x / LD, c = x - ul * LD;
            if (c > kf) continue;
            P[static_cast<int64_t>(tile_users[tm.x + ul].x) * LD + c] = static_cast<float>(Ul[ul * LU + c]) * fx_inv;
        }
        __syncthreads();
    }
    if (lane == 0) gb_partial[static_cast<int64_t>(blockIdx.x) * NW + w] = contrib;
}

// Y pass: item j applies its runs' maps (A, B) in run order; one wave per item, 8 maps in flight
template <int E>
__global__ __launch_bounds__(256) void pp_tile_ymap_kernel(float* __restrict__ Y, const float* __restrict__ maps,
                                                           const int32_t* __restrict__ item_off,
                                                           const int32_t* __restrict__ item_runs, int32_t n_items, int32_t kf) {
    constexpr int LD = 64 * E;
    const int lane = threadIdx.x & 63;
    const int32_t j = static_cast<int32_t>(blockIdx.x) * 4 + static_cast<int32_t>(threadIdx.x >> 6);
    if (j >= n_items) return;
    float y[E];
#pragma unroll
    for (int x = 0; x < E; ++x) y[x] = Y[static_cast<int64_t>(j) * LD + lane + 64 * x];
    const int32_t b = item_off[j], e = item_off[j + 1];
    for (int32_t t = b; t < e; t += 8) {
        float A[8], B[8][E];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int32_t r = t + q < e ? item_runs[t + q] : -1;
            const float* mrow = maps + static_cast<int64_t>(r < 0 ? 0 : r) * LD;
            A[q] = r < 0 ? 1.f : mrow[kf];
#pragma unroll
            for (int x = 0; x < E; ++x) B[q][x] = r < 0 ? 0.f : mrow[lane + 64 * x];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int x = 0; x < E; ++x) y[x] = __builtin_fmaf(A[q], y[x], B[q][x]);
    }
#pragma unroll
    for (int x = 0; x < E; ++x) {
        const int32_t c = lane + 64 * x;
        Y[static_cast<int64_t>(j) * LD + c] = c < kf ? y[x] : 0.f;
    }
}

__global__ __launch_bounds__(1024) void pp_tile_gb_fold_kernel(const double* __restrict__ partial, int64_t n,
                                                               double* __restrict__ gb, double inv_nnz) {
    __shared__ double s[16];
    double t = 0.0;
    for (int64_t x = threadIdx.x; x < n; x += 1024) t += partial[x];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        double g = 0.0;
        for (int w = 0; w < 16; ++w) g += s[w];
        gb[0] += g * inv_nnz;
    }
}

template <int E>
void launch_pp_tile(int32_t grid, int32_t nw, const DevBuf<int4>& tiles, int32_t n_tiles, const DevBuf<int2>& users,
                    const DevBuf<int32_t>& streams, const DevBuf<int2>& runs, const DevBuf<int2>& recs,
                    const DevBuf<int64_t>& rowptr, DevBuf<float>& P, DevBuf<float>& Q, const DevBuf<float>& S,
                    DevBuf<float>& maps, const DevBuf<double>& gb, DevBuf<double>& part, float lr, float reg, float fx,
                    int32_t kf, float log2a, size_t lds, hipStream_t s) {
    const int32_t q_bytes = buffer_bytes32(Q.n, sizeof(float), "item factor matrix");
    auto go = [&](auto kern, int threads) {
        static bool attr = false;
        if (!attr) {
            RS_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(kTileLdsBudget)));
            attr = true;
        }
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, s, tiles.p, n_tiles, users.p, streams.p, runs.p, recs.p,
                           rowptr.p, P.p, reinterpret_cast<int32_t*>(Q.p), q_bytes, S.p, maps.p, gb.p, part.p, lr, reg,
                           fx, kf, log2a);
    };
    if (nw == 1) go(svdpp_tile_kernel<E, 1, 2>, 64);
    else go(svdpp_tile_kernel<E, 16, 2>, 1024);
}

}  // namespace

// The tile schedule of an SVD++ fit (host build, K1's rule with three LDS rows per user); false where it does not
// apply (a user too heavy for one tile's LDS).  Exported for the restatement test through rs_svdpp_tile_order.
bool pp_tile_schedule(rs_ctx* ctx, const UserCSR& csr, int64_t nnz, int32_t n_users, int32_t n_items, int32_t k,
                      int32_t workgroups, int32_t waves, bool want_pos, TileHost& th, int32_t& grid) {
    rs_svd_plan sp;
    sp.ctx = ctx;
    sp.n_users = n_users;
    sp.n_items = n_items;
    sp.k = k;
    sp.nnz = nnz;
    sp.h_rowptr = csr.rowptr;
    sp.h_cols.assign(csr.cols.begin(), csr.cols.begin() + nnz);
    sp.h_vals.assign(csr.vals.begin(), csr.vals.begin() + nnz);
    sp.tile_waves = waves;
    sp.tile_claim = 0;  // runs dealt to the waves on the host (streams)
    sp.tile_wg = workgroups;
    const int32_t LD = 64 * ((k + 2 + 63) / 64);
    sp.tile_user_lds = 3 * LD + 3;  // p, S, C~ rows and m, n, 1 / sqrt n
    grid = tile_grid0(&sp);
    std::vector<int32_t> bt, bu;
    build_tile_blocks(&sp, grid, want_pos, th, bt, bu);
    if (!th.split.empty()) return false;
    grid = std::max(1, std::min<int32_t>(grid, static_cast<int32_t>(th.tiles.size())));
    return true;
}

// FAST SVD++ on the tile schedule (rs_svdpp_fit's default where the schedule applies).  P / Q / Y / biases as
// rs_svdpp_fit: host f64 in and out; Q is int32 fixed point (2^-shift) on the device, P and Y fp32.
int svdpp_fit_tile(rs_ctx* ctx, const rs_ratings* r, const rs_sgd_params* p, const UserCSR& csr, int32_t shift,
                   int32_t workgroups, int32_t waves, double* P, double* Q, double* Y, double* bu, double* bi, double* gb,
                   bool* applied) {
    *applied = false;
    const int32_t k = p->n_factors, E = (k + 2 + 63) / 64, LD = 64 * E;
    if (E > 8) return RS_OK;
    TileHost th;
    int32_t grid = 0;
    if (!pp_tile_schedule(ctx, csr, r->nnz, r->n_users, r->n_items, k, workgroups, waves, false, th, grid)) return RS_OK;
    *applied = true;
    hipStream_t s = ctx->stream;
    const int32_t nw = waves;
    const int32_t n_tiles = static_cast<int32_t>(th.tiles.size());
    // the runs of every item in run order (tile order): the Y pass's map sequence
    std::vector<int32_t> item_off(static_cast<size_t>(r->n_items) + 1, 0), item_runs;
    for (int32_t t = 0; t < n_tiles; ++t) {
        const int32_t n_runs = th.streams[static_cast<size_t>(t) * (nw + 1) + nw];
        for (int32_t x = 0; x < n_runs; ++x) item_off[th.runs[th.tiles[t].z + x].x + 1]++;
    }
    for (int32_t i = 0; i < r->n_items; ++i) item_off[i + 1] += item_off[i];
    item_runs.resize(item_off[r->n_items]);
    {
        std::vector<int32_t> at(item_off.begin(), item_off.end() - 1);
        for (int32_t t = 0; t < n_tiles; ++t) {
            const int32_t n_runs = th.streams[static_cast<size_t>(t) * (nw + 1) + nw];
            for (int32_t x = 0; x < n_runs; ++x) item_runs[at[th.runs[th.tiles[t].z + x].x]++] = th.tiles[t].z + x;
        }
    }
    // LDS bytes of the largest tile: 3 LD + 3 ints per user (+ pad), records, run headers
    size_t lds = 16;
    for (int32_t t = 0; t < n_tiles; ++t) {
        const int32_t nu = th.tiles[t].y, n_runs = th.streams[static_cast<size_t>(t) * (nw + 1) + nw];
        const int32_t n_rec = th.runs[th.tiles[t].z + n_runs].y;
        lds = std::max(lds, static_cast<size_t>(nu) * (3 * LD + 3) * 4 + static_cast<size_t>(nu & 1) * 4 +
                                static_cast<size_t>(n_rec) * 8 + static_cast<size_t>(n_runs + 1) * 8);
    }
    if (lds > kTileLdsBudget) throw std::logic_error("SVD++ tile exceeds the LDS");
    // host packing: P fp32 (b_u in column k), Q int32 fixed point (b_i in column k), Y fp32
    const float fx = static_cast<float>(1u << shift);
    std::vector<float> hP(static_cast<size_t>(std::max(1, r->n_users)) * LD, 0.f), hY(static_cast<size_t>(std::max(1, r->n_items)) * LD, 0.f);
    std::vector<int32_t> hQ(static_cast<size_t>(std::max(1, r->n_items)) * LD, 0);
    for (int32_t u = 0; u < r->n_users; ++u) {
        for (int32_t c = 0; c < k; ++c) hP[static_cast<size_t>(u) * LD + c] = static_cast<float>(P[static_cast<size_t>(u) * k + c]);
        hP[static_cast<size_t>(u) * LD + k] = static_cast<float>(bu[u]);
    }
    for (int32_t i = 0; i < r->n_items; ++i) {
        for (int32_t c = 0; c < k; ++c) {
            hQ[static_cast<size_t>(i) * LD + c] = static_cast<int32_t>(std::lrint(static_cast<float>(Q[static_cast<size_t>(i) * k + c]) * fx));
            hY[static_cast<size_t>(i) * LD + c] = static_cast<float>(Y[static_cast<size_t>(i) * k + c]);
        }
        hQ[static_cast<size_t>(i) * LD + k] = static_cast<int32_t>(std::lrint(static_cast<float>(bi[i]) * fx));
    }
    DevBuf<int4> dt(std::max<size_t>(1, th.tiles.size()));
    DevBuf<int2> du(std::max<size_t>(1, th.users.size())), dr(std::max<size_t>(1, th.runs.size())), dc(std::max<size_t>(1, th.recs.size()));
    DevBuf<int32_t> dst(std::max<size_t>(1, th.streams.size())), doff(item_off.size()), druns(std::max<size_t>(1, item_runs.size()));
    DevBuf<int64_t> drow(csr.rowptr.size());
    DevBuf<int32_t> dcol(csr.cols.size());
    DevBuf<float> dP(hP.size()), dQ(hQ.size()), dY(hY.size()), dS(hP.size()), dmap(std::max<size_t>(1, th.runs.size()) * LD);
    DevBuf<double> dgb(1), dpart(static_cast<size_t>(grid) * nw);
    dt.upload(th.tiles.data(), th.tiles.size(), s);
    du.upload(th.users.data(), th.users.size(), s);
    dr.upload(th.runs.data(), th.runs.size(), s);
    dc.upload(th.recs.data(), th.recs.size(), s);
    dst.upload(th.streams.data(), th.streams.size(), s);
    doff.upload(item_off.data(), item_off.size(), s);
    druns.upload(item_runs.data(), item_runs.size(), s);
    drow.upload(csr.rowptr.data(), csr.rowptr.size(), s);
    dcol.upload(csr.cols.data(), csr.cols.size(), s);
    dP.upload(hP.data(), hP.size(), s);
    RS_HIP(hipMemcpyAsync(dQ.p, hQ.data(), hQ.size() * 4, hipMemcpyHostToDevice, s));
    dY.upload(hY.data(), hY.size(), s);
    if (p->n_epochs > 0) *gb = gb_warm_start(r, bu, bi);  // FAST's GlobalBias warm start (common.hpp)
    dgb.upload(gb, 1, s);
    const double inv_nnz = r->nnz > 0 ? 1.0 / static_cast<double>(r->nnz) : 0.0;
    const float lr = static_cast<float>(p->lr), reg = static_cast<float>(p->reg);
    const float log2a = std::log2(1.f - lr * reg);
    RS_HIP(hipStreamSynchronize(s));
    kernel_span_begin(ctx);
    for (int32_t ep = 0; ep < p->n_epochs && n_tiles > 0; ++ep) {
        auto epoch = [&](auto e_tag) {
            constexpr int EE = decltype(e_tag)::value;
            hipLaunchKernelGGL(pp_tile_sum_kernel<EE>, dim3((r->n_users + 3) / 4), dim3(256), 0, s, drow.p, dcol.p,
                               r->n_users, dY.p, dS.p, k);
            launch_pp_tile<EE>(grid, nw, dt, n_tiles, du, dst, dr, dc, drow, dP, dQ, dS, dmap, dgb, dpart, lr, reg, fx, k,
                               log2a, lds, s);
            hipLaunchKernelGGL(pp_tile_ymap_kernel<EE>, dim3((r->n_items + 3) / 4), dim3(256), 0, s, dY.p, dmap.p, doff.p,
                               druns.p, r->n_items, k);
        };
        switch (E) {
            case 1: epoch(std::integral_constant<int, 1>{}); break;
            case 2: epoch(std::integral_constant<int, 2>{}); break;
            case 3: epoch(std::integral_constant<int, 3>{}); break;
            case 4: epoch(std::integral_constant<int, 4>{}); break;
            case 5: epoch(std::integral_constant<int, 5>{}); break;
            case 6: epoch(std::integral_constant<int, 6>{}); break;
            case 7: epoch(std::integral_constant<int, 7>{}); break;
            default: epoch(std::integral_constant<int, 8>{}); break;
        }
        hipLaunchKernelGGL(pp_tile_gb_fold_kernel, dim3(1), dim3(1024), 0, s, dpart.p, static_cast<int64_t>(grid) * nw,
                           dgb.p, inv_nnz);
        RS_HIP(hipGetLastError());
    }
    kernel_span_end(ctx);
    dP.download(hP.data(), hP.size(), s);
    RS_HIP(hipMemcpyAsync(hQ.data(), dQ.p, hQ.size() * 4, hipMemcpyDeviceToHost, s));
    dY.download(hY.data(), hY.size(), s);
    dgb.download(gb, 1, s);
    RS_HIP(hipStreamSynchronize(s));
    bool bad = !std::isfinite(*gb);
    const double lim = 0.5 * 2147483648.0;
    for (int32_t u = 0; u < r->n_users; ++u) {
        for (int32_t c = 0; c < k; ++c) P[static_cast<size_t>(u) * k + c] = hP[static_cast<size_t>(u) * LD + c];
        bu[u] = hP[static_cast<size_t>(u) * LD + k];
        bad = bad || !std::isfinite(bu[u]);
    }
    for (int32_t i = 0; i < r->n_items; ++i) {
        for (int32_t c = 0; c <= k; ++c) {
            const int32_t v = hQ[static_cast<size_t>(i) * LD + c];
            bad = bad || std::fabs(static_cast<double>(v)) >= lim;
            const double d = static_cast<double>(static_cast<float>(v) / fx);
            if (c < k) Q[static_cast<size_t>(i) * k + c] = d;
            else bi[i] = d;
        }
        for (int32_t c = 0; c < k; ++c) {
            Y[static_cast<size_t>(i) * k + c] = hY[static_cast<size_t>(i) * LD + c];
            bad = bad || !std::isfinite(Y[static_cast<size_t>(i) * k + c]);
        }
    }
    if (bad)
        return set_error(ctx, RS_ERR_NUMERIC, "SVD++ factors left the fixed-point range (or went non-finite) during the "
                                              "fit; the returned model is not trustworthy");
    return RS_OK;
}

}  // namespace rs

extern "C" int rs_svdpp_set_schedule(rs_ctx* ctx, int32_t schedule, int32_t workgroups, int32_t waves) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    if (schedule < RS_PP_SCHED_AUTO || schedule > RS_PP_SCHED_USER)
        return rs::set_error(ctx, RS_ERR_INVALID, "schedule must be RS_PP_SCHED_AUTO, _TILE or _USER");
    if (workgroups < 0 || (waves != 1 && waves != 16))
        return rs::set_error(ctx, RS_ERR_INVALID, "workgroups must be >= 0 and waves 1 or 16");
    ctx->pp_schedule = schedule;
    ctx->pp_tile_wg = workgroups;
    ctx->pp_tile_waves = waves;
    return RS_OK;
}

extern "C" int rs_svdpp_schedule_used(const rs_ctx* ctx, int32_t* schedule) {
    if (!ctx || !schedule) return rs::set_error(nullptr, RS_ERR_INVALID, "NULL argument");
    *schedule = ctx->pp_used;
    return RS_OK;
}

extern "C" int rs_svdpp_tile_order(rs_ctx* ctx, const rs_ratings* r, int32_t n_factors, int32_t workgroups,
                                   int32_t waves, int64_t* pos, int64_t* run_off, int32_t* tile_off, int64_t* n_runs,
                                   int32_t* n_tiles) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        int st = rs::check_ratings(ctx, r);
        if (st != RS_OK) return st;
        if (!n_runs || !n_tiles) return rs::set_error(ctx, RS_ERR_INVALID, "NULL argument");
        if (n_factors < 1 || n_factors > 510 || workgroups < 0 || (waves != 1 && waves != 16))
            return rs::set_error(ctx, RS_ERR_INVALID, "n_factors, workgroups or waves out of range");
        rs::UserCSR csr;
        rs::build_csr(r->nnz, r->n_users, r->users, r->items, r->ratings, csr);
        rs::TileHost th;
        int32_t grid = 0;
        if (!rs::pp_tile_schedule(ctx, csr, r->nnz, r->n_users, r->n_items, n_factors, workgroups, waves, true, th, grid))
            return rs::set_error(ctx, RS_ERR_UNSUPPORTED, "a user's row exceeds one tile's LDS");
        const int32_t nt = static_cast<int32_t>(th.tiles.size());
        int64_t nr = 0;
        for (int32_t t = 0; t < nt; ++t) nr += th.streams[static_cast<size_t>(t) * (waves + 1) + waves];
        *n_runs = nr;
        *n_tiles = nt;
        if (!pos || !run_off || !tile_off) return RS_OK;
        int64_t at = 0;
        for (int32_t t = 0; t < nt; ++t) {
            const int4 tm = th.tiles[t];
            const int32_t nrt = th.streams[static_cast<size_t>(t) * (waves + 1) + waves];
            tile_off[t] = static_cast<int32_t>(at);
            for (int32_t x = 0; x < nrt; ++x) run_off[at++] = tm.w + th.runs[tm.z + x].y;
        }
        tile_off[nt] = static_cast<int32_t>(at);
        run_off[nr] = static_cast<int64_t>(th.recs.size());
        std::copy(th.pos.begin(), th.pos.end(), pos);
        return RS_OK;
    });
}
