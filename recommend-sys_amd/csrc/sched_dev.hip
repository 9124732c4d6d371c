// sched_dev.hip -- the tile schedule of sgd_tile.hip built on the device (RS_TILE_RULE_FILL_DEVICE), so that
// a one-shot rs_svd_fit (the Go Fit, reference core/svd.go:63-132) spends no host time on it.
//
// The rule is the host build's RS_TILE_RULE_FILL (build_tile_host), restated with radix sorts:
//   1. degrees: histogram of the COO's users and items; one readback {active users, max user degree,
//      max item degree} fixes the tile count, the run cap and the key widths on the host;
//   2. tiles: the users sorted by degree (descending; a stable sort keeps ties in id order); the first
//      kFillSnakeRounds * T are dealt boustrophedon -- position p, round r = p / T, tile r even ? p % T :
//      T - 1 - p % T --; the tiles' deficits against the mean load, sorted (descending, ties by tile), are laid
//      end to end and the remaining users, heaviest first, go to the tile whose stretch holds the midpoint of
//      their prefix sums; a second stable sort of the users by tile gives every tile its entries in user order;
//   3. runs: the ratings sorted by (tile, run_key(item, tile), tile-local user) -- one stable LSD sort, so a
//      run's ratings come in user order and a user's repeated item in COO order, as the host's CSR scan
//      gives them -- are cut where (tile, key) changes; a run longer than the cap is cut into
//      min(ceil(c / cap), waves) adjacent pieces at c * p / pieces, as in the host's claim queue;
//   4. emit: tiles {first entry, entries, first run, first record}, entries {user, 1.0f}, streams
//      {0, n, ..., n}, run headers {item, first record} + a sentinel {-1, records} per tile, records
//      {tile-local user, rating bits}; a second readback brings the LDS bytes of the largest tile.
// Keys are distinct within a tile (run_key is a bijection of the item), so no tie rule is needed and the
// two builds are byte-identical (tests/test_sched_dev_gpu.py compares rs_svd_plan_schedule_digest).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "common.hpp"
#include "sgd_plan.hpp"

namespace rs {
namespace {

constexpr int kB = 256;
inline int blocks_for(int64_t n) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + kB - 1) / kB, 1 << 20))); }
inline int bit_len(uint64_t x) { int b = 0; while (x) { ++b; x >>= 1; } return b; }

// exclusive prefix sum on the stream (rocPRIM's device scan; a null temp pointer queries its bytes)
template <class T>
hipError_t excl_sum(void* temp, size_t& bytes, const T* in, T* out, int64_t n, hipStream_t s) {
    return rocprim::exclusive_scan(temp, bytes, in, out, T{0}, static_cast<size_t>(n), rocprim::plus<T>(), s);
}

// stats: [0] active users, [1] max user degree, [2] max item degree, [3] LDS bytes of the largest tile,
// [4] run-header entries (pieces + one sentinel per tile)
__global__ __launch_bounds__(kB) void degrees_kernel(const int32_t* __restrict__ users, const int32_t* __restrict__ items,
                                                     int64_t n, int32_t* __restrict__ deg_u, int32_t* __restrict__ deg_i) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(kB) + threadIdx.x; j < n; j += static_cast<int64_t>(gridDim.x) * kB) {
        atomicAdd(deg_u + users[j], 1);
        atomicAdd(deg_i + items[j], 1);
    }
}

__global__ __launch_bounds__(kB) void degree_stats_kernel(const int32_t* __restrict__ deg_u, int32_t nu,
                                                          const int32_t* __restrict__ deg_i, int32_t ni,
                                                          int32_t* __restrict__ stats) {
    int32_t act = 0, mu = 0, mi = 0;
    for (int32_t x = blockIdx.x * kB + threadIdx.x; x < nu || x < ni; x += gridDim.x * kB) {
        if (x < nu) { act += deg_u[x] > 0; mu = max(mu, deg_u[x]); }
        if (x < ni) mi = max(mi, deg_i[x]);
    }
    for (int o = 32; o > 0; o >>= 1) {  // wave reductions, one atomic per wave
        act += __shfl_xor(act, o);
        mu = max(mu, __shfl_xor(mu, o));
        mi = max(mi, __shfl_xor(mi, o));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(stats + 0, act);
        atomicMax(stats + 1, mu);
        atomicMax(stats + 2, mi);
    }
}

// keys of the degree sort (descending degree = ascending dmax - d; inactive users last) and the identity
__global__ __launch_bounds__(kB) void degree_keys_kernel(const int32_t* __restrict__ deg_u, int32_t nu, int32_t dmax,
                                                         uint32_t* __restrict__ key, int32_t* __restrict__ iota) {
    const int32_t u = blockIdx.x * kB + threadIdx.x;
    if (u >= nu) return;
    key[u] = static_cast<uint32_t>(dmax - deg_u[u]);
    iota[u] = u;
}

// boustrophedon deal of the first ns users of the degree order over T tiles, with the tiles' loads; the rest
// of the active users are placed by fill_kernel (inactive users: tile T, sorted past every tile)
// (weights: the LDS bytes w0 + w1 d of a user, w0 = 4 ld, w1 = 16)
__global__ __launch_bounds__(kB) void snake_kernel(const int32_t* __restrict__ by_deg, const int32_t* __restrict__ deg_u,
                                                   int32_t nu, int32_t n_active, int32_t ns, int32_t T, int32_t w0,
                                                   int32_t w1, uint32_t* __restrict__ tile_of,
                                                   unsigned long long* __restrict__ load, int64_t* __restrict__ rem_w) {
    const int32_t p = blockIdx.x * kB + threadIdx.x;
    if (p >= nu) return;
    const int32_t u = by_deg[p];
    const int64_t wu = w0 + static_cast<int64_t>(w1) * deg_u[u];
    if (p < ns) {
        const int32_t r = p / T, i = p - r * T;
        const int32_t t = (r & 1) ? T - 1 - i : i;
        tile_of[u] = static_cast<uint32_t>(t);
        atomicAdd(load + t, static_cast<unsigned long long>(wu));
    } else if (p < n_active) {
        rem_w[p - ns] = wu;
    } else {
        tile_of[u] = static_cast<uint32_t>(T);
    }
}

// deficit keys of the line: ascending key = descending deficit (a stable sort keeps ties in tile order)
__global__ __launch_bounds__(kB) void deficit_kernel(const unsigned long long* __restrict__ load, int32_t T, int64_t mean,
                                                     uint64_t* __restrict__ key, int32_t* __restrict__ iota) {
    const int32_t t = blockIdx.x * kB + threadIdx.x;
    if (t >= T) return;
    const int64_t d = max<int64_t>(0, mean - static_cast<int64_t>(load[t]));
    key[t] = static_cast<uint64_t>(INT64_MAX - d);
    iota[t] = t;
}

__global__ __launch_bounds__(kB) void line_kernel(const unsigned long long* __restrict__ load, const int32_t* __restrict__ lt,
                                                  int32_t T, int64_t mean, int64_t* __restrict__ dl) {
    const int32_t j = blockIdx.x * kB + threadIdx.x;
    if (j < T) dl[j] = max<int64_t>(0, mean - static_cast<int64_t>(load[lt[j]]));
    if (j == T) dl[T] = 0;
}

// the remaining users: the tile whose stretch of the line (exclusive prefix E, T + 1 entries) holds the
// midpoint of their prefix sum R: first j with 2 E[j + 1] > 2 R + d
__global__ __launch_bounds__(kB) void fill_kernel(const int32_t* __restrict__ by_deg, int32_t ns, int32_t n_rem,
                                                  const int64_t* __restrict__ rem_d, const int64_t* __restrict__ R,
                                                  const int64_t* __restrict__ E, const int32_t* __restrict__ lt,
                                                  int32_t T, uint32_t* __restrict__ tile_of) {
    const int32_t q = blockIdx.x * kB + threadIdx.x;
    if (q >= n_rem) return;
    const int64_t m2 = 2 * R[q] + rem_d[q];
    int32_t lo = 0, hi = T;  // over j in [0, T): predicate 2 E[j + 1] > m2 is monotone
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (2 * E[mid + 1] > m2) hi = mid;
        else lo = mid + 1;
    }
    tile_of[by_deg[ns + q]] = static_cast<uint32_t>(lt[min(lo, T - 1)]);
}

// entries (users in tile order): per tile its first entry, users and ratings; per user its tile-local index
__global__ __launch_bounds__(kB) void entries_kernel(const int32_t* __restrict__ entry_user, int32_t n_active,
                                                     const uint32_t* __restrict__ tile_of, const int32_t* __restrict__ deg_u,
                                                     int32_t* __restrict__ first_entry, int32_t* __restrict__ users_t,
                                                     int32_t* __restrict__ recs_t) {
    const int32_t x = blockIdx.x * kB + threadIdx.x;
    if (x >= n_active) return;
    const int32_t u = entry_user[x];
    const int32_t t = static_cast<int32_t>(tile_of[u]);
    if (x == 0 || static_cast<int32_t>(tile_of[entry_user[x - 1]]) != t) first_entry[t] = x;
    atomicAdd(users_t + t, 1);
    atomicAdd(recs_t + t, deg_u[u]);
}

__global__ __launch_bounds__(kB) void local_index_kernel(const int32_t* __restrict__ entry_user, int32_t n_active,
                                                         const uint32_t* __restrict__ tile_of,
                                                         const int32_t* __restrict__ first_entry, int32_t* __restrict__ ul_of,
                                                         int2* __restrict__ t_users) {
    const int32_t x = blockIdx.x * kB + threadIdx.x;
    if (x >= n_active) return;
    const int32_t u = entry_user[x];
    ul_of[u] = x - first_entry[tile_of[u]];
    t_users[x] = make_int2(u, 0x3F800000);  // {user, 1.0f}: whole users only (no pieces under this rule)
}

// the ratings' sort keys: tile | run key | tile-local user (bit widths from the host)
__global__ __launch_bounds__(kB) void rating_keys_kernel(const int32_t* __restrict__ users, const int32_t* __restrict__ items,
                                                         int64_t n, const uint32_t* __restrict__ tile_of,
                                                         const int32_t* __restrict__ ul_of, int ulb,
                                                         uint64_t* __restrict__ key, int32_t* __restrict__ idx) {
    for (int64_t j = blockIdx.x * static_cast<int64_t>(kB) + threadIdx.x; j < n; j += static_cast<int64_t>(gridDim.x) * kB) {
        const int32_t u = users[j];
        const uint32_t t = tile_of[u];
        key[j] = (static_cast<uint64_t>(t) << (32 + ulb)) | (static_cast<uint64_t>(run_key(items[j], static_cast<int32_t>(t))) << ulb) |
                 static_cast<uint64_t>(ul_of[u]);
        idx[j] = static_cast<int32_t>(j);
    }
}

// run heads (a change of (tile, key)) and the records {tile-local user, rating bits}
__global__ __launch_bounds__(kB) void heads_kernel(const uint64_t* __restrict__ key, const int32_t* __restrict__ perm,
                                                   const float* __restrict__ vals, int64_t n, int ulb,
                                                   int32_t* __restrict__ head, int2* __restrict__ recs) {
    for (int64_t o = blockIdx.x * static_cast<int64_t>(kB) + threadIdx.x; o < n; o += static_cast<int64_t>(gridDim.x) * kB) {
        const uint64_t k = key[o];
        head[o] = (o == 0 || (k >> ulb) != (key[o - 1] >> ulb)) ? 1 : 0;
        recs[o] = make_int2(static_cast<int32_t>(k & ((uint64_t{1} << ulb) - 1)), __float_as_int(vals[perm[o]]));
    }
}

// run r starts at position o (head); its pieces: min(ceil(c / cap), waves), or 1
__global__ __launch_bounds__(kB) void run_start_kernel(const int32_t* __restrict__ head, const int32_t* __restrict__ rid,
                                                       int64_t n, int32_t* __restrict__ run_start) {
    for (int64_t o = blockIdx.x * static_cast<int64_t>(kB) + threadIdx.x; o < n; o += static_cast<int64_t>(gridDim.x) * kB)
        if (head[o]) run_start[rid[o]] = static_cast<int32_t>(o);
}

__global__ __launch_bounds__(kB) void pieces_kernel(const int32_t* __restrict__ head, const int32_t* __restrict__ rid,
                                                    const int32_t* __restrict__ run_start, int64_t n, int32_t cap,
                                                    int32_t waves, int32_t* __restrict__ pieces) {
    const int32_t n_runs = rid[n - 1] + head[n - 1];
    for (int64_t o = blockIdx.x * static_cast<int64_t>(kB) + threadIdx.x; o < n; o += static_cast<int64_t>(gridDim.x) * kB) {
        if (!head[o]) continue;
        const int32_t r = rid[o];
        const int64_t c = (r + 1 < n_runs ? run_start[r + 1] : n) - o;
        pieces[r] = cap > 0 ? static_cast<int32_t>(min<int64_t>((c + cap - 1) / cap, waves)) : 1;
    }
}

// run headers: piece q of run r (tile t, tile-local first record b, c ratings) at pscan[r] + t + q
__global__ __launch_bounds__(kB) void runs_kernel(const int32_t* __restrict__ head, const int32_t* __restrict__ rid,
                                                  const int32_t* __restrict__ run_start, const int32_t* __restrict__ pscan,
                                                  const uint64_t* __restrict__ key, const int32_t* __restrict__ perm,
                                                  const int32_t* __restrict__ items, const int32_t* __restrict__ rec_at,
                                                  int64_t n, int ulb, int2* __restrict__ runs) {
    const int32_t n_runs = rid[n - 1] + head[n - 1];
    for (int64_t o = blockIdx.x * static_cast<int64_t>(kB) + threadIdx.x; o < n; o += static_cast<int64_t>(gridDim.x) * kB) {
        if (!head[o]) continue;
        const int32_t r = rid[o];
        const int32_t t = static_cast<int32_t>(key[o] >> (32 + ulb));
        const int64_t c = (r + 1 < n_runs ? run_start[r + 1] : n) - o;
        const int32_t b = static_cast<int32_t>(o) - rec_at[t], pcs = pscan[r + 1] - pscan[r];
        const int32_t item = items[perm[o]];
        for (int32_t q = 0; q < pcs; ++q)
            runs[pscan[r] + t + q] = make_int2(item, b + static_cast<int32_t>(c * q / pcs));
    }
}

// cold runs (sgd_plan.hpp kRunCold): the header bit for items with fewer than dcold ratings, as the host build sets it
__global__ __launch_bounds__(kB) void cold_runs_kernel(int2* __restrict__ runs, int64_t n_runs, const int32_t* __restrict__ deg,
                                                       int32_t n_items, int64_t dcold) {
    for (int64_t r = blockIdx.x * static_cast<int64_t>(kB) + threadIdx.x; r < n_runs; r += static_cast<int64_t>(gridDim.x) * kB) {
        const int32_t it = runs[r].x;
        if (it >= 0 && it < n_items && deg[it] < dcold) runs[r].x = it | kRunCold;
    }
}

// per tile: its header {first entry, entries, first run, first record}, sentinel, streams and LDS bytes
__global__ __launch_bounds__(kB) void tiles_kernel(const int32_t* __restrict__ first_entry, const int32_t* __restrict__ users_t,
                                                   const int32_t* __restrict__ recs_t, const int32_t* __restrict__ rec_at,
                                                   const int32_t* __restrict__ head, const int32_t* __restrict__ rid,
                                                   const int32_t* __restrict__ pscan, int64_t n, int32_t T, int32_t waves, int32_t ld,
                                                   int4* __restrict__ tiles, int2* __restrict__ runs,
                                                   int32_t* __restrict__ streams, int32_t* __restrict__ stats) {
    const int32_t t = blockIdx.x * kB + threadIdx.x;
    if (t >= T) return;
    const int32_t n_runs_total = rid[n - 1] + head[n - 1];
    const int32_t r0 = pscan[rid[rec_at[t]]] + t;
    const int32_t r1 = t + 1 < T ? pscan[rid[rec_at[t + 1]]] + t + 1 : pscan[n_runs_total] + T;
    const int32_t n_runs = r1 - r0 - 1;
    runs[r1 - 1] = make_int2(-1, recs_t[t]);
    int32_t* st = streams + static_cast<int64_t>(t) * (waves + 1);
    st[0] = 0;
    for (int32_t s = 1; s <= waves; ++s) st[s] = n_runs;
    tiles[t] = make_int4(first_entry[t], users_t[t], r0, rec_at[t]);
    const int64_t bytes = static_cast<int64_t>(users_t[t]) * ld * 4 + static_cast<int64_t>(recs_t[t]) * 8 +
                          static_cast<int64_t>(n_runs + 1) * 8;
    atomicMax(stats + 3, static_cast<int32_t>(min<int64_t>(bytes, 0x7FFFFFFF)));
    if (t == T - 1) stats[4] = r1;
}

// workspace carving (256-B aligned pieces of one allocation)
struct Carve {
    char* base;
    size_t at = 0;
    template <typename T>
    T* take(size_t count) {
        T* p = reinterpret_cast<T*>(base ? base + at : nullptr);
        at += (count * sizeof(T) + 255) / 256 * 256;
        return p;
    }
};


}  // namespace

bool tile_build_device(rs_svd_plan* pl) {
    static const bool trace = std::getenv("RSGPU_FIT_TRACE") != nullptr;  // (syncs: phase times on stderr)
    auto tprev = std::chrono::steady_clock::now();
    auto tmark = [&](const char* what) {
        if (!trace) return;
        (void)hipStreamSynchronize(pl->ctx->stream);
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "sched-dev %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t1 - tprev).count());
        tprev = t1;
    };
    if (pl->tile_claim <= 0 || pl->tile_ublocks != 1 || !pl->ublock_bounds.empty() || !pl->iblock_bounds.empty())
        return false;
    const int64_t n = pl->nnz;
    if (n <= 0 || n >= (int64_t{1} << 31) || !pl->coo_users.p) return false;
    hipStream_t s = pl->ctx->stream;
    const int32_t nu = pl->n_users, ni = std::max(1, pl->n_items), nw = pl->tile_waves;
    const int32_t grid0 = tile_grid0(pl);  // (the host build's own function: the two builds agree)
    const int32_t ld = tile_lds_row(pl);
    const int64_t rec_cap = static_cast<int64_t>((kTileLdsBudget - 16 - static_cast<size_t>(ld) * 4) / 16);
    int32_t* h = static_cast<int32_t*>(pinned_small(pl->ctx, kPinSched));  // 8 ints of readback

    // workspace (sizes bounded by n, the users and the items; the tiles are at most the active users)
    auto carve = [&](Carve& c) {
        struct W {
            int32_t *deg_u, *deg_i, *stats, *iota, *by_deg, *entry_user, *ul_of, *first_entry, *users_t, *recs_t, *rec_at;
            uint32_t *dkey, *dkey_o, *tile_of, *tkey_o;
            uint64_t *key, *key_o;
            int32_t *idx, *perm, *head, *rid, *run_start, *pieces, *pscan;
            int32_t* lt;
            unsigned long long* load;
            uint64_t *lkey, *lkey_o;
            int64_t *rem_w, *R, *dl, *E;
            void* temp;
        } w;
        const size_t U = static_cast<size_t>(std::max(1, nu)), N = static_cast<size_t>(n);
        w.deg_u = c.take<int32_t>(U);
        w.deg_i = c.take<int32_t>(static_cast<size_t>(ni));
        w.stats = c.take<int32_t>(8);
        w.iota = c.take<int32_t>(U);
        w.by_deg = c.take<int32_t>(U);
        w.entry_user = c.take<int32_t>(U);
        w.ul_of = c.take<int32_t>(U);
        w.first_entry = c.take<int32_t>(U + 1);
        w.users_t = c.take<int32_t>(U + 1);
        w.recs_t = c.take<int32_t>(U + 1);
        w.rec_at = c.take<int32_t>(U + 1);
        w.dkey = c.take<uint32_t>(U);
        w.dkey_o = c.take<uint32_t>(U);
        w.tile_of = c.take<uint32_t>(U);
        w.tkey_o = c.take<uint32_t>(U);
        w.key = c.take<uint64_t>(N);
        w.key_o = c.take<uint64_t>(N);
        w.idx = c.take<int32_t>(N);
        w.perm = c.take<int32_t>(N);
        w.head = c.take<int32_t>(N);
        w.rid = c.take<int32_t>(N);
        w.run_start = c.take<int32_t>(N);
        w.pieces = c.take<int32_t>(N + 1);
        w.pscan = c.take<int32_t>(N + 1);
        w.load = c.take<unsigned long long>(U + 1);
        w.lkey = c.take<uint64_t>(U + 1);
        w.lkey_o = c.take<uint64_t>(U + 1);
        w.lt = c.take<int32_t>(U + 1);
        w.rem_w = c.take<int64_t>(U + 1);
        w.R = c.take<int64_t>(U + 1);
        w.dl = c.take<int64_t>(U + 1);
        w.E = c.take<int64_t>(U + 1);
        w.temp = nullptr;
        return w;
    };
    // rocPRIM temp storage: the largest of the five sorts / scans, queried with null pointers
    size_t tmp = 0, t1 = 0;
    RS_HIP(rocprim::radix_sort_pairs(nullptr, t1, static_cast<const uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr),
                                              static_cast<const int32_t*>(nullptr), static_cast<int32_t*>(nullptr), std::max(1, nu), 0, 32, s));
    tmp = std::max(tmp, t1);
    RS_HIP(rocprim::radix_sort_pairs(nullptr, t1, static_cast<const uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr),
                                              static_cast<const int32_t*>(nullptr), static_cast<int32_t*>(nullptr), n, 0, 64, s));
    tmp = std::max(tmp, t1);
    RS_HIP(excl_sum(nullptr, t1, static_cast<const int32_t*>(nullptr), static_cast<int32_t*>(nullptr), n + 1, s));
    tmp = std::max(tmp, t1);
    RS_HIP(excl_sum(nullptr, t1, static_cast<const int64_t*>(nullptr), static_cast<int64_t*>(nullptr),
                                            static_cast<int64_t>(std::max(1, nu)) + 1, s));
    tmp = std::max(tmp, t1);
    RS_HIP(rocprim::radix_sort_pairs(nullptr, t1, static_cast<const uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr),
                                              static_cast<const int32_t*>(nullptr), static_cast<int32_t*>(nullptr), std::max(1, nu), 0, 64, s));
    tmp = std::max(tmp, t1);
    Carve probe{nullptr};
    (void)carve(probe);
    const size_t ws_bytes = probe.at + (tmp + 255) / 256 * 256;
    if (pl->sched_ws.n < ws_bytes) pl->sched_ws.alloc(ws_bytes);
    Carve cv{pl->sched_ws.p};
    auto w = carve(cv);
    w.temp = pl->sched_ws.p + cv.at;
    tmark("workspace");

    // 1. degrees and the first readback
    RS_HIP(hipMemsetAsync(w.deg_u, 0, sizeof(int32_t) * std::max(1, nu), s));
    RS_HIP(hipMemsetAsync(w.deg_i, 0, sizeof(int32_t) * ni, s));
    RS_HIP(hipMemsetAsync(w.stats, 0, sizeof(int32_t) * 8, s));
    hipLaunchKernelGGL(degrees_kernel, dim3(std::min(blocks_for(n), 4096)), dim3(kB), 0, s, pl->coo_users.p, pl->coo_items.p,
                       n, w.deg_u, w.deg_i);
    hipLaunchKernelGGL(degree_stats_kernel, dim3(std::min(blocks_for(std::max(nu, ni)), 1024)), dim3(kB), 0, s, w.deg_u, nu,
                       w.deg_i, ni, w.stats);
    RS_HIP(hipGetLastError());
    RS_HIP(hipMemcpyAsync(h, w.stats, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (pl->build_overlap) {  // the caller's host work (rs_svd_fit: GlobalBias warm start, factor packing) runs
        auto f = std::move(pl->build_overlap);  // under the COO upload and the degree kernels
        pl->build_overlap = nullptr;
        f();
    }
    RS_HIP(hipStreamSynchronize(s));
    const int32_t n_active = h[0], dmax_u = h[1], dmax_i = h[2];
    tmark("degrees");
    if (n_active <= 0 || dmax_u > rec_cap) {  // users cut into pieces: the host builds
        if (trace) std::fprintf(stderr, "sched-dev fallback: active %d, max degree %d, LDS record cap %lld\n", n_active, dmax_u,
                                static_cast<long long>(rec_cap));
        return false;
    }
    const int64_t target = pl->tile_target > 0 ? pl->tile_target
                                               : std::max<int64_t>({64, dmax_u, (n + grid0 - 1) / std::max(1, grid0)});
    const int64_t n_target = (n + target - 1) / std::max<int64_t>(target, 1);
    const double bytes = static_cast<double>(n_active) * (static_cast<double>(ld) * 4) + 16.0 * static_cast<double>(n);
    const int64_t n_lds = static_cast<int64_t>(std::ceil(bytes / (0.85 * static_cast<double>(kTileLdsBudget))));
    const int32_t T = static_cast<int32_t>(std::min<int64_t>(std::max<int64_t>({1, n_target, n_lds}), n_active));
    const int32_t cap = (pl->tile_run_cap > 0 ? pl->tile_run_cap : run_cap_rule(n, dmax_i, grid0, nw, pl->k));
    const int32_t cap_eff = (cap > 0 && nw > 1) ? cap : 0;
    // tile-local user index width: a tile holds at most kFillSnakeRounds dealt users plus the users whose
    // midpoints fall in its stretch of the line, at most its deficit + 1 <= mean + 1 (every user spans >= 1)
    // (the weights are LDS bytes: a user weighs >= 4 ld + 16, so a stretch holds at most mean / that + 1 users)
    const int64_t wmin = int64_t{4} * ld + 16;
    const int64_t mean_w = (int64_t{4} * ld * n_active + 16 * n + T - 1) / T;
    const int ulb = bit_len(static_cast<uint64_t>(std::min<int64_t>(n_active - 1, kFillSnakeRounds + mean_w / wmin + 1)));
    const int tb = bit_len(static_cast<uint64_t>(T));  // tile ids 0..T (T: inactive users' sort key)
    if (tb + 32 + ulb > 64) {
        if (trace) std::fprintf(stderr, "sched-dev fallback: key bits %d + 32 + %d\n", tb, ulb);
        return false;
    }

    // 2. tiles: degree order, boustrophedon deal of the heaviest, deficit fill of the rest, entries in tile order
    const int ub = blocks_for(nu);
    hipLaunchKernelGGL(degree_keys_kernel, dim3(ub), dim3(kB), 0, s, w.deg_u, nu, dmax_u, w.dkey, w.iota);
    size_t tb_bytes = tmp;
    RS_HIP(rocprim::radix_sort_pairs(w.temp, tb_bytes, w.dkey, w.dkey_o, w.iota, w.by_deg, nu, 0,
                                              std::max(1, bit_len(static_cast<uint64_t>(dmax_u))), s));
    const int32_t ns = static_cast<int32_t>(std::min<int64_t>(n_active, static_cast<int64_t>(kFillSnakeRounds) * T));
    const int32_t n_rem = n_active - ns;
    // loads in LDS bytes, as build_tile_host
    const int32_t w0 = 4 * ld, w1 = 16;
    const int64_t wsum = static_cast<int64_t>(w0) * n_active + static_cast<int64_t>(w1) * n;
    const int64_t mean = (wsum + T - 1) / T;
    RS_HIP(hipMemsetAsync(w.load, 0, sizeof(unsigned long long) * (T + 1), s));
    hipLaunchKernelGGL(snake_kernel, dim3(ub), dim3(kB), 0, s, w.by_deg, w.deg_u, nu, n_active, ns, T, w0, w1, w.tile_of,
                       w.load, w.rem_w);
    if (n_rem > 0) {  // the deficit line and the fill
        hipLaunchKernelGGL(deficit_kernel, dim3(blocks_for(T)), dim3(kB), 0, s, w.load, T, mean, w.lkey, w.iota);  // (iota[t] = t: unchanged)
        tb_bytes = tmp;
        RS_HIP(rocprim::radix_sort_pairs(w.temp, tb_bytes, w.lkey, w.lkey_o, w.iota, w.lt, T, 0, 64, s));
        hipLaunchKernelGGL(line_kernel, dim3(blocks_for(T + 1)), dim3(kB), 0, s, w.load, w.lt, T, mean, w.dl);
        tb_bytes = tmp;
        RS_HIP(excl_sum(w.temp, tb_bytes, w.dl, w.E, T + 1, s));
        tb_bytes = tmp;
        RS_HIP(excl_sum(w.temp, tb_bytes, w.rem_w, w.R, n_rem, s));
        hipLaunchKernelGGL(fill_kernel, dim3(blocks_for(n_rem)), dim3(kB), 0, s, w.by_deg, ns, n_rem, w.rem_w, w.R, w.E,
                           w.lt, T, w.tile_of);
    }
    tb_bytes = tmp;
    RS_HIP(rocprim::radix_sort_pairs(w.temp, tb_bytes, w.tile_of, w.tkey_o, w.iota, w.entry_user, nu, 0, tb, s));
    RS_HIP(hipMemsetAsync(w.users_t, 0, sizeof(int32_t) * (T + 1), s));
    RS_HIP(hipMemsetAsync(w.recs_t, 0, sizeof(int32_t) * (T + 1), s));
    hipLaunchKernelGGL(entries_kernel, dim3(blocks_for(n_active)), dim3(kB), 0, s, w.entry_user, n_active, w.tile_of,
                       w.deg_u, w.first_entry, w.users_t, w.recs_t);
    tb_bytes = tmp;
    RS_HIP(excl_sum(w.temp, tb_bytes, w.recs_t, w.rec_at, T + 1, s));
    // outputs (upper bounds: pieces <= ratings)
    const size_t runs_cap = static_cast<size_t>(n) + static_cast<size_t>(T);
    if (pl->t_tiles.n < static_cast<size_t>(T)) pl->t_tiles.alloc(static_cast<size_t>(T));
    if (pl->t_users.n < static_cast<size_t>(n_active)) pl->t_users.alloc(static_cast<size_t>(n_active));
    if (pl->t_streams.n < static_cast<size_t>(T) * (nw + 1)) pl->t_streams.alloc(static_cast<size_t>(T) * (nw + 1));
    if (pl->t_runs.n < runs_cap) pl->t_runs.alloc(runs_cap);
    if (pl->t_recs.n < static_cast<size_t>(n)) pl->t_recs.alloc(static_cast<size_t>(n));
    tmark("tiles");
    hipLaunchKernelGGL(local_index_kernel, dim3(blocks_for(n_active)), dim3(kB), 0, s, w.entry_user, n_active, w.tile_of,
                       w.first_entry, w.ul_of, pl->t_users.p);

    // 3. runs: ratings by (tile, key, tile-local user), heads, pieces
    const int nb = std::min(blocks_for(n), 8192);
    hipLaunchKernelGGL(rating_keys_kernel, dim3(nb), dim3(kB), 0, s, pl->coo_users.p, pl->coo_items.p, n, w.tile_of, w.ul_of,
                       ulb, w.key, w.idx);
    tb_bytes = tmp;
    RS_HIP(rocprim::radix_sort_pairs(w.temp, tb_bytes, w.key, w.key_o, w.idx, w.perm, n, 0, tb + 32 + ulb, s));
    hipLaunchKernelGGL(heads_kernel, dim3(nb), dim3(kB), 0, s, w.key_o, w.perm, pl->coo_vals.p, n, ulb, w.head, pl->t_recs.p);
    tb_bytes = tmp;
    RS_HIP(excl_sum(w.temp, tb_bytes, w.head, w.rid, n, s));
    hipLaunchKernelGGL(run_start_kernel, dim3(nb), dim3(kB), 0, s, w.head, w.rid, n, w.run_start);
    RS_HIP(hipMemsetAsync(w.pieces, 0, sizeof(int32_t) * (n + 1), s));
    hipLaunchKernelGGL(pieces_kernel, dim3(nb), dim3(kB), 0, s, w.head, w.rid, w.run_start, n, cap_eff, nw, w.pieces);
    tb_bytes = tmp;
    RS_HIP(excl_sum(w.temp, tb_bytes, w.pieces, w.pscan, n + 1, s));

    // 4. emit
    tmark("runs");
    hipLaunchKernelGGL(runs_kernel, dim3(nb), dim3(kB), 0, s, w.head, w.rid, w.run_start, w.pscan, w.key_o, w.perm,
                       pl->coo_items.p, w.rec_at, n, ulb, pl->t_runs.p);
    hipLaunchKernelGGL(tiles_kernel, dim3(blocks_for(T)), dim3(kB), 0, s, w.first_entry, w.users_t, w.recs_t, w.rec_at,
                       w.head, w.rid, w.pscan, n, T, nw, ld, pl->t_tiles.p, pl->t_runs.p, pl->t_streams.p, w.stats);
    RS_HIP(hipGetLastError());
    RS_HIP(hipMemcpyAsync(h + 3, w.stats + 3, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    RS_HIP(hipStreamSynchronize(s));
    const size_t lds = static_cast<size_t>(h[3]);
    tmark("emit");
    if (lds > kTileLdsBudget) {  // (the t_* buffers are rebuilt by the host build)
        if (trace) std::fprintf(stderr, "sched-dev fallback: largest tile %zu B of LDS\n", lds);
        return false;
    }

    pl->n_tiles = T;
    pl->tile_grid = std::max(1, std::min(grid0, T));
    {
        const int64_t dcold = cold_degree_used(pl->cold_runs, n, ni, pl->tile_grid, nw);
        pl->tile_cold = dcold > 0;
        if (dcold > 0 && h[4] > 0)
            hipLaunchKernelGGL(cold_runs_kernel, dim3(blocks_for(h[4])), dim3(kB), 0, s, pl->t_runs.p, static_cast<int64_t>(h[4]),
                               w.deg_i, ni, dcold);
        RS_HIP(hipGetLastError());
    }
    pl->tile_lds = std::max<size_t>(lds, 16);
    pl->t_n_runs = h[4];
    pl->t_n_users = n_active;
    pl->t_n_split = 0;
    if (!pl->t_split_rows.p) pl->t_split_rows.alloc(1);
    pl->t_block_tile = {0, T};
    pl->t_block_user = {0, pl->n_users};
    pl->t_block_split = {0, 0};
    pl->t_item_deg.alloc(static_cast<size_t>(std::max(1, ni)));  // the hot-run damping's degrees (sgd_tile.hip)
    RS_HIP(hipMemcpyAsync(pl->t_item_deg.p, w.deg_i, sizeof(int32_t) * ni, hipMemcpyDeviceToDevice, s));
    pl->tile_damp = tile_damp_rule(dmax_i, pl->tile_grid, pl->tile_waves, n);
    const size_t parts = static_cast<size_t>(tile_partials(pl));
    if (pl->partial.n < parts) pl->partial.alloc(parts);
    pl->tiles_built = true;
    return true;
}

void upload_coo_from_csr(rs_svd_plan* pl) {
    const size_t n = static_cast<size_t>(pl->nnz);
    std::vector<int32_t> u(n);
    for (int32_t x = 0; x < pl->n_users; ++x)
        std::fill(u.begin() + pl->h_rowptr[x], u.begin() + pl->h_rowptr[x + 1], x);
    hipStream_t s = pl->ctx->stream;
    pl->coo_users.alloc(std::max<size_t>(1, n));
    pl->coo_items.alloc(std::max<size_t>(1, n));
    pl->coo_vals.alloc(std::max<size_t>(1, n));
    pl->coo_users.upload(u.data(), n, s);
    pl->coo_items.upload(pl->h_cols.data(), n, s);
    pl->coo_vals.upload(pl->h_vals.data(), n, s);
    RS_HIP(hipStreamSynchronize(s));
}

void ensure_host_csr(rs_svd_plan* pl) {
    if (pl->nnz == 0 || !pl->h_cols.empty() || !pl->coo_users.p) return;
    const size_t n = static_cast<size_t>(pl->nnz);
    std::vector<int32_t> u(n), i(n);
    std::vector<float> v(n);
    hipStream_t s = pl->ctx->stream;
    pl->coo_users.download(u.data(), n, s);
    pl->coo_items.download(i.data(), n, s);
    pl->coo_vals.download(v.data(), n, s);
    RS_HIP(hipStreamSynchronize(s));
    std::vector<double> vd(v.begin(), v.end());
    pl->h_rowptr.assign(static_cast<size_t>(pl->n_users) + 1, 0);
    pl->h_cols.resize(n);
    pl->h_vals.resize(n);
    csr_build(pl->nnz, pl->n_users, u.data(), i.data(), vd.data(), 0, pl->h_rowptr.data(), pl->h_cols.data(),
              pl->h_vals.data());
}

}  // namespace rs
