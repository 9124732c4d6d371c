// multi.hip -- item-sharded multi-GPU SGD behind the C-ABI (north_star), the epoch of
// core/svd.go:92-130 over Q sharded by item range, P / b_u / GlobalBias replicated.
//
// Protocol.  Every shard's plan runs the tile schedule in delta mode: P stays
// at the epoch start and the kernel writes dP[u] = w_u (p_u(end) - p_u(start)) (bias column
// included), w_u = the shard's share of u's ratings (a plain sum of shard deltas overshoots for users
// split over shards).  The ranks sum dP and the GlobalBias partials and every rank applies the same
// sum, so the replicated state stays bitwise identical.
//
// Pipelining.  The users are cut into B blocks of consecutive users with near-equal ratings, each
// with its own tiles (rs_svd_plan_set_user_blocks).  Block b's kernel is launched on the compute
// stream; when it ends, the comm stream all-reduces block b's dP rows (RCCL over xGMI, in place) and
// applies them to P while the compute stream runs block b + 1 -- block b + 1 touches other P rows,
// and the shard's own Q rows never leave the device.  Only the last block's all-reduce and the
// GlobalBias fold are exposed at the epoch boundary (the next epoch's kernels read the new
// GlobalBias).  RCCL is limited to kCommCTAs workgroups and the tile launch leaves that many CUs free,
// so the collective's kernels run beside the SGD kernel instead of queueing behind its 160-KiB-LDS
// workgroups.
//
// Two exchanges share this code: RCCL (ncclComm per rank: rs_svd_plan_join for one process per GPU,
// rs_svd_group_create for one process driving several GPUs) and an in-process host-barrier exchange
// for shards that share a device (tests; no overlap: a fixed-order sum over the shards' buffers).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "sgd_plan.hpp"

namespace rs {

constexpr int kMaxLocal = 16;  // shards of one in-process exchange

struct LocalGroup {  // host-barrier exchange between the shards of one process
    int n = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool failed = false;
    std::vector<float*> dP;
    std::vector<double*> gbs;
    void barrier() {
        std::unique_lock<std::mutex> l(m);
        if (failed) throw std::runtime_error("another shard of the group failed");
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != g || failed; });
            if (failed) throw std::runtime_error("another shard of the group failed");
        }
    }
    void fail() {
        std::lock_guard<std::mutex> l(m);
        failed = true;
        cv.notify_all();
    }
};

struct ShardComm {
    int rank = 0, nranks = 1, device = 0;
    ncclComm_t nccl = nullptr;
    bool own_nccl = true;
    std::shared_ptr<LocalGroup> local;
    hipStream_t cs = nullptr;  // comm stream (RCCL exchange)
    hipEvent_t ev_epoch = nullptr;
    std::vector<hipEvent_t> ev_done;
    DevBuf<float> dP, sum;      // n_users x ldd; sum: the in-process exchange's result
    DevBuf<double> gbs, gbs_sum;  // per block
    int32_t ldd = 0;
    double total_nnz = 0.0;
    ~ShardComm() {
        (void)hipSetDevice(device);
        if (cs) (void)hipStreamSynchronize(cs);
        if (nccl && own_nccl) (void)ncclCommDestroy(nccl);
        for (hipEvent_t e : ev_done) (void)hipEventDestroy(e);
        if (ev_epoch) (void)hipEventDestroy(ev_epoch);
        if (cs) (void)hipStreamDestroy(cs);
    }
};

namespace {

void check_nccl(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

int32_t comm_ctas() {
    static const int v = std::getenv("RSGPU_COMM_CTAS") ? std::atoi(std::getenv("RSGPU_COMM_CTAS")) : 32;
    return std::max(1, std::min(v, 128));
}

// P rows [u0, u1) += the summed deltas (row stride ldd, k + 1 columns: factors and the bias)
__global__ __launch_bounds__(256) void apply_rows_kernel(float* __restrict__ P, const float* __restrict__ D,
                                                         int64_t n, int32_t ld, int32_t ldd, int32_t kf) {
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; t < n;
         t += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t u = t / ldd;
        const int32_t c = static_cast<int32_t>(t - u * ldd);
        if (c <= kf) P[u * ld + c] += D[t];
    }
}

struct Srcs {
    const float4* p[kMaxLocal];
    const double* g[kMaxLocal];
};

// in-process exchange: out = sum over the shards in shard order (every shard gets the same bits)
__global__ __launch_bounds__(256) void local_sum_kernel(Srcs src, int32_t n_src, int64_t off4, int64_t n4,
                                                        float4* __restrict__ out, int32_t blk,
                                                        double* __restrict__ gout) {
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; t < n4;
         t += static_cast<int64_t>(gridDim.x) * 256) {
        float4 a = src.p[0][off4 + t];
        for (int32_t r = 1; r < n_src; ++r) {
            const float4 b = src.p[r][off4 + t];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        out[off4 + t] = a;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        double g = src.g[0][blk];
        for (int32_t r = 1; r < n_src; ++r) g += src.g[r][blk];
        gout[blk] = g;
    }
}

// GlobalBias after the epoch: gb += sum_b gbs[b] / total ratings (fixed order)
__global__ void gb_fold_blocks_kernel(double* __restrict__ gb, const double* __restrict__ gbs, int32_t nb,
                                      double inv_total) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double t = 0.0;
        for (int32_t b = 0; b < nb; ++b) t += gbs[b];
        gb[0] += t * inv_total;
    }
}

int grid_for(int64_t n) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(4096, (n + 255) / 256))); }

int32_t auto_blocks(const rs_svd_plan* pl, int32_t nranks, int32_t ldd) {
    if (nranks <= 1) return 1;
    const double bytes = static_cast<double>(pl->n_users) * ldd * 4.0;
    const int32_t b = static_cast<int32_t>(bytes / (256.0 * 1024 * 1024) + 0.5);
    return std::max(2, std::min(32, b));
}

// weights w_u = local / total ratings of u; totals from the caller (host, n_users)
void set_weights(rs_svd_plan* pl, const std::vector<double>& tot) {
    std::vector<float> w(static_cast<size_t>(std::max(1, pl->n_users)), 0.f);
    for (int32_t u = 0; u < pl->n_users; ++u) {
        const double c = static_cast<double>(pl->h_rowptr[u + 1] - pl->h_rowptr[u]);
        w[u] = tot[u] > 0 ? static_cast<float>(c / tot[u]) : 0.f;
    }
    pl->uw.alloc(w.size());
    pl->uw.upload(w.data(), w.size(), pl->ctx->stream);
    RS_HIP(hipStreamSynchronize(pl->ctx->stream));
}

// buffers, blocks and (RCCL) the comm stream of a shard whose comm / local group is set; tot: every
// user's ratings over all shards (the user blocks must be the same on every shard)
void shard_setup(rs_svd_plan* pl, ShardComm& c, int32_t n_blocks, const std::vector<double>& tot) {
    if (pl->write_back != RS_SGD_WB_TILE)
        throw std::invalid_argument("the item-sharded epoch runs the tile schedule (RS_SGD_WB_TILE)");
    c.device = pl->ctx->device;
    c.ldd = round_up4(pl->k + 1);
    pl->tile_ublocks = n_blocks > 0 ? n_blocks : auto_blocks(pl, c.nranks, c.ldd);
    std::vector<int64_t> cum(static_cast<size_t>(pl->n_users) + 1, 0);
    for (int32_t u = 0; u < pl->n_users; ++u) cum[u + 1] = cum[u] + static_cast<int64_t>(tot[u]);
    pl->ublock_bounds = user_block_bounds(cum.data(), pl->n_users, std::max(1, std::min(pl->tile_ublocks, std::max(1, pl->n_users))));
    if (c.nccl && c.nranks > 1 && pl->tile_wg == 0) {  // leave CUs to the collective's workgroups
        int cus = 0;
        RS_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device));
        pl->tile_wg = std::max(1, cus - comm_ctas());
    }
    tile_build(pl);
    const int32_t nb = static_cast<int32_t>(pl->t_block_tile.size()) - 1;
    c.dP.alloc(static_cast<size_t>(std::max(1, pl->n_users)) * c.ldd);
    RS_HIP(hipMemsetAsync(c.dP.p, 0, c.dP.n * sizeof(float), pl->ctx->stream));
    c.gbs.alloc(static_cast<size_t>(nb));
    if (c.local) {
        c.sum.alloc(c.dP.n);
        c.gbs_sum.alloc(static_cast<size_t>(nb));
    }
    if (c.nccl) {
        RS_HIP(hipStreamCreateWithFlags(&c.cs, hipStreamNonBlocking));
        RS_HIP(hipEventCreateWithFlags(&c.ev_epoch, hipEventDisableTiming));
        c.ev_done.resize(static_cast<size_t>(nb), nullptr);
        for (hipEvent_t& e : c.ev_done) RS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    RS_HIP(hipStreamSynchronize(pl->ctx->stream));
}

}  // namespace

// n_epochs of the item-sharded schedule on stream s (every rank calls it with the same arguments)
void epochs_sharded(rs_svd_plan* pl, int32_t n_epochs, float lr, float reg, hipStream_t s) {
    ShardComm& c = *pl->shard;
    if (!pl->tiles_built) tile_build(pl);
    const int32_t nb = static_cast<int32_t>(pl->t_block_tile.size()) - 1;
    if (static_cast<int32_t>(c.gbs.n) != nb) throw std::logic_error("user blocks changed after the join");
    const double inv_total = c.total_nnz > 0 ? 1.0 / c.total_nnz : 0.0;
    RS_HIP(hipEventRecord(pl->ev0, s));
    q_convert(pl, s, 1);
    for (int32_t e = 0; e < n_epochs; ++e) {
        for (int32_t b = 0; b < nb; ++b) {
            const int32_t u0 = pl->t_block_user[b], u1 = pl->t_block_user[b + 1];
            const int64_t off = static_cast<int64_t>(u0) * c.ldd, n = static_cast<int64_t>(u1 - u0) * c.ldd;
            if (n > 0) RS_HIP(hipMemsetAsync(c.dP.p + off, 0, n * sizeof(float), s));  // users absent here
            const int32_t parts = tile_launch_range(pl, lr, reg, s, c.dP.p, c.ldd, pl->t_block_tile[b],
                                                    pl->t_block_tile[b + 1]);
            gb_sum(pl->partial.p, parts, c.gbs.p + b, s);
            if (c.nccl) {
                RS_HIP(hipEventRecord(c.ev_done[b], s));
                RS_HIP(hipStreamWaitEvent(c.cs, c.ev_done[b], 0));
                check_nccl(ncclGroupStart(), "ncclGroupStart");
                if (n > 0)
                    check_nccl(ncclAllReduce(c.dP.p + off, c.dP.p + off, static_cast<size_t>(n), ncclFloat32, ncclSum,
                                             c.nccl, c.cs), "ncclAllReduce(dP)");
                check_nccl(ncclAllReduce(c.gbs.p + b, c.gbs.p + b, 1, ncclFloat64, ncclSum, c.nccl, c.cs),
                           "ncclAllReduce(GlobalBias)");
                check_nccl(ncclGroupEnd(), "ncclGroupEnd");
                if (n > 0)
                    hipLaunchKernelGGL(apply_rows_kernel, dim3(grid_for(n)), dim3(256), 0, c.cs, pl->P.p + static_cast<int64_t>(u0) * pl->ld,
                                       c.dP.p + off, n, pl->ld, c.ldd, pl->k);
            } else {
                LocalGroup& g = *c.local;
                RS_HIP(hipStreamSynchronize(s));
                g.barrier();  // every shard's block b is in its dP
                Srcs src{};
                for (int r = 0; r < g.n; ++r) {
                    src.p[r] = reinterpret_cast<const float4*>(g.dP[r]);
                    src.g[r] = g.gbs[r];
                }
                hipLaunchKernelGGL(local_sum_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s, src, g.n, off / 4, n / 4,
                                   reinterpret_cast<float4*>(c.sum.p), b, c.gbs_sum.p);
                RS_HIP(hipGetLastError());
                RS_HIP(hipStreamSynchronize(s));
                g.barrier();  // every shard has read block b of every dP
                if (n > 0)
                    hipLaunchKernelGGL(apply_rows_kernel, dim3(grid_for(n)), dim3(256), 0, s, pl->P.p + static_cast<int64_t>(u0) * pl->ld,
                                       c.sum.p + off, n, pl->ld, c.ldd, pl->k);
            }
            RS_HIP(hipGetLastError());
        }
        if (c.nccl) {
            hipLaunchKernelGGL(gb_fold_blocks_kernel, dim3(1), dim3(64), 0, c.cs, pl->gb.p, c.gbs.p, nb, inv_total);
            RS_HIP(hipEventRecord(c.ev_epoch, c.cs));
            RS_HIP(hipStreamWaitEvent(s, c.ev_epoch, 0));  // the next epoch reads P and the new GlobalBias
        } else {
            hipLaunchKernelGGL(gb_fold_blocks_kernel, dim3(1), dim3(64), 0, s, pl->gb.p, c.gbs_sum.p, nb, inv_total);
        }
        RS_HIP(hipGetLastError());
    }
    q_convert(pl, s, 0);
    RS_HIP(hipEventRecord(pl->ev1, s));
    pl->last_launches = n_epochs;  // rs_svd_plan_last_kernel_ms: the call's device span per epoch
    pl->last_stream = s;
    pl->last_ms = -1.0;
}

}  // namespace rs

struct rs_svd_group {
    std::vector<rs_svd_plan*> plans;
    std::shared_ptr<rs::LocalGroup> local;
};

namespace {

using rs::ShardComm;

// one process, several shards: RCCL when every shard has its own device, else the in-process exchange
void group_join(rs_svd_group* g, int32_t n_blocks) {
    const int n = static_cast<int>(g->plans.size());
    std::vector<int> devs;
    for (rs_svd_plan* pl : g->plans) devs.push_back(pl->ctx->device);
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (!distinct && n > rs::kMaxLocal) throw std::invalid_argument("at most 16 shards share devices");
    // user weights and the total from the shards' host CSRs (no collective needed in one process)
    const int32_t nu = g->plans[0]->n_users;
    std::vector<double> tot(static_cast<size_t>(std::max(1, nu)), 0.0);
    double total = 0.0;
    for (rs_svd_plan* pl : g->plans) {
        if (pl->n_users != nu || pl->k != g->plans[0]->k)
            throw std::invalid_argument("shards must have the same users and n_factors");
        for (int32_t u = 0; u < nu; ++u) tot[u] += static_cast<double>(pl->h_rowptr[u + 1] - pl->h_rowptr[u]);
        total += static_cast<double>(pl->nnz);
    }
    std::vector<ncclComm_t> comms(static_cast<size_t>(n), nullptr);
    if (distinct) {
        ncclUniqueId id;
        rs::check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.maxCTAs = rs::comm_ctas();
        rs::check_nccl(ncclGroupStart(), "ncclGroupStart");
        for (int r = 0; r < n; ++r) {
            RS_HIP(hipSetDevice(devs[r]));
            rs::check_nccl(ncclCommInitRankConfig(&comms[r], n, id, r, &cfg), "ncclCommInitRankConfig");
        }
        rs::check_nccl(ncclGroupEnd(), "ncclGroupEnd");
    } else {
        g->local = std::make_shared<rs::LocalGroup>();
        g->local->n = n;
        for (int a = 0; a < n; ++a)  // peer reads between distinct devices of the group
            for (int b = 0; b < n; ++b)
                if (devs[a] != devs[b]) {
                    RS_HIP(hipSetDevice(devs[a]));
                    hipError_t e = hipDeviceEnablePeerAccess(devs[b], 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) RS_HIP(e);
                    (void)hipGetLastError();
                }
    }
    for (int r = 0; r < n; ++r) {
        rs_svd_plan* pl = g->plans[r];
        RS_HIP(hipSetDevice(devs[r]));
        rs::plan_sync_last(pl);
        auto c = std::make_shared<ShardComm>();
        c->rank = r;
        c->nranks = n;
        c->nccl = comms[r];
        c->local = g->local;
        c->total_nnz = total;
        rs::set_weights(pl, tot);
        rs::shard_setup(pl, *c, n_blocks, tot);
        pl->shard = std::move(c);
    }
    if (g->local) {
        for (rs_svd_plan* pl : g->plans) {
            g->local->dP.push_back(pl->shard->dP.p);
            g->local->gbs.push_back(pl->shard->gbs.p);
        }
    }
}

}  // namespace

extern "C" int rs_comm_unique_id(void* id) {
    if (!id) return rs::set_error(nullptr, RS_ERR_INVALID, "id is NULL");
    return rs_guard(nullptr, [&]() -> int {
        ncclUniqueId u;
        rs::check_nccl(ncclGetUniqueId(&u), "ncclGetUniqueId");
        static_assert(sizeof(u) == RS_COMM_ID_BYTES, "RCCL unique id size");
        std::memcpy(id, &u, sizeof(u));
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_set_user_blocks(rs_svd_plan* pl, int32_t n_blocks, const int32_t* bounds) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    if (n_blocks < 1) return rs::set_error(pl->ctx, RS_ERR_INVALID, "n_blocks must be >= 1");
    if (bounds) {
        if (bounds[0] != 0 || bounds[n_blocks] != pl->n_users)
            return rs::set_error(pl->ctx, RS_ERR_INVALID, "bounds must run from 0 to n_users");
        for (int32_t b = 0; b < n_blocks; ++b)
            if (bounds[b + 1] < bounds[b]) return rs::set_error(pl->ctx, RS_ERR_INVALID, "bounds must not decrease");
    }
    return rs_guard(pl->ctx, [&]() -> int {
        if (pl->shard) return rs::set_error(pl->ctx, RS_ERR_INVALID, "plan is joined to a group (leave first)");
        rs::plan_sync_last(pl);
        pl->tile_ublocks = n_blocks;
        if (bounds) pl->ublock_bounds.assign(bounds, bounds + n_blocks + 1);
        else pl->ublock_bounds.clear();
        if (pl->write_back == RS_SGD_WB_TILE) {
            rs::tile_build(pl);
            pl->n_blocks = rs::tile_partials(pl);
        } else {
            pl->tiles_built = false;
        }
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_join(rs_svd_plan* pl, const void* id, int32_t rank, int32_t n_ranks, int32_t n_blocks) {
    if (!pl || !id) return rs::set_error(pl ? pl->ctx : nullptr, RS_ERR_INVALID, "plan or id is NULL");
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks || n_blocks < 0)
        return rs::set_error(pl->ctx, RS_ERR_INVALID, "bad rank / n_ranks / n_blocks");
    return rs_guard(pl->ctx, [&]() -> int {
        if (pl->shard) return rs::set_error(pl->ctx, RS_ERR_INVALID, "plan already joined");
        if (pl->write_back != RS_SGD_WB_TILE)
            return rs::set_error(pl->ctx, RS_ERR_UNSUPPORTED, "the item-sharded epoch runs the tile schedule");
        rs::plan_sync_last(pl);
        auto c = std::make_shared<ShardComm>();
        c->rank = rank;
        c->nranks = n_ranks;
        c->device = pl->ctx->device;
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.maxCTAs = rs::comm_ctas();
        rs::check_nccl(ncclCommInitRankConfig(&c->nccl, n_ranks, u, rank, &cfg), "ncclCommInitRankConfig");
        // per-user rating counts and the total over all shards (one all-reduce each)
        hipStream_t s = pl->ctx->stream;
        const int32_t nu = pl->n_users;
        std::vector<double> cnt(static_cast<size_t>(std::max(1, nu)), 0.0);
        for (int32_t u2 = 0; u2 < nu; ++u2) cnt[u2] = static_cast<double>(pl->h_rowptr[u2 + 1] - pl->h_rowptr[u2]);
        cnt.push_back(static_cast<double>(pl->nnz));
        rs::DevBuf<double> d(cnt.size());
        d.upload(cnt.data(), cnt.size(), s);
        rs::check_nccl(ncclAllReduce(d.p, d.p, cnt.size(), ncclFloat64, ncclSum, c->nccl, s), "ncclAllReduce(counts)");
        d.download(cnt.data(), cnt.size(), s);
        RS_HIP(hipStreamSynchronize(s));
        c->total_nnz = cnt.back();
        cnt.pop_back();
        rs::set_weights(pl, cnt);
        rs::shard_setup(pl, *c, n_blocks, cnt);
        pl->shard = std::move(c);
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_leave(rs_svd_plan* pl) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        rs::plan_sync_last(pl);
        pl->shard.reset();  // the tiles keep the group's blocks until the next rs_svd_plan_set_user_blocks
        return RS_OK;
    });
}

extern "C" int rs_svd_plan_epochs_sharded(rs_svd_plan* pl, int32_t n_epochs, float lr, float reg, void* stream) {
    if (!pl) return rs::set_error(nullptr, RS_ERR_INVALID, "plan is NULL");
    return rs_guard(pl->ctx, [&]() -> int {
        if (!pl->shard) return rs::set_error(pl->ctx, RS_ERR_INVALID, "plan is not joined (rs_svd_plan_join)");
        if (n_epochs < 0) return rs::set_error(pl->ctx, RS_ERR_INVALID, "n_epochs < 0");
        if (pl->shard->local) return rs::set_error(pl->ctx, RS_ERR_INVALID, "group shards run through rs_svd_group_epochs");
        rs::epochs_sharded(pl, n_epochs, lr, reg, stream ? static_cast<hipStream_t>(stream) : pl->ctx->stream);
        return RS_OK;
    });
}

extern "C" int rs_svd_group_create(rs_svd_plan* const* plans, int32_t n, int32_t n_blocks, rs_svd_group** out) {
    if (!plans || !out || n < 1 || n_blocks < 0) return rs::set_error(nullptr, RS_ERR_INVALID, "bad group arguments");
    *out = nullptr;
    for (int32_t r = 0; r < n; ++r)
        if (!plans[r] || plans[r]->shard) return rs::set_error(nullptr, RS_ERR_INVALID, "NULL or already joined plan");
    auto* g = new rs_svd_group();
    g->plans.assign(plans, plans + n);
    const int st = rs_guard(nullptr, [&]() -> int {
        group_join(g, n_blocks);
        return RS_OK;
    });
    if (st != RS_OK) {
        for (rs_svd_plan* pl : g->plans) {
            (void)hipSetDevice(pl->ctx->device);
            pl->shard.reset();
        }
        delete g;
        return st;
    }
    *out = g;
    return RS_OK;
}

extern "C" int rs_svd_group_epochs(rs_svd_group* g, int32_t n_epochs, float lr, float reg) {
    if (!g || n_epochs < 0) return rs::set_error(nullptr, RS_ERR_INVALID, "bad group arguments");
    const size_t n = g->plans.size();
    std::vector<std::string> errs(n);
    std::vector<std::thread> th;
    for (size_t r = 0; r < n; ++r)
        th.emplace_back([&, r] {  // one host thread per shard
            rs_svd_plan* pl = g->plans[r];
            try {
                RS_HIP(hipSetDevice(pl->ctx->device));
                rs::epochs_sharded(pl, n_epochs, lr, reg, pl->ctx->stream);
                RS_HIP(hipStreamSynchronize(pl->ctx->stream));
            } catch (const rs::HipError& e) {
                errs[r] = e.what;
            } catch (const std::exception& e) {
                errs[r] = e.what();
            }
            if (!errs[r].empty() && g->local) g->local->fail();
        });
    for (std::thread& t : th) t.join();
    for (size_t r = 0; r < n; ++r)
        if (!errs[r].empty()) return rs::set_error(g->plans[r]->ctx, RS_ERR_HIP, "shard " + std::to_string(r) + ": " + errs[r]);
    return RS_OK;
}

extern "C" void rs_svd_group_destroy(rs_svd_group* g) {
    if (!g) return;
    for (rs_svd_plan* pl : g->plans) {
        (void)hipSetDevice(pl->ctx->device);
        if (pl->last_stream) (void)hipStreamSynchronize(pl->last_stream);
        pl->shard.reset();
    }
    delete g;
}

// Item ranges of near-equal ratings (contiguous inner item ids): shard r owns [bounds[r], bounds[r+1]).
extern "C" int rs_item_shards(int64_t nnz, const int32_t* items, int32_t n_items, int32_t n_shards, int32_t* bounds) {
    if ((nnz > 0 && !items) || !bounds || n_items < 0 || n_shards < 1)
        return rs::set_error(nullptr, RS_ERR_INVALID, "bad shard arguments");
    std::vector<int64_t> cnt(static_cast<size_t>(n_items) + 1, 0);
    for (int64_t t = 0; t < nnz; ++t) {
        if (items[t] < 0 || items[t] >= n_items) return rs::set_error(nullptr, RS_ERR_INVALID, "item id out of range");
        cnt[items[t] + 1]++;
    }
    for (int32_t x = 0; x < n_items; ++x) cnt[x + 1] += cnt[x];
    bounds[0] = 0;
    for (int32_t r = 1; r < n_shards; ++r) {
        const int64_t want = nnz * r / n_shards;
        const int32_t b = static_cast<int32_t>(std::lower_bound(cnt.begin(), cnt.end(), want) - cnt.begin());
        bounds[r] = std::max(bounds[r - 1], std::min(b, n_items));
    }
    bounds[n_shards] = n_items;
    return RS_OK;
}

extern "C" int rs_svd_fit_multi(const int32_t* devices, int32_t n_devices, const rs_ratings* r,
                                const rs_sgd_params* p, int32_t n_blocks, double* P, double* Q, double* bu,
                                double* bi, double* gb) {
    if (!devices || n_devices < 1 || !r || !p || !P || !Q || !bu || !bi || !gb || n_blocks < 0)
        return rs::set_error(nullptr, RS_ERR_INVALID, "bad arguments");
    if (p->mode != RS_SGD_FAST || p->write_back != RS_SGD_WB_TILE)
        return rs::set_error(nullptr, RS_ERR_UNSUPPORTED, "multi-GPU fit runs the FAST tile schedule");
    if (r->nnz < 0 || r->n_users < 0 || r->n_items < 0 || (r->nnz > 0 && (!r->users || !r->items || !r->ratings)))
        return rs::set_error(nullptr, RS_ERR_INVALID, "bad ratings");
    const int32_t n = n_devices, k = p->n_factors;
    std::vector<int32_t> bounds(static_cast<size_t>(n) + 1);
    int st = rs_item_shards(r->nnz, r->items, r->n_items, n, bounds.data());
    if (st != RS_OK) return st;
    std::vector<rs_ctx*> ctxs(n, nullptr);
    std::vector<rs_svd_plan*> plans(n, nullptr);
    rs_svd_group* g = nullptr;
    auto cleanup = [&] {
        if (g) rs_svd_group_destroy(g);
        for (rs_svd_plan* pl : plans) rs_svd_plan_destroy(pl);
        for (rs_ctx* c : ctxs) rs_close(c);
    };
    st = rs_guard(nullptr, [&]() -> int {
        *gb = p->n_epochs > 0 ? rs::gb_warm_start(r, bu, bi) : *gb;  // as rs_svd_fit (FAST)
        for (int32_t s = 0; s < n; ++s) {
            int e = rs_open(devices[s], &ctxs[s]);
            if (e != RS_OK) return e;
            const int32_t lo = bounds[s], hi = bounds[s + 1];
            std::vector<int32_t> su, si;
            std::vector<double> sr;
            for (int64_t t = 0; t < r->nnz; ++t)
                if (r->items[t] >= lo && r->items[t] < hi) {
                    su.push_back(r->users[t]);
                    si.push_back(r->items[t] - lo);
                    sr.push_back(r->ratings[t]);
                }
            rs_ratings sh{static_cast<int64_t>(su.size()), r->n_users, hi - lo, su.data(), si.data(), sr.data()};
            e = rs_svd_plan_create(ctxs[s], &sh, k, &plans[s]);
            if (e != RS_OK) return e;
            e = rs_svd_plan_upload(plans[s], P, Q + static_cast<int64_t>(lo) * k, bu, bi + lo, gb);
            if (e != RS_OK) return e;
        }
        int e = rs_svd_group_create(plans.data(), n, n_blocks, &g);
        if (e != RS_OK) return e;
        e = rs_svd_group_epochs(g, p->n_epochs, static_cast<float>(p->lr), static_cast<float>(p->reg));
        if (e != RS_OK) return e;
        for (int32_t s = 0; s < n; ++s) {  // P, b_u, GlobalBias are identical on every shard: take shard 0's
            const int32_t lo = bounds[s];
            e = rs_svd_plan_download(plans[s], s == 0 ? P : nullptr, Q + static_cast<int64_t>(lo) * k,
                                     s == 0 ? bu : nullptr, bi + lo, s == 0 ? gb : nullptr);
            if (e != RS_OK) return e;
        }
        return RS_OK;
    });
    std::string err = st != RS_OK ? std::string(rs_last_error(nullptr)) : std::string();
    for (int32_t s = 0; s < n && st != RS_OK && err.empty(); ++s)
        if (ctxs[s]) err = rs_last_error(ctxs[s]);
    cleanup();
    if (st != RS_OK) return rs::set_error(nullptr, st, err);
    return RS_OK;
}
