// sgd_plan.hpp -- the device-resident SVD plan shared by sgd.hip (hybrid / direct / ordered
// schedules, C-ABI) and sgd_tile.hip (tile schedule, the FAST default).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <memory>
#include <vector>

#include "common.hpp"
#include "wave.hpp"

namespace rs {
struct ShardComm;  // multi.hip
}

namespace rs {
// Cold runs (sgd_tile.hip, round 6): a run header's item carries kRunCold when the item has so few ratings that
// another run of it is rarely in flight -- R_i = deg_i x workgroups x waves / nnz below cold_runs -- and the run then
// ends with plain write-through stores of its new row (an update of the same item landing in between is lost,
// with probability about R_i) instead of the memory-side atomic unit, which bounds the epoch.
constexpr int32_t kRunCold = 0x40000000, kRunItemMask = 0x3FFFFFFF;  // item ids below 2^30
// 0.05 (round 6, scripts/experiments/exp_cold_store.py, profiles/r06/): configs[4]'s whole set 0.588 -> 0.419 s per
// epoch and its 8-shard QDELTA fit 0.954 -> 0.766 s on one GPU, held-out RMSE unchanged (0.6081 / 0.6174 after 10
// epochs against 0.6079 / 0.6172); the ML-1M epoch unchanged (152 us, 0.6684); 0.2 costs ML-1M 0.003 of RMSE.
constexpr double kColdRunsDefault = 0.05;
// items with fewer ratings than this are cold (0: none); the host and the device schedule builds both use it
inline int64_t cold_degree(double cold_runs, int64_t nnz, int32_t grid, int32_t waves) {
    if (!(cold_runs > 0.0) || nnz <= 0 || grid <= 0 || waves <= 0) return 0;
    return static_cast<int64_t>(std::ceil(cold_runs * static_cast<double>(nnz) / (static_cast<double>(grid) * waves)));
}
// The schedule marks cold runs, and the launch takes the kernel variant with the stores, only where the mean item
// is cold (dcold >= nnz / n_items): the store path costs the ML-1M epoch 8 % even with no run marked (147 -> 159 us:
// one more exit per run; profiles/r06/k1_cold_variant_cost.log), and there runs of cold items are few.  configs[4]
// (whole set and QDELTA shards) is far inside the rule, ML-1M and the 1M-rating stability sets far outside it.
inline int64_t cold_degree_used(double cold_runs, int64_t nnz, int32_t n_items, int32_t grid, int32_t waves) {
    const int64_t d = n_items < kRunCold ? cold_degree(cold_runs, nnz, grid, waves) : 0;
    return d > 0 && d * static_cast<int64_t>(n_items) >= nnz ? d : 0;
}
}  // namespace rs

struct rs_svd_plan {
    rs_ctx* ctx = nullptr;
    int32_t n_users = 0, n_items = 0, k = 0, ld = 0, n_work = 0;
    int64_t nnz = 0;
    std::vector<int64_t> h_rowptr;  // host user-CSR row pointers (work items are rebuilt from it)
    std::vector<int32_t> h_cols;    // host user-CSR item ids (item copies are rebuilt from it)
    rs::DevBuf<int32_t> items;      // user-CSR item rows (copies of split items), padded by 128
    rs::DevBuf<float> ratings;
    rs::DevBuf<int32_t> wk_user;      // work items: user, [begin, end) into the CSR, len / deg
    rs::DevBuf<int64_t> wk_rng;
    rs::DevBuf<float> wk_frac;
    // users with more ratings are split into pieces (0: never).  Default 1200, measured on the ML-1M
    // shape with heavy_min 1000 and fixed-point Q (scripts/experiments/exp_split_sweep.py): epoch 572 -> 491 us,
    // 20-epoch held-out RMSE 0.6676 -> 0.6684 against 0.6683 for the reference visit order
    int32_t split_cap = 1200;
    rs::DevBuf<float> dPs;            // split-user deltas (single GPU), zero between epochs
    rs::DevBuf<int32_t> split_rows;   // users split into pieces
    int32_t n_split = 0;
    int32_t item_cap = 0;             // items with more ratings get row copies (0: never)
    int32_t n_qrows = 0;              // item rows incl. copies (Q holds n_qrows x ld)
    rs::DevBuf<int4> isplit_meta;     // split items: {row, first copy row, copies, frac offset}
    rs::DevBuf<float> isplit_frac;
    int32_t n_isplit = 0;
    rs::DevBuf<float> P, Q;  // bias in column k
    rs::DevBuf<double> gb, partial;
    rs::DevBuf<double> gb_smooth;  // tile epochs: per (workgroup, wave) the smoothed GlobalBias fold's {sum b, sum (1 - a)}
    int32_t gb_fold = RS_GB_FOLD_SMOOTH;  // how a single-GPU tile epoch folds GlobalBias (rs_svd_plan_set_gb_fold)
    rs::DevBuf<float> uw;  // per-user share of this shard (multi-GPU delta mode)
    // hot replicas: most-rated items and copies each (0: none).  Default 256 x 8, measured on the
    // ML-1M shape (scripts/experiments/exp_replicas.py): epoch 760 -> 585 us, held-out RMSE unchanged
    int32_t live_req = 256, live_copies = 8;
    int32_t n_live = 0;
    rs::DevBuf<int4> live_meta;  // {item row, first extra row, copies, -}
    rs::DevBuf<float> qlast;     // last merged value of every live item (n_live x ld)
    rs::DevBuf<int32_t> done;     // blocks finished (the merger's exit condition)
    rs::DevBuf<int32_t> numflag;  // raised by svd_q_fixed_kernel (RS_ERR_NUMERIC at download)
    rs::DevBuf<float> iw;  // per-item share of this shard (user-sharded multi-GPU mode)
    rs::DevBuf<float> Q0;  // Q at the epoch start (user-sharded mode)
    int32_t n_blocks = 0;
    int32_t write_back = RS_SGD_WB_TILE;
    int32_t heavy_min = 1000;  // work items with at least this many ratings get a producer + 3 writers
    int32_t n_heavy = 0;       // leading (LPT-ordered) work items that are heavy
    int32_t light_blocks = 0;  // cap on the light blocks (each wave strides over light items; 0 = none)
    rs::DevBuf<int64_t> trace;  // diagnostic: {start, chain end, drained} per work item (RS_SGD_WB_ATOMIC)
    // q_i prefetch distance of the light waves: 16 since the end of round 1 (ML-1M shape with the
    // default schedule: epoch 435 -> 428 us, held-out RMSE 0.6685 either way; exp_split_sweep.py)
    int32_t ring_depth = 16;
    int32_t fixed_q = 1;           // hybrid epochs keep Q as int32 fixed point (rs_svd_plan_set_fixed_q)
    bool live_merged = false;      // the fixed-point epoch already ran the live items' final round
    bool hoisted = false;          // plan_epochs: Q stays int32 across epochs, the epilogue re-arms done
    double mean_rating = 0.0;  // of the plan's ratings (FAST GlobalBias warm start at init)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0;
    int32_t last_launches = 0;
    bool timing = false;
    hipStream_t last_stream = nullptr;  // stream of the last enqueued epochs (synced before copies)
    std::vector<hipEvent_t> tev;        // timing mode: [2 * epoch] start, [2 * epoch + 1] end
    int32_t tev_used = 0;
    // tile schedule (RS_SGD_WB_TILE, the default; sgd_tile.hip): users cut into tiles whose P rows
    // stay in one workgroup's LDS for the epoch, the tile's ratings grouped into per-item runs
    int32_t tile_wg = 0;      // workgroups of the launch (0 = one per CU)
    int32_t tile_waves = 16;  // waves per workgroup (1, 2, 4, 8 or 16)
    int32_t tile_target = 0;  // ratings per tile (0 = nnz / workgroups, bounded by the LDS)
    int32_t tile_run_cap = 0; // runs longer than this are cut over waves (0 = never)
    int32_t tile_ring = 0;    // q_i rows prefetched per wave (0 = auto: 2)
    int32_t tile_claim = 4;   // runs per claim from the tile's run queue (4 or 8; 0 = runs dealt on the host)
    int32_t n_tiles = 0, tile_grid = 0;
    size_t tile_lds = 0;      // dynamic LDS bytes of the launch (the largest tile)
    bool tiles_built = false, hybrid_built = false;
    std::vector<float> h_vals;  // host user-CSR ratings (the hybrid structures are built lazily)
    rs::DevBuf<int4> t_tiles;   // {first user (into t_users), users, first run, first record}
    rs::DevBuf<int2> t_users;       // tile entries {user, frac bits} (frac < 1: a piece of a split user)
    rs::DevBuf<int32_t> t_streams;  // per tile: waves + 1 run offsets
    rs::DevBuf<int2> t_runs;    // {item, first record (tile-local)}, a sentinel after each tile
    rs::DevBuf<int2> t_recs;    // {user (tile-local), rating bits}
    rs::DevBuf<int32_t> t_split_rows;  // users cut into pieces over several tiles
    rs::DevBuf<int32_t> t_item_deg;    // every item's ratings in the schedule (the hot-run damping, sgd_tile.hip)
    bool tile_damp = false;            // the schedule's hottest item has >= kTileDampRuns runs in flight: damped kernel
    // cold runs (round 6): items with fewer ratings than cold_degree(cold_runs, ...) -- fewer than cold_runs of their
    // runs in flight on average -- end their runs with write-through stores of the new row instead of memory-side
    // atomics (header bit kRunCold); 0 turns it off (rs_svd_plan_set_cold_store)
    double cold_runs = rs::kColdRunsDefault;
    bool tile_cold = false;  // the schedule marks cold runs (rs::cold_degree_used): the launch takes the store variant
    float damp_kconc = 0.f;            // test hook (rs_svd_plan_set_damp_concurrency): > 0 forces the damped kernel with
                                       // runs in flight R = deg x damp_kconc instead of deg x workgroups x waves / nnz
    int32_t t_n_split = 0;
    int64_t t_n_runs = 0, t_n_users = 0;  // entries of t_runs / t_users in use (the buffers may be larger)
    // user blocks: consecutive user ranges of near-equal ratings, each with its own tiles (tiles
    // [t_block_tile[b], t_block_tile[b+1]) hold users [t_block_user[b], t_block_user[b+1])); the
    // item-sharded multi-GPU epoch all-reduces a block's user deltas while the next block computes
    int32_t tile_ublocks = 1;
    int32_t tile_user_lds = 0;  // LDS ints per user (0 = one row of k + 2)
    std::vector<int32_t> ublock_bounds;  // caller's block bounds (tile_ublocks + 1), or empty: own ratings
    std::vector<int32_t> t_block_tile, t_block_user;
    // item blocks (RS_EXCHANGE_ROTATE_Q, multi.hip): when set (n_blocks + 1 item ids from 0 to n_items) the
    // tiles are built per stratum -- block b's tiles hold this plan's ratings of items
    // [iblock_bounds[b], iblock_bounds[b+1]) over all its users -- instead of per user block
    std::vector<int32_t> iblock_bounds;
    // hot items of a ROTATE_Q shard (multi.hip): a stratum concentrates an item's ratings n_blocks-fold, and a
    // Zipf head then holds a large share of one stratum's runs in flight at once (Hogwild staleness beyond
    // what lr tolerates).  Each hot item gets one row copy per item block (rows n_items + b * H + h, h < H),
    // its ratings dealt to the copies by user hash, and the copies are averaged once per epoch.
    std::vector<int32_t> hot_items;      // canonical ids (H = size)
    rs::DevBuf<int32_t> hot_rows;        // the same on the device
    std::vector<int2> hot_meta_h;        // per hot item {natural block, copies in use}
    rs::DevBuf<int2> hot_meta;
    double hot_share = 0.02;             // an item is hot above this share of its stratum's ratings ...
    int64_t hot_min_stratum = int64_t{1} << 17;  // ... when strata hold at least this many ratings (0 share: off)
    int32_t hot_merge = RS_HOT_SCALED;  // how the copies merge once per epoch
    std::vector<double> hot_count;       // every hot item's ratings over all ranks
    std::vector<int32_t> t_block_split;  // block b's split users: t_split_rows[t_block_split[b], t_block_split[b+1])
    std::shared_ptr<rs::ShardComm> shard;  // item-sharded multi-GPU state (multi.hip), or empty
    int32_t exchange = RS_EXCHANGE_ROTATE;  // the multi-GPU exchange a join sets up
    int32_t qdelta_wire = 16;               // QDELTA: bits per item move on the wire (16: fp16, 32: int32 fixed point)
    double qdelta_hot = 4.0;                // QDELTA: ratings per rank and block that make an item hot (<= 0: all hot)
    int32_t qdelta_cold_every = 2;          // QDELTA: most blocks between a cold item's merges (multi.hip kQdelta*)
    // QDELTA: curvature of the factor columns' merge weights, a = 1 - lr x this (the bias column: 1).  configs[4], 8
    // shards, 10 / 20 epochs against the whole-set fit's 0.6081 / 0.5901 (profiles/r06/config4_qdelta_curvature*.log):
    // 1 -> 0.6174 / 0.5918, 0.5 -> 0.6147, 0.25 -> 0.6127 / 0.5910, 0.1 left the fixed-point range
    double qdelta_curv = 0.25;
    int32_t fault_sub_epoch = -1;  // test hook (rs_svd_plan_inject_fault): the next sharded call throws there
    // how tiles are formed (rs_svd_plan_set_tile_rule): RS_TILE_RULE_LPT (host: LPT by ratings + cost
    // refinement), RS_TILE_RULE_FILL (host: users by degree dealt boustrophedon), RS_TILE_RULE_FILL_DEVICE
    // (the same rule built on the device from coo_*; one-shot rs_svd_fit's default)
    int32_t tile_rule = RS_TILE_RULE_LPT;
    rs::DevBuf<int32_t> coo_users, coo_items;  // device COO of a device-built schedule (any rating order)
    rs::DevBuf<float> coo_vals;
    rs::DevBuf<char> sched_ws;                 // its build workspace (kept for refits)
    std::function<void()> build_overlap;       // host work run (once) while the device build's kernels execute
    // divergence guard of the tile schedule (rs_svd_plan_set_guard, default on): a call's epochs that leave the
    // fixed-point range, go non-finite, raise the training loss or pass the guard bound are redone from the
    // call-start state on a quarter of the workgroups and half the run cap (sgd.hip plan_epochs).  Memory: the
    // snapshot is a second resident copy of P and Q (allocated on a guarded plan's first call), and every
    // guarded call ends in one small readback the host waits for.
    int32_t guard = 1;
    int32_t refits = 0;                        // redone calls so far (rs_svd_plan_refits)
    rs::DevBuf<float> P_snap, Q_snap;          // the call-start state (allocated on first use)
    rs::DevBuf<double> gb_snap;                // {GlobalBias, loss state} at the call start
    rs::DevBuf<float> loss_part;               // per (workgroup, wave): sum of (lr diff)^2 of the last epoch
    rs::DevBuf<double> loss_state;             // last epoch's training MSE (0: none since the factors were set)
    rs::DevBuf<int32_t> guard_flag;            // the guard's own signals (a rising loss, |p| or |q| >= guard bound): redo, not an error
    int32_t soft_refits = 0;                   // redos the guard's own signals alone asked for (the grid is restored after them)
    bool tiles_deferred = false;               // a soft redo restored the caller's grid: rebuilt by the next epochs call
    int32_t own_fx_shift = -1, own_tile_wg = -1;  // while joined: the plan's own shift and grid (rs_svd_plan_leave restores them)
    // Fixed-point scale of the FAST schedules: P / Q values are held as int32 round(v * 2^fx_shift)
    // while a call runs, so |v| < 2^(31 - fx_shift).  The shift follows the ratings (fx_shift_for): 24 (|v| < 128)
    // on star scales, fewer bits of fraction where the biases must reach further (1-100 ratings: 20, |v| < 2048).
    int32_t fx_shift = 24;
    float fx() const { return static_cast<float>(1u << fx_shift); }
    float fx_inv() const { return 1.f / fx(); }
    float fx_range() const { return static_cast<float>(1u << (31 - fx_shift)); }  // |v| must stay below
    float guard_bound() const { return fx_range() / 4.f; }                        // the guard's range scan
    ~rs_svd_plan() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        for (hipEvent_t e : tev) (void)hipEventDestroy(e);
    }
};

namespace rs {
constexpr int32_t kOutOfRange = 0x7FFFFFF0;  // buffer offset past num_records: load 0 / drop store
constexpr int kSgdAux = 16;                  // sc1
// Fixed-point rows: 2^-fx_shift resolution, |v| < 2^(31 - fx_shift); fx_shift from the ratings (below)
// The plan's fixed-point shift for ratings in [lo, hi] with mean m: a bias moves a rating by at most about
// d = max(hi - m, m - lo) and a factor product by less, so the range is 32 U with U = 2^ceil(log2(max(d, 4))):
// 2^-24 resolution and |v| < 128 on star scales (d <= 4, as before round 5), 2^-20 / 2048 for 1-100 ratings.
// The guard's range scan sits at a quarter of that (8 U: 32 on stars).
inline int32_t fx_shift_for(double lo, double hi, double mean) {
    const double d = std::max({hi - mean, mean - lo, 4.0});
    if (!(d < 1e30)) return 8;
    int32_t lg = 0;
    while (lg < 16 && static_cast<double>(int64_t{1} << lg) < d) ++lg;
    return std::max(8, std::min(24, 26 - lg));
}

// Sum over the 64 lanes of a wave: DPP inside each 16-lane row, then the gfx950 permlane swaps
// across rows.  Every lane ends with the bitwise-identical total.
__device__ __forceinline__ float wave_sum(float x) {
    x = group_sum<16>(x);
    auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
    auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

// Fixed-point item rows (rs_svd_plan_set_fixed_q): during a hybrid FAST epoch Q holds
// round(q * 2^s) as int32 (s = the plan's fx_shift) and the q_i deltas are integer atomics.  Measured on gfx950
// (scripts/experiments/exp_atomics.hip, exp_atomics2.hip): memory-side u32 atomic adds sustain 1.69 TB/s of
// added bytes against 1.32 TB/s for f32 -- and the epoch is bound by that rate.  At s = 24 (star ratings) the
// resolution 2^-24 is the fp32 ulp at |q| in [0.5, 1); the range is |q| < 2^(31-s) (v_cvt_i32_f32 saturates).
// Integer adds are exact and associative, so the sum of the deltas no longer depends on their order.
__device__ __forceinline__ float fx_to_f(uint32_t bits, float fx_inv) { return static_cast<float>(static_cast<int32_t>(bits)) * fx_inv; }
__device__ __forceinline__ int32_t fx_delta(float qn, float q, float fx) { return __float2int_rn((qn - q) * fx); }

// Row layout of the FAST plan: lane l's register x holds column l + 64 x, except lane 63's last
// register, which holds the bias in column kf (right after the kf factors).  The other lanes of the
// last register whose column is >= kf are padding: never loaded (they read 0) and never written, so
// the 64-B lines past column kf get no memory request at all -- row atomics are priced per 64-B line,
// not per dword (scripts/experiments/exp_atomics2.hip: 1.69 -> 1.93 TB/s of row bytes with one line of eight
// masked off); k = 100 rows take 7 line requests instead of 8.
template <int E>
__device__ __forceinline__ int32_t last_col(int lane, int32_t kf) {  // column of register E-1, or -1
    const int32_t c = lane == 63 ? kf : lane + 64 * (E - 1);
    return (lane == 63 || c < kf) ? c : -1;
}
// byte offset of register x of this lane in the row at byte offset `row` (kOutOfRange: padding)
template <int E>
__device__ __forceinline__ int32_t roff(int32_t row, int x, int32_t lane4, int32_t lc) {
    return x < E - 1 ? row + lane4 + 256 * x : (lc >= 0 ? row + 4 * lc : kOutOfRange);
}

__device__ __forceinline__ float lane63(float x) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

// byte size of a buffer the kernels address through a buffer resource with 32-bit offsets (the row
// offsets are int32 too): 2 GiB or more is rejected instead of silently dropping loads and atomics
inline int32_t buffer_bytes32(size_t elems, size_t elem_size, const char* what) {
    const size_t b = elems * elem_size;
    if (b >= (size_t{1} << 31))
        throw std::invalid_argument(std::string(what) + " of 2 GiB or more: beyond the kernels' 32-bit buffer offsets");
    return static_cast<int32_t>(b);
}

// sgd.hip
int32_t fast_ld(int32_t k);            // row stride of the FAST plans (k factors + bias, 64-float lines)
void plan_sync_last(rs_svd_plan* pl);  // waits for the stream of the last enqueued epochs
bool plan_range_ok(rs_svd_plan* pl);   // P and Q finite and below the guard bound (syncs the stream)
int32_t* numflag(rs_svd_plan* pl);  // the RS_ERR_NUMERIC device flag (allocated on first use)
void q_convert(rs_svd_plan* pl, hipStream_t s, int32_t to_fixed);  // Q <-> int32 fixed point in place
void gb_sum(const double* partial, int64_t n, double* out, hipStream_t s);  // fixed-order sum
// split users t_split_rows[r0, r1) of the tile schedule: P += dPs, dPs = 0 (the pieces' merge)
void merge_tile_split_rows(rs_svd_plan* pl, int32_t r0, int32_t r1, hipStream_t s);

// sgd_ordered.hip: RS_SGD_ORDERED epochs, one workgroup over conflict-free batches, rows of ld floats in the folded layout
// P [p_0 .. p_{k-1}, b_u, 1, 0 ..], Q [q_0 .. q_{k-1}, 1, b_i, 0 ..] (ld % 4 == 0, k + 2 <= ld <= 512);
// the id / rating arrays allocated for ordered_padded(nnz) entries
int64_t ordered_padded(int64_t nnz);
// the batched ORDERED kernel's schedule: batch starts (n_batches + 1 offsets; no user or item twice in a
// batch, at most wmax ratings) and per rating the slots of the previous batch that wrote its rows
struct OrderedSchedule {
    std::vector<int64_t> start;
    std::vector<int32_t> fwd;
};
OrderedSchedule ordered_batches(const int32_t* users, const int32_t* items, int64_t nnz, int32_t n_users,
                                int32_t n_items, int32_t wmax);
int32_t ordered_wmax(int32_t ld);  // the kernel's batch size limit for rows of ld floats
void ordered_epochs(const int32_t* users, const int32_t* items, const float* ratings, const int32_t* fwd,
                    int64_t nnz, const int64_t* bstart, int64_t n_batches, float* P, int64_t p_floats, float* Q,
                    int64_t q_floats, int32_t ld, int32_t kf, double* gb, int32_t epochs, float lr, float reg,
                    hipStream_t s);

// sgd_tile.hip
constexpr size_t kTileLdsBudget = 160 * 1024 - 512;  // gfx950: 160 KiB of LDS per workgroup
// LDS ints per tile user (k factors + two bias columns, or the caller's tile_user_lds)
inline int32_t tile_lds_row(const rs_svd_plan* pl) {
    return pl->tile_user_lds > 0 ? pl->tile_user_lds : 64 * ((pl->k + 2 + 63) / 64);
}
// LDS bytes of a tile: P rows, records, run headers + sentinel (ld: the LDS row)
inline size_t tile_bytes(int64_t users, int64_t recs, int64_t runs, int32_t ld) {
    return static_cast<size_t>(users) * ld * 4 + static_cast<size_t>(recs) * 8 + static_cast<size_t>(runs + 1) * 8;
}
// Queue key of item `item`'s run in tile `tile`: runs are queued in key order, a per-tile pseudo-random
// item order.  fmix32 (murmur3's finaliser) of item ^ salt(tile) is a bijection of the item id, so no two
// items of a tile share a key and the order needs no tie rule (host and device builds agree by construction).
__host__ __device__ inline uint32_t run_key(int32_t item, int32_t tile) {
    uint32_t x = static_cast<uint32_t>(item) ^ (static_cast<uint32_t>(tile) * 0x9E3779B1u);
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}
constexpr int32_t kFillSnakeRounds = 4;  // RS_TILE_RULE_FILL: boustrophedon rounds before the deficit fill
int32_t device_cus(const rs_ctx* ctx);
int32_t tile_grid0(const rs_svd_plan* pl);
// Hot-run damping (sgd_tile.hip) where the hottest item's runs in flight -- deg x workgroups x waves / nnz --
// reach this many
constexpr double kTileDampRuns = 40.0;
inline bool tile_damp_rule(int64_t dmax, int32_t grid, int32_t waves, int64_t nnz) {
    return nnz > 0 && static_cast<double>(dmax) * grid * waves / static_cast<double>(nnz) >= kTileDampRuns;
}  // the tile launch's workgroups (tile_wg, or the library's choice)
// the run cap the library picks (see auto_run_cap, sgd_tile.hip) from the item degree maximum
int32_t run_cap_rule(int64_t nnz, int64_t dmax_item, int32_t grid, int32_t waves, int32_t k);
void tile_build(rs_svd_plan* pl);  // (re)builds the tile schedule (host CSR, or the device for RS_TILE_RULE_FILL_DEVICE)
std::vector<int32_t> user_block_bounds(const int64_t* cum, int32_t n_users, int32_t nb);
void tile_launch(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP);  // one epoch (Q int32)
// tiles [t0, t1) only (one user block), delta mode into dP (row stride ldd); returns the number of
// GlobalBias partials written to pl->partial
int32_t tile_launch_range(rs_svd_plan* pl, float lr, float reg, hipStream_t s, float* dP, int32_t ldd,
                          int32_t t0, int32_t t1);
int32_t tile_partials(const rs_svd_plan* pl);  // GlobalBias partials the launch writes
int32_t tile_cap_in_use(const rs_svd_plan* pl);  // the run cap the schedule is built with (uncut: the max degree)
// visit order of the tile schedule (user-CSR positions, nnz entries) and its GlobalBias work items
// (one per tile and wave: n_works + 1 offsets into pos); any pointer may be NULL
void tile_order(rs_svd_plan* pl, int64_t* pos, int64_t* work_off, int32_t* n_works);

// sched_dev.hip: the fill-rule tile schedule built on the device from the plan's device COO (coo_*).
// Returns false, with nothing of the plan changed, where the rule does not apply (a user above the LDS
// bound, keys past 64 bits, a tile past the LDS): the caller builds on the host instead.
bool tile_build_device(rs_svd_plan* pl);
// the device COO of a plan built from the host CSR (rows expanded), for tile_build_device
void upload_coo_from_csr(rs_svd_plan* pl);
// the host CSR of a plan built on the device (downloaded COO, stable CSR build) -- for the host builders
void ensure_host_csr(rs_svd_plan* pl);
}  // namespace rs
