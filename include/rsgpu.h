/*
 * rsgpu.h -- C-ABI of the MI355X (gfx950) hot path for Oneaccount1/recommend-sys.
 *
 * This is the drop-in boundary: the entry points a cgo binding behind the reference's Go
 * `core.Estimator` types would call (INTEGRATION.md shows the binding).  Plain pointers and sizes
 * only; no torch or HIP types in the signatures (`stream` arguments are `hipStream_t` passed as
 * `void*`, NULL = the context's own stream).
 *
 * Reference interfaces replaced (all paths relative to the reference repository root):
 *   rs_svd_fit        <- core/svd.go:63-132    (*SVD).Fit            (per-epoch SGD, K1)
 *   rs_svdpp_fit      <- core/svd.go:316-427   (*SVDPP).Fit          (K2)
 *   rs_nmf_fit        <- core/svd.go:158-251   (*NMF).Fit            (K3)
 *   rs_knn_sims       <- core/knn.go:143-217   (*KNN).Fit pair loop  (K4 Cosine/MSD, K5 Pearson)
 *   rs_knn_sims_part  <- core/knn.go:195-215   the nJobs row split, one part per GPU
 *                        with core/sim.go:10-81 Cosine / MSD / Pearson as the pair function
 *   rs_sim_pair       <- core/sim.go:7-81      Sim func(a, b SortedIdRatings) float64
 *   rs_knn_plan_*     <- core/knn.go:143-217 + knn.go:75-141 (*KNN).Predict on the device (§8f row 2)
 *   rs_svd_predict    <- core/svd.go:32-51     (*SVD).Predict (batched, host)
 *   rs_svd_plan_predict / _evaluate <- svd.go:32-51, utils.go:162-180 on the device (§8f row 1)
 *   rs_baseline_fit   <- core/base.go:135-163  (*BaseLine).Fit (used by KNN-baseline knn.go:179)
 *   rs_knn_sims(kind RS_DEV_SLOPE_ONE) <- core/slope_one.go:47-93 (*SlopeOne).Fit dev matrix (§8f row 4)
 *   rs_slope_one_predict <- core/slope_one.go:21-45 (*SlopeOne).Predict on the device-resident dev
 *
 * Conventions
 *   - Ratings arrive as the TrainSet's COO triples (core/data.go:109-127) in TRAIN-SET ORDER with
 *     INNER ids (core/data.go:131-154: ids assigned by first appearance).  The library builds the
 *     user-CSR it needs itself and never retains a caller pointer after a call returns (cgo rule).
 *   - Model state is float64 on the host side (the reference's [][]float64 rows, flattened row-major
 *     with row stride = n_factors) and float32 on the device, converted at the boundary.
 *   - Every call returns an int status: RS_OK (0) or a negative RS_ERR_*; the message is available
 *     from rs_last_error(ctx) (thread-local when ctx is NULL).
 *   - Re-entrant: no global mutable state; each rs_ctx owns one HIP stream on one device and every
 *     entry point calls hipSetDevice(ctx->device) first (goroutines migrate OS threads).  A ctx must
 *     not be used by two threads at once; use one ctx per goroutine / CrossValidate fold.
 */
#ifndef RSGPU_H
#define RSGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_OK 0
#define RS_ERR_INVALID (-1)     /* bad argument (null pointer, id out of range, bad size)        */
#define RS_ERR_HIP (-2)         /* a HIP runtime call failed (message names it)                   */
#define RS_ERR_NOMEM (-3)       /* host or device allocation failed                               */
#define RS_ERR_UNSUPPORTED (-4) /* valid request this build does not implement                    */
#define RS_ERR_NO_DEVICE (-5)   /* no gfx950 device visible                                       */
#define RS_ERR_NUMERIC (-6)     /* the model left its number format (non-finite, or |q| past the fixed-point
                                   range: 128 on star ratings, wider for wider rating scales);
                                   the values are still returned                                   */

/* SGD visit schedule (SURVEY §8a parity contract P1/P2) */
#define RS_SGD_FAST 0    /* the FAST schedule of rs_sgd_params.write_back (default RS_SGD_WB_TILE: user
                            tiles in LDS, one memory-side atomic per (item, tile) run), work-local global bias */
#define RS_SGD_ORDERED 1 /* exact train-set order and update order of svd.go:93-129 (conflict-free batches, one workgroup) */

/* FAST-mode schedule / write-back of the item rows (rs_sgd_params.write_back, rs_svd_plan_set_mode) */
#define RS_SGD_WB_TILE 0          /* default: user tiles in LDS (integer LDS atomics), one memory-side
                                    integer atomic per (item, tile) run (sgd_tile.hip) */
#define RS_SGD_WB_STORE 1         /* per-user waves, write-through stores: Hogwild, concurrent updates of a
                                    row can be lost */
#define RS_SGD_WB_ATOMIC_DIRECT 2 /* per-user waves, each issuing its q_i deltas as memory-side atomics */
#define RS_SGD_WB_ATOMIC 3        /* per-user waves, memory-side atomic deltas with hot replicas, user
                                    splitting and heavy users' deltas through LDS rings to writer waves */

/* Similarity kinds: core/sim.go Cosine (10-25), MSD (28-44), Pearson (47-81) */
#define RS_SIM_COSINE 0
#define RS_SIM_MSD 1
#define RS_SIM_PEARSON 2
/* Not a similarity: the SlopeOne deviation matrix dev (core/slope_one.go:64-92), computed by the same
 * pairwise machinery (rs_knn_sims / _part / rs_knn_plan_create with left = items, right = users):
 * dev[i][j] = mean over co-rating users of (r_ui - r_uj), dev[j][i] = -dev[i][j], 0 on the diagonal
 * and where nothing is co-rated. */
#define RS_DEV_SLOPE_ONE 3

typedef struct rs_ctx rs_ctx;

/* COO ratings of a TrainSet in train-set order, inner ids (core/data.go:21-25, 109-127). */
typedef struct {
    int64_t nnz;
    int32_t n_users; /* TrainSet.UserCount */
    int32_t n_items; /* TrainSet.ItemCount */
    const int32_t* users;
    const int32_t* items;
    const double* ratings;
} rs_ratings;

/* Hyper-parameters read by SVD/SVD++ Fit (core/svd.go:65-71, 317-324). */
typedef struct {
    int32_t n_factors; /* "nFactors" */
    int32_t n_epochs;  /* "nEpochs"  */
    double lr;         /* "lr"       */
    double reg;        /* "reg"      */
    int32_t mode;      /* RS_SGD_FAST or RS_SGD_ORDERED */
    int32_t write_back; /* FAST only: RS_SGD_WB_* (RS_SGD_WB_TILE = 0 is the default) */
} rs_sgd_params;

/* ---- TrainSet construction on the host (no GPU involved) ------------------ *
 * rs_trainset_ids   <- core/data.go:137-151 NewTrainSet inner-id maps: inner[t] = first-appearance
 *                      index of outer[t] (call once for Users, once for Items); outer_of_inner
 *                      (n_unique entries, may be NULL) is the inverse map.  Parallel over n_threads
 *                      (<= 0: up to 16), result independent of it.
 * rs_csr_build      <- core/data.go:185-216 UserRatings / ItemRatings: stable CSR of COO rows (data
 *                      order inside a row); rowptr n_rows + 1, cols_out / vals_out nnz (vals_out may be
 *                      NULL), caller-allocated.
 * rs_global_mean    <- core/data.go:134 stat.Mean(Ratings): fixed-order chunked sum / n.           */
int rs_trainset_ids(int64_t n, const int64_t* outer, int32_t n_threads, int32_t* inner,
                    int64_t* outer_of_inner, int32_t* n_unique);
int rs_csr_build(int64_t nnz, int32_t n_rows, const int32_t* rows, const int32_t* cols,
                 const double* vals, int32_t n_threads, int64_t* rowptr, int32_t* cols_out,
                 float* vals_out);
int rs_global_mean(int64_t n, const double* ratings, int32_t n_threads, double* mean);

/* ---- synthetic benchmark sets (not a reference function; BASELINE configs[4] generator) ------- *
 * Inner-id user-CSR of n_users x n_items: lognormal user degrees (mean mean_deg, sigma, clamped to
 * [min_deg, max_deg]), Zipf(zipf_s) item popularity over a seeded id permutation, no repeated
 * (u, i), integer ratings 1..5 from a planted rank-4 model.  Only the ratings of items in
 * [item_lo, item_hi) are kept (an item-range shard of the same full set), and only the rows of users
 * [user_lo, user_hi) are generated (a user-range shard: row x is user user_lo + x; the CSR has
 * user_hi - user_lo rows).  Deterministic in seed, independent of n_threads.  rs_synth_csr exposes
 * the arrays (owned by the handle). */
typedef struct rs_synth rs_synth;
int rs_synth_create(int32_t n_users, int32_t n_items, double mean_deg, double sigma, int32_t min_deg,
                    int32_t max_deg, double zipf_s, uint64_t seed, int32_t item_lo, int32_t item_hi,
                    int32_t user_lo, int32_t user_hi, int32_t n_threads, rs_synth** out);
int rs_synth_csr(const rs_synth* s, int64_t* nnz, const int64_t** rowptr, const int32_t** cols,
                 const float** vals);
void rs_synth_destroy(rs_synth* s);

/* ---- context -------------------------------------------------------------------------------- */
int32_t rs_version(void);
int rs_device_count(int32_t* n);
int rs_open(int32_t device, rs_ctx** out);
void rs_close(rs_ctx* ctx);
/* The message of the last failed call on ctx (per ctx), or with ctx == NULL of the last failed ctx-less call
 * on the CALLING OS THREAD.  A host whose threads move between calls (Go: a goroutine may resume on another OS
 * thread between two cgo calls) reads ctx-less errors from an rs_report instead (rs_open_r, rs_svd_fit_multi). */
const char* rs_last_error(const rs_ctx* ctx);
/* Per-call report of the ctx-less entry points: written by the call itself before it returns, so it needs no
 * thread-local state.  error: the message of a failed call, NUL-terminated (truncated to fit), "" on success;
 * refits: rs_svd_fit_multi's divergence refits (0..3). */
typedef struct rs_report {
    int32_t refits;
    char error[508];
} rs_report;
/* rs_open with its error (if any) in *report (report may be NULL). */
int rs_open_r(int32_t device, rs_ctx** out, rs_report* report);
int rs_synchronize(rs_ctx* ctx);
/* Device time (ms, HIP events on the ctx stream) of the kernels of the last estimator call on ctx
 * (rs_svd_fit, rs_svdpp_fit, rs_nmf_fit, rs_baseline_fit, rs_knn_sims): uploads, host packing and
 * downloads excluded. */
int rs_last_kernel_ms(const rs_ctx* ctx, double* ms);

/* ---- estimators (host buffers in/out) ------------------------------------------------------- */

/* core/svd.go:63-132.  P (n_users x n_factors), Q (n_items x n_factors): injected initial factors
 * in (svd.go:80-85 draws them; the draw is unseeded in the reference, Q4), fitted factors out.
 * bu, bi, gb: in/out (the reference starts them at zero).
 * FAST mode keeps its plan (user-CSR, tile schedule, device buffers) and a host copy of the COO
 * (16 bytes per rating) on the ctx for the next rs_svd_fit of the same ratings (an exact comparison;
 * GridSearchCV / CrossValidate refit the same folds); sets of more than 2^26 ratings are not kept, any
 * other estimator call on the ctx (or rs_close) frees it, RSGPU_FIT_CACHE=0 turns it off. */
int rs_svd_fit(rs_ctx* ctx, const rs_ratings* r, const rs_sgd_params* p, double* P, double* Q,
               double* bu, double* bi, double* gb);
/* Divergence refits of the last rs_svd_fit on this ctx (FAST tile schedule): a fit whose model left the
 * fixed-point range or went non-finite is redone from the caller's inputs on a quarter of the workgroups and half the run cap (less
 * Hogwild staleness on the hot item rows), up to three times, before RS_ERR_NUMERIC is returned. */
int rs_fit_refits(const rs_ctx* ctx, int32_t* n);

/* core/svd.go:32-51 for n (inner user, inner item) pairs; -1 = unknown id (data.go:129). */
int rs_svd_predict(rs_ctx* ctx, int64_t n, const int32_t* users, const int32_t* items,
                   int32_t n_users, int32_t n_items, int32_t n_factors, const double* P,
                   const double* Q, const double* bu, const double* bi, double gb, double* out);

/* core/svd.go:316-427.  Y (n_items x n_factors) = ImplFactor.  RS_SGD_ORDERED runs the literal
 * per-rating y-update of svd.go:399-422; RS_SGD_FAST runs the user-CSR kernel with the lazy
 * per-user y-update. */
int rs_svdpp_fit(rs_ctx* ctx, const rs_ratings* r, const rs_sgd_params* p, double* P, double* Q,
                 double* Y, double* bu, double* bi, double* gb);

/* core/svd.go:158-251.  as_written=1 reproduces svd.go:243-249 (Q5), 0 the intended update. */
int rs_nmf_fit(rs_ctx* ctx, const rs_ratings* r, int32_t n_factors, int32_t n_epochs, double reg,
               int32_t as_written, double* P, double* Q);

/* core/base.go:135-163 BaseLine.Fit (bias-only SGD, ORDERED semantics). */
int rs_baseline_fit(rs_ctx* ctx, const rs_ratings* r, int32_t n_epochs, double lr, double reg,
                    double* bu, double* bi, double* gb);

/* core/knn.go:143-217 pair loop: sims (n_left x n_left, row-major float64) = sim(left_a, left_b)
 * over the co-rated right ids, NaN where nothing is co-rated and on the diagonal (knn.go:157,283).
 * Rows are CSR (rowptr[n_left+1], ids in [0, n_right), ratings) in any order within a row. */
int rs_knn_sims(rs_ctx* ctx, int32_t kind, int32_t n_left, int32_t n_right, const int64_t* rowptr,
                const int32_t* ids, const double* ratings, double* sims);

/* Multi-GPU form of rs_knn_sims (the knn.go:195-215 nJobs row split, one part per GPU).
 * The rows are cut into 128-row blocks; part p of n_parts owns the blocks t with t mod 2n in
 * {p, 2n-1-p} (near-equal triangle work) and writes ONLY the entries S[a][b] and S[b][a] with a in
 * its blocks and b >= a.  Parts write disjoint entries of the same n_left x n_left buffer, so
 * n_parts calls -- one per device, concurrently, into one shared host buffer -- assemble exactly
 * the rs_knn_sims result with no collective.  part 0 of 1 is rs_knn_sims. */
int rs_knn_sims_part(rs_ctx* ctx, int32_t kind, int32_t n_left, int32_t n_right,
                     const int64_t* rowptr, const int32_t* ids, const double* ratings, int32_t part,
                     int32_t n_parts, double* sims);
/* Host only: owned[t] = 1 for the 128-row blocks t of part (ceil(n_left / 128) entries). */
int rs_knn_part_blocks(int32_t n_left, int32_t part, int32_t n_parts, int32_t* owned);

/* core/sim.go one pair (ID-ascending inputs), computed on the device by the K5 merge kernel. */
int rs_sim_pair(rs_ctx* ctx, int32_t kind, int64_t na, const int32_t* a_ids, const double* a_r,
                int64_t nb, const int32_t* b_ids, const double* b_r, double* out);

/* ---- device-resident KNN: similarities stay in HBM, Predict runs on them ---- */
typedef struct rs_knn_plan rs_knn_plan;
/* core/knn.go:143-217 pair loop, as rs_knn_sims, keeping the n_left x n_left float64 Sims on the
 * device (K4 / K5). */
int rs_knn_plan_create(rs_ctx* ctx, int32_t kind, int32_t n_left, int32_t n_right,
                       const int64_t* rowptr, const int32_t* ids, const double* ratings,
                       rs_knn_plan** out);
void rs_knn_plan_destroy(rs_knn_plan* plan);
int rs_knn_plan_sims(rs_knn_plan* plan, double* sims /* host, n_left x n_left */);
/* core/knn.go:75-141 KNN.Predict for n (left, right) inner-id pairs (-1 / out of range = unknown):
 * candidates RightRatings[right] (right CSR over n_right rows, data order, ids are left ids) with a
 * non-NaN Sims[left][id], ordered as knn.go:107-108's sort.Sort orders them (RS_TIE_GO_SORT, default:
 * Go 1.24's pdqsort restated call for call, so equal similarities end in the reference's order), or by
 * (sim desc, position asc) (RS_TIE_STABLE, rs_knn_plan_set_tie_order); the first k summed in that order;
 * type 0 basic, 1 centered (means), 2 zscore (means, stddevs), 3 baseline (bias), arrays over left ids.
 * Bitwise equal to the restatement (oracle or_knn_predict / or_knn_predict_stable). */
#define RS_TIE_GO_SORT 0
#define RS_TIE_STABLE 1
int rs_knn_plan_set_tie_order(rs_knn_plan* plan, int32_t tie);
int rs_knn_plan_predict(rs_knn_plan* plan, int32_t type, int32_t n_right, const int64_t* right_rowptr,
                        const int32_t* right_ids, const double* right_r, const double* means,
                        const double* stddevs, const double* bias, double global_mean, int32_t k,
                        int32_t min_k, int64_t n, const int32_t* left, const int32_t* right,
                        double* out);

/* ---- device-resident SVD plan (bench / multi-GPU hosts; device pointers) -------------------- */
/* A plan uploads the user-CSR once and keeps the model resident in HBM: P (n_users x ld) and
 * Q (n_items x ld) float32 with ld = 64 * ceil((n_factors + 1) / 64); columns [0, n_factors) hold
 * the factors, column n_factors the bias (b_u in P, b_i in Q), the rest is zero; GlobalBias is one
 * float64.  Epochs are enqueued on `stream` without host syncs. */
typedef struct rs_svd_plan rs_svd_plan;

/* SlopeOne.Predict (core/slope_one.go:21-45) on a plan created with kind RS_DEV_SLOPE_ONE: user CSR of
 * the TrainSet in data order (UserRatings, data.go:185-199), inner ids (-1 = unknown -> global mean /
 * user mean as the reference); bitwise equal to the sequential definition. */
int rs_slope_one_predict(rs_knn_plan* plan, int32_t n_users, const int64_t* user_rowptr,
                         const int32_t* user_items, const double* user_ratings, double global_mean,
                         int64_t n, const int32_t* users, const int32_t* items, double* out);

int rs_svd_plan_create(rs_ctx* ctx, const rs_ratings* r, int32_t n_factors, rs_svd_plan** out);
/* The same plan from a user-CSR already in hand (rs_csr_build's output, or a generator's): rowptr has
 * n_users + 1 entries, cols / vals are in data order inside each row (data.go:185-199).  Skips the
 * COO -> CSR pass; the caller's arrays are copied and not retained. */
int rs_svd_plan_create_csr(rs_ctx* ctx, int32_t n_users, int32_t n_items, const int64_t* rowptr,
                           const int32_t* cols, const float* vals, int32_t n_factors, rs_svd_plan** out);
/* Device-side init, replacing svd.go:77-85 without a host round trip of the factors: biases 0,
 * factor entries N(mean, std_dev) from a counter-based hash of (seed, row, column), rows of P then Q
 * (the reference's draws come from the unseeded global math/rand, Q4: distribution kept, sequence
 * not); GlobalBias set to the FAST warm start (the mean rating, biases being 0). */
int rs_svd_plan_init_normal(rs_svd_plan* plan, double mean, double std_dev, uint64_t seed);
void rs_svd_plan_destroy(rs_svd_plan* plan);
/* host f64 -> device f32 (any of the pointers may be NULL = leave unchanged) */
int rs_svd_plan_upload(rs_svd_plan* plan, const double* P, const double* Q, const double* bu,
                       const double* bi, const double* gb);
int rs_svd_plan_download(rs_svd_plan* plan, double* P, double* Q, double* bu, double* bi,
                         double* gb);
/* Enqueue n_epochs fast-mode epochs (one SGD kernel + one epilogue -- global-bias fold, split users'
 * merge -- per epoch; Q converted to int32 fixed point before the first and back after the last). */
int rs_svd_plan_epochs(rs_svd_plan* plan, int32_t n_epochs, float lr, float reg, void* stream);
/* write_back: RS_SGD_WB_TILE (default), _STORE, _ATOMIC_DIRECT or _ATOMIC; ring_depth: item-row prefetch
 * distance in ratings of the per-user schedules (4, 8, 16 = default). */
int rs_svd_plan_set_mode(rs_svd_plan* plan, int32_t write_back, int32_t ring_depth);
/* RS_SGD_WB_TILE parameters: workgroups of the launch (0 = one per CU), waves per workgroup (1, 2, 4,
 * 8 or 16; default 16), ratings per tile (0 = nnz / workgroups, bounded by the 160 KiB LDS), run cap
 * (an item's run in a tile longer than this is cut into pieces on different waves; 0 = auto: hot items
 * cut so that ~100 of an item's updates are in flight; a huge value = never; ignored with
 * one wave), ring (q_i rows each wave loads ahead, in runs: 0 = auto = 2; with claimed runs (the default,
 * rs_svd_plan_set_tile_claim) 2, or for k <= 126 a ring of 3 or more becomes 4 on chunks of 8 runs (the
 * ring must divide the chunk); with host-dealt runs 2 or 4, and 3, 6, 8, 12 for
 * k <= 126; other values round down; deeper rings read hot rows earlier, i.e. staler).  Rebuilds the
 * schedule. */
int rs_svd_plan_set_tiles(rs_svd_plan* plan, int32_t workgroups, int32_t waves, int32_t target,
                          int32_t run_cap, int32_t ring);
/* Work distribution inside a tile: runs_per_claim = 4 (default) or 8 -- the tile's runs form one queue
 * and each wave claims that many consecutive runs at a time from an LDS counter (a workgroup ends about
 * one claim after its average wave); 0 -- the runs are dealt to the waves on the host (round-3
 * schedule).  Rebuilds the schedule. */
int rs_svd_plan_set_tile_claim(rs_svd_plan* plan, int32_t runs_per_claim);
/* How the users are cut into tiles (round 4):
 *   RS_TILE_RULE_LPT          (plans' default) host build: users dealt largest first to the least-loaded
 *                             tile, then moved between tiles by a per-run cost model;
 *   RS_TILE_RULE_FILL         host build: users by degree (descending, ties by id) over T = min(tiles,
 *                             active users) tiles; the first 4T dealt boustrophedon, the rest laid by prefix
 *                             sums on the line of the tiles' deficits against the mean load (midpoint rule);
 *                             no refinement;
 *   RS_TILE_RULE_FILL_DEVICE  the same rule built on the device (radix sorts and scans) -- rs_svd_fit's default
 *                             for sets of at most 2^24 ratings: the one-shot Fit's schedule costs no host time.
 * Both fill builds give byte-identical schedules (rs_svd_plan_schedule_digest); where the rule does not
 * apply (a user above the LDS bound, a tile past the LDS) the device build falls back to RS_TILE_RULE_LPT
 * and RS_TILE_RULE_FILL fails with RS_ERR_UNSUPPORTED.  Rebuilds the schedule. */
/* Divergence guard of the tile schedule (default on): every epoch measures its training MSE and flags one
 * that rises more than 1.03x over the previous epoch's (the history starts over on upload / init);
 * rs_svd_plan_epochs checks a call's epochs once at the end (that flag, fixed-point range of P and Q, a
 * finite GlobalBias; one small readback, so the call waits for its epochs) and redoes a failed call from its start state -- P, Q and GlobalBias copied on the device first --
 * on a quarter of the workgroups and half the run cap, up to three times.  The plan keeps the smaller grid after a hard
 * signal (the range flag, a non-finite GlobalBias); after redos that only the loss rule or the guard bound asked for
 * it returns to the caller's grid for the next call (until such redos have come three times).  The guard bound is a
 * quarter of the fixed-point range, which follows the ratings' spread (|v| < 32 on star scales, 512 for 1-100
 * ratings).  A call still failing leaves the flag for the download (RS_ERR_NUMERIC).  rs_svd_fit always runs
 * guarded.  Cost: a second resident copy of P and Q on the device (the call-start snapshot) and one host wait per
 * call.  off: no snapshot, no wait. */
int rs_svd_plan_set_guard(rs_svd_plan* plan, int32_t on);
/* Calls the guard has redone on this plan so far. */
int rs_svd_plan_refits(const rs_svd_plan* plan, int32_t* n);
/* The plan's fixed-point shift S (FAST P / Q / Y held as int32 round(v 2^S) while a call runs; from the ratings'
 * spread, lowered to the group's smallest while the plan is in a group or joined -- rs_svd_plan_leave /
 * rs_svd_group_destroy restore it). */
int rs_svd_plan_fixed_point(const rs_svd_plan* plan, int32_t* shift);
#define RS_TILE_RULE_LPT 0
#define RS_TILE_RULE_FILL 1
#define RS_TILE_RULE_FILL_DEVICE 2
int rs_svd_plan_set_tile_rule(rs_svd_plan* plan, int32_t rule);
/* The rule the plan's current schedule was built with (a device build that fell back reports LPT). */
int rs_svd_plan_tile_rule(const rs_svd_plan* plan, int32_t* rule);
/* 64-bit FNV-1a digest of the plan's tile schedule as the kernel reads it from HBM (tile count, LDS bytes,
 * tiles, tile users, streams, run headers, records). */
int rs_svd_plan_schedule_digest(rs_svd_plan* plan, uint64_t* digest);
/* The same digest, and the tile rule, of the plan the last FAST rs_svd_fit on ctx built and cached (a
 * one-shot Fit builds with RS_TILE_RULE_FILL_DEVICE from the caller's COO; tests compare it with a
 * plan's host RS_TILE_RULE_FILL build).  RS_ERR_INVALID when no such plan is cached. */
int rs_fit_schedule_digest(rs_ctx* ctx, uint64_t* digest, int32_t* rule);
/* Visit order of the tile schedule: pos[n] = user-CSR position (rowptr order, data order inside a row)
 * of the n-th rating (nnz entries) as the kernel's streams walk it -- tile by tile, a tile's waves in
 * order, a wave's runs in order --, and work_off (n_works + 1 entries) the boundaries of the (tile,
 * wave) streams, the kernel's GlobalBias work items; n_works = tiles x waves.  With claimed runs the
 * whole queue is stream 0 of its tile (the other streams empty): with one wave it is the visit order,
 * with several the waves' shares are decided at run time.  Any pointer may be
 * NULL (call once with pos = work_off = NULL for n_works).  With one workgroup of one wave an epoch
 * is exactly the sequential SGD of svd.go:93-129 in this order with the work-local GlobalBias fold
 * (the oracle's or_svd_fit_works restates it). */
int rs_svd_plan_tile_order(rs_svd_plan* plan, int64_t* pos, int64_t* work_off, int32_t* n_works);
/* Diagnostic (experiments): per-wave phase clocks of the last timed tile epoch (RSGPU_TILE_DIAG=16):
 * {staging, q-ring waits, rating loops, write-back} shader cycles per wave, up to n int64 values. */
int rs_svd_plan_tile_clocks(rs_svd_plan* plan, int64_t* out, int64_t n);
/* Diagnostic, host only (no device needed): builds the tile schedule of a user-CSR the way a plan
 * would (workgroups, waves, user blocks; n_blocks < 0: -n_blocks item blocks, a ROTATE_Q shard's strata)
 * and reports
 * its host time in ms, the tile count and, for non-NULL outputs, the visit order pos (nnz user-CSR
 * positions, as rs_svd_plan_tile_order) and the tiles' first records tile_off (n_tiles + 1); rank (nnz)
 * is zero-filled.  svdpp must be 0: the SVD++ tile schedule it selected was removed in round 3
 * (RS_ERR_UNSUPPORTED). */
int rs_tile_schedule_host(int32_t n_users, int32_t n_items, const int64_t* rowptr, const int32_t* cols,
                          const float* vals, int32_t n_factors, int32_t workgroups, int32_t waves,
                          int32_t n_blocks, int32_t svdpp, int64_t* pos, int64_t* tile_off, int32_t* rank,
                          int32_t* n_tiles, double* ms);
/* RS_SGD_WB_ATOMIC schedule.  Work items with at least heavy_min ratings (default 1000; 0 = none) run
 * as one SGD wave plus three writer waves that issue its atomics; the other (light) items are
 * strided over light_blocks blocks of four waves (default < 0: 1.5 per CU; 0: one wave per item).
 * Same arithmetic and results class as RS_SGD_WB_ATOMIC_DIRECT; only the visit timing changes
 * (DESIGN.md K1). */
int rs_svd_plan_set_schedule(rs_svd_plan* plan, int32_t heavy_min, int32_t light_blocks);
/* Diagnostic: out == NULL enables a per-work-item timeline for RS_SGD_WB_ATOMIC epochs; otherwise
 * copies the last epoch's {start, chain end, write-back end} (100 MHz ticks, 3 int64 per work item, LPT
 * order) to out and the work items' users to user (may be NULL). */
int rs_svd_plan_trace(rs_svd_plan* plan, int64_t* out, int32_t* user);
/* FAST-mode work items: users with more than split_cap ratings (default 1200; 0 = never split) run as
 * ceil(deg / split_cap) near-equal pieces on separate waves from the same p_u, and the row becomes the
 * count-weighted average of the pieces' end states after the epoch (or_svd_fit_chunked restates it).
 * Cuts the heaviest users' serial chains, which set the epoch's tail.  Measured trade-off (DESIGN.md
 * K1): at 1200 the ML-1M-shaped held-out RMSE moves by +0.0008 (to within 0.0001 of the reference
 * visit order's); at 256 by +0.024. */
int rs_svd_plan_set_split(rs_svd_plan* plan, int32_t split_cap);
/* RS_SGD_WB_ATOMIC (hybrid) hot items: an item with more than item_cap ratings gets
 * ceil(deg / item_cap) row copies; its ratings are dealt over them in user-CSR order and the copies
 * are merged by count-weighted average after every epoch.  Spreads the atomics of hot rows.
 * item_cap = 0 (default) is automatic: only items too hot for hot replicas (more than 65536 x copies
 * ratings, whose live copies diverge) are cut, into 65536-rating pieces.
 * The tile schedule (RS_SGD_WB_TILE) bounds hot-item staleness by its own run cap instead. */
int rs_svd_plan_set_item_split(rs_svd_plan* plan, int32_t item_cap);
/* Hot replicas: the n_hot most-rated items (0 = none) get `copies` row copies (2..8) over which their
 * ratings are dealt, and in RS_SGD_WB_ATOMIC (hybrid) epochs one extra block keeps the copies merged
 * while the epoch runs (delta sum: every update reaches every copy, at most one merge round late; a
 * final round after the epoch leaves them equal).  Spreads a hot item's memory-side float atomics
 * over several rows.  Hot replicas win over item_cap splitting for the items they take.
 * Default 256 x 8 (set n_hot = 0 to turn them off). */
int rs_svd_plan_set_hot_replicas(rs_svd_plan* plan, int32_t n_hot, int32_t copies);
/* Fixed-point item rows (default on; 0 turns it off): RS_SGD_WB_ATOMIC (hybrid) epochs convert Q in place to int32
 * round(q * 2^24) before the epoch kernel and back after it, and the q_i deltas become integer
 * atomics (memory-side u32 adds run at 1.69 TB/s against 1.32 TB/s for f32 on gfx950).  The
 * resolution is the fp32 ulp at |q| in [0.5, 1); |q| must stay below 128: the conversion to int32
 * saturates, but integer atomics wrap, so the conversion back flags a row that reached the range
 * limit or a non-finite value and the next call returns RS_ERR_NUMERIC.  The tile schedule
 * (RS_SGD_WB_TILE) always keeps Q in this format during a call, with the same check. */
int rs_svd_plan_set_fixed_q(rs_svd_plan* plan, int32_t on);
/* ---- item-sharded multi-GPU (north_star: Q sharded by item range, users replicated) --------- *
 * Each rank builds a plan over its item shard.  Per epoch: rs_svd_plan_epoch_delta leaves P at the
 * epoch start and writes dP[u] = w_u (p_u(end) - p_u(start)) (bias column included; for a split
 * user the count-weighted average over its pieces) and
 * gbsum = sum_w n_w (gb_w - gb); the caller all-reduces (sum) dP and gbsum over the ranks (RCCL)
 * and calls rs_svd_plan_apply_delta(inv_total_nnz = 1 / total ratings over all ranks).
 * w_u = (ratings of u in this shard) / (ratings of u over all shards): the count-weighted average of
 * the shards' user deltas (a plain sum of per-shard deltas overshoots for users split over shards).
 * dP: device buffer of n_users x ld float32; gbsum: device float64. */
int rs_svd_plan_set_user_weights(rs_svd_plan* plan, const float* w /* host, n_users; NULL clears */);
int rs_svd_plan_epoch_delta(rs_svd_plan* plan, float lr, float reg, void* dP, void* gbsum,
                            void* stream);
int rs_svd_plan_apply_delta(rs_svd_plan* plan, const void* dP, const void* gbsum,
                            double inv_total_nnz, void* stream);
/* ---- item-sharded multi-GPU behind the library (RCCL over xGMI; multi.hip) ------------------- *
 * Q and b_i are sharded by item range (one plan per rank over its shard; same users, same n_factors).
 * Two exchanges, chosen per plan before the join (rs_svd_plan_set_exchange):
 *
 * RS_EXCHANGE_ROTATE (default) -- the stratum rotation, exact.  The users are cut into n_ranks
 * rank-blocks of near-equal ratings (from every user's ratings over all shards, so the blocks agree on
 * every rank), each of `pieces` user blocks with their own tiles.  An epoch is n_ranks sub-epochs: in
 * sub-epoch s rank g trains its shard against rank-block (g + s) mod n_ranks with P updated in place,
 * then sends those rows to rank g - 1 and receives rank-block (g + s + 1) from rank g + 1 (RCCL
 * send/recv on a library comm stream, piece by piece while the next piece computes).  Every rating is
 * trained once per epoch against the current p_u and q_i; no rows are averaged.  GlobalBias is folded
 * once per epoch from every stratum's work-local partials (all-reduced).  After the call the
 * rank-blocks are broadcast, so P, b_u and GlobalBias are identical on every rank again.  n_blocks =
 * user blocks in all (rounded up to a multiple of n_ranks; 0 = automatic: 2..16 pieces of ~64 MiB of
 * P per rank-block).
 * This replaces north_star's per-epoch all-reduce of user-factor deltas, which RS_EXCHANGE_AVERAGE
 * keeps (the averaged deltas miss the reference's RMSE).
 *
 * RS_EXCHANGE_AVERAGE -- round 2's protocol: the epoch of every rank in delta mode from the same P, the
 * count-weighted user deltas all-reduced per user block while the next block computes and applied
 * (n_blocks 0 = automatic: about 256 MiB of deltas per block, 2..32).
 *
 * One process per GPU (the Go host's one-process-per-GPU mode, bench.py --gpus N): rank 0 calls
 * rs_comm_unique_id and sends the RS_COMM_ID_BYTES bytes to every rank (any channel); every rank
 * builds a plan over its item shard, uploads the same P / b_u / GlobalBias and calls rs_svd_plan_join
 * (collective: all ranks together), then rs_svd_plan_epochs_sharded on every rank with the same
 * arguments.  rs_svd_plan_leave frees the communicator (rs_svd_plan_destroy does too).
 * rs_comm_info reports the RCCL library the process runs against (its version code and the path of
 * the one librccl mapped; path_len bytes incl. the terminating NUL; either pointer may be NULL). */
#define RS_EXCHANGE_ROTATE 0
#define RS_EXCHANGE_AVERAGE 1
/* RS_EXCHANGE_ROTATE_Q -- the dual rotation (round 4), exact like ROTATE, for U > I (configs[4]: 10M users,
 * 1M items): the factor matrix that travels is the smaller one.  Rank g's plan holds the ratings of its
 * user range (global user and item ids, all items: each rank's users a contiguous range, ascending by
 * rank).  The items are cut into n_ranks item rank-blocks of near-equal ratings (from every item's ratings
 * over all ranks), each of `pieces` item blocks, and the plan's tiles are built per stratum (its users x
 * one item block).  In sub-epoch s rank g trains its users against item rank-block (g + s) mod n_ranks,
 * then sends those Q rows (b_i in column k) to rank g - 1 and receives item rank-block (g + s + 1) from
 * rank g + 1, piece by piece; P rows never move during the call.  At configs[4] a sub-epoch moves
 * 1M / 8 Q rows (160 MB at k = 256) instead of 10M / 8 P rows (1.6 GB).  After the call the item
 * rank-blocks and every rank's user range are broadcast, so P, Q, the biases and GlobalBias are identical
 * on every rank.  n_blocks = item blocks in all (rounded up to a multiple of n_ranks; 0 = automatic: 2..16
 * pieces of ~64 MiB of Q per rank-block). */
#define RS_EXCHANGE_ROTATE_Q 2
/* RS_EXCHANGE_QDELTA -- north_star's once-per-epoch all-reduce, on the smaller factor matrix (round 5; for
 * U > I, configs[4]).  As ROTATE_Q the ranks hold user ranges (contiguous, ascending by rank) and every item;
 * the rank's users are cut into n_blocks merges per epoch (user blocks of near-equal ratings; 0 = 16, the fewest
 * that keep configs[4]'s held-out RMSE within 0.01 of the whole-set fit after 10 epochs) and each
 * block is one plain tile launch of those users against the whole Q (P in place), after which the rank's item
 * moves are all-reduced (n_items rows of the plan's row stride):
 * q_i <- q_i,start + sum over ranks of w_i (q_i,end - q_i,start), with w_i = kappa_i / c_i over the c_i ranks
 * that rate item i, kappa_i = (1 - a^(c_i n_i)) / (1 - a^n_i), n_i = its ratings per rank and merge, a = 1 - lr
 * (the moves of a unit-curvature coordinate that c_i ranks each close by 1 - a^n_i, scaled to the sequential
 * 1 - a^(c_i n_i)): exact for items of one rank, the mean of converged moves.  Hot items -- rated on several
 * ranks, at least 4 ratings per rank and block -- are merged after every block; the others (cold) only after
 * every cold_every-th block (the largest divisor of the merges per epoch up to 2; rs_svd_plan_set_qdelta_split),
 * where every item is merged (a full merge), their n_i counted over those blocks.  Pipelined: a rank applies its own weighted moves at
 * once and the other ranks' (sum - own) at the row's next merge, so merge m's all-reduce runs behind block
 * m + 1's kernel; the call's last merge is a full one, after which every rank holds the same Q.  The moves travel
 * as fp16 factor units (rs_svd_plan_set_qdelta_wire 16, the default: half the bytes) or int32 fixed point (32:
 * exact integer sums); either way every rank applies the same rounded values.  GlobalBias: the ranks'
 * partials, one f64 all-reduce per merge (applied with the same one-merge delay).  After the call the ranks'
 * P ranges are broadcast. */
#define RS_EXCHANGE_QDELTA 3
int rs_svd_plan_set_exchange(rs_svd_plan* plan, int32_t mode);
/* RS_EXCHANGE_QDELTA's wire width: 16 (fp16 moves, default) or 32 (int32 fixed point).  Set before the join;
 * every rank of a group must use the same width (the join checks). */
int rs_svd_plan_set_qdelta_wire(rs_svd_plan* plan, int32_t bits);
/* RS_EXCHANGE_QDELTA's hot / cold split: items rated on several ranks with at least hot_ratings ratings per rank
 * and block are hot (merged after every block; hot_ratings <= 0: every such item); the others are merged after
 * every cold_every-th block (the largest divisor of the merges per epoch up to cold_every; 1: every merge is a
 * full one).  Set before the join, the same on every rank. */
int rs_svd_plan_set_qdelta_split(rs_svd_plan* plan, double hot_ratings, int32_t cold_every);
/* RS_EXCHANGE_QDELTA's merge weights on the factor columns: the contraction per rating a = 1 - lr x gamma in
 * kappa_i (default 0.25, round 6: configs[4]'s 8-shard fit within 0.005 of the whole-set fit at 10 and 20 epochs,
 * where gamma = 1, the unit curvature above, left 0.0093 at 10; 0: w_i = 1, the plain sum of the moves).  The bias
 * column keeps the unit curvature of its own gradient.  Set before the join, the same on every rank. */
int rs_svd_plan_set_qdelta_curvature(rs_svd_plan* plan, double gamma);
/* Test hook: the tile schedule's hot-run damping with the runs in flight of an item taken
 * as R = its ratings x kconc (kconc > 0 forces the damped kernel; 0 restores the library's rule, R = ratings x
 * workgroups x waves / nnz, damped where the hottest item reaches 40).  With one wave the runs never overlap, so
 * the damped kernel is checked against the oracle's restatement (or_svd_fit_works_damped). */
int rs_svd_plan_set_damp_concurrency(rs_svd_plan* plan, float kconc);
/* Cold runs of the tile schedule (round 6): an item with so few ratings that on average fewer than
 * `runs_in_flight` of its runs are in flight at once (ratings x workgroups x waves / nnz) ends each run with plain
 * write-through stores of its new row instead of memory-side atomic adds -- a concurrent run of the same item
 * then loses its update, which happens with about that probability.  0 turns it off; default 0.05.  Runs are
 * marked, and the kernel variant with the stores launched, only where the mean item is cold (the threshold degree
 * reaches nnz / n_items: configs[4], not ML-1M -- the variant's extra exit costs a set of few cold runs more than the
 * stores save).  With one wave per workgroup a store equals the atomic (no run overlaps).  Rebuilds the schedule. */
int rs_svd_plan_set_cold_store(rs_svd_plan* plan, double runs_in_flight);
/* How a single-GPU tile epoch folds GlobalBias (svd.go:104-106's chain, run per (tile, wave) stream from the epoch's
 * start value): RS_GB_FOLD_SMOOTH (default since round 6) -- the streams' chains composed with their rates at
 * their mean, gb' = A gb + (1 - A) T (sgd_tile.hip header); RS_GB_FOLD_MEAN -- the count-weighted mean of the
 * streams' moves (rounds 1-5; the multi-GPU exchanges always fold this way). */
#define RS_GB_FOLD_MEAN 0
#define RS_GB_FOLD_SMOOTH 1
int rs_svd_plan_set_gb_fold(rs_svd_plan* plan, int32_t mode);
/* RS_EXCHANGE_ROTATE_Q on Zipf-headed sets: a stratum (one rank's users x one item block) holds an item's
 * ratings n_blocks-fold concentrated, so the head's rows get many concurrent runs in flight (Hogwild staleness
 * that diverges at lr 0.005; configs[4]: the hottest item is 0.8 % of the set but 12.7 % of its stratum).  An
 * item whose share of its stratum would pass `share` (default 0.02) -- when strata hold at least min_stratum
 * ratings (default 2^17) -- is split: one row copy per item block, its ratings dealt to the copies by user
 * hash (each copy trained in its block's strata, travelling with the block; as few copies as bring the
 * item's share under `share`), the copies merged once per epoch into the item's row on every rank as the
 * last merged value plus w x the sum of the copies' moves since: RS_HOT_SCALED (default) w = kappa / c with
 * kappa = (1 - (1 - lr)^(c n)) / (1 - (1 - lr)^n), c copies of n ratings each per epoch (the ratio of what
 * sequential SGD over all c n ratings and what one copy closes of a unit-curvature gap: c for lightly trained
 * copies, 1 for converged ones); RS_HOT_AVERAGE w = 1 / c (the copies' mean); RS_HOT_SUM w = 1 (diverges on
 * the Zipf head: measured).  share = 0 turns it off.  Set before the join. */
#define RS_HOT_SCALED 0
#define RS_HOT_AVERAGE 1
#define RS_HOT_SUM 2
int rs_svd_plan_set_hot_split(rs_svd_plan* plan, double share, int64_t min_stratum, int32_t merge);
/* Diagnostic: one epoch of the plan with each user block / stratum of its tile schedule (a joined plan's,
 * or rs_svd_plan_set_user_blocks') launched alone and timed -- ms[b] = block b's SGD kernel in
 * milliseconds (n >= the plan's blocks).  It trains the model like an epoch.  Used to table the
 * per-stratum times the sub-epochs of a sharded run wait on (DESIGN.md Multi-GPU). */
int rs_svd_plan_time_blocks(rs_svd_plan* plan, float lr, float reg, double* ms, int32_t n);
/* Test hook (fault injection): the next rs_svd_plan_epochs_sharded / rs_svd_group_epochs call on this
 * plan throws at the start of its sub-epoch `sub_epoch` (once), so tests can check that the other ranks
 * are released.  RS_FAULT_DIVERGE instead changes one word of this rank's replicated factors just before
 * the call's consistency check (below).  -1 clears it.  Nothing else reads it.
 *
 * Consistency check: after every sharded call (every exchange, n_ranks > 1) the ranks compare checksums of
 * their replicated state -- P with b_u and GlobalBias, and Q with b_i under ROTATE_Q / QDELTA -- by RCCL max
 * and min all-reduces (or the in-process group's barrier); a mismatch is RS_ERR_NUMERIC on every rank
 * (rs_svd_fit_multi redoes the fit, as for a divergence). */
#define RS_FAULT_DIVERGE (-2)
int rs_svd_plan_inject_fault(rs_svd_plan* plan, int32_t sub_epoch);
/* Host only: RS_EXCHANGE_ROTATE's sub-epoch `sub_epoch` of `rank` -- out[0] the rank-block it trains,
 * out[1] the rank its rows are sent to, out[2] the rank-block it receives, out[3] the rank that sends
 * it.  The schedule rs_svd_plan_epochs_sharded runs. */
int rs_rotation_step(int32_t rank, int32_t n_ranks, int32_t sub_epoch, int32_t* out /* 4 */);
int rs_comm_info(int32_t* version, char* path, int32_t path_len);
/* A joined plan's rank and rank count (from the RCCL communicator when there is one), its exchange and
 * its user blocks in all (any pointer may be NULL). */
int rs_svd_plan_shard_info(rs_svd_plan* plan, int32_t* rank, int32_t* n_ranks, int32_t* exchange,
                           int32_t* n_blocks);
/* RS_EXCHANGE_QDELTA's item split of a joined plan: the hot items (merged after every block) and the blocks
 * between full merges (either pointer may be NULL). */
int rs_svd_plan_qdelta_info(rs_svd_plan* plan, int32_t* n_hot, int32_t* cold_every);
#define RS_COMM_ID_BYTES 128
int rs_comm_unique_id(void* id /* RS_COMM_ID_BYTES */);
int rs_svd_plan_join(rs_svd_plan* plan, const void* id, int32_t rank, int32_t n_ranks, int32_t n_blocks);
/* On an error inside the call the plan aborts its communicator (ncclCommAbort) and stays unusable until
 * rs_svd_plan_leave; its peers may be blocked in a transfer with it, which RCCL does not cancel across
 * processes -- a one-process-per-GPU host needs its own watchdog (e.g. the launcher's timeout). */
int rs_svd_plan_epochs_sharded(rs_svd_plan* plan, int32_t n_epochs, float lr, float reg, void* stream);
int rs_svd_plan_leave(rs_svd_plan* plan);
/* User blocks of the tile schedule (default 1): the visit order becomes block by block.  bounds
 * (n_blocks + 1 user ids from 0 to n_users, or NULL: from this plan's ratings, the b-th bound being the
 * first user whose ratings start at or past b / n_blocks of them).  A joined plan uses the same rule on
 * every user's ratings over all shards, so the blocks agree across shards; passing those bounds here
 * lets a single plan reproduce a joined plan's visit order. */
int rs_svd_plan_set_user_blocks(rs_svd_plan* plan, int32_t n_blocks, const int32_t* bounds);
/* One process driving n shards (one host thread per shard): RCCL when every plan has its own device,
 * otherwise (shards sharing a device: tests) an in-process exchange behind host barriers (ROTATE: the
 * rank-blocks copied between the shards' P; AVERAGE: the deltas summed in shard order; same arithmetic,
 * no overlap).  If a shard fails, the others are released (barrier failure, ncclCommAbort) and the
 * call returns its error.  The plans stay owned by the caller; rs_svd_group_destroy detaches them. */
typedef struct rs_svd_group rs_svd_group;
int rs_svd_group_create(rs_svd_plan* const* plans, int32_t n, int32_t n_blocks, rs_svd_group** out);
int rs_svd_group_epochs(rs_svd_group* group, int32_t n_epochs, float lr, float reg);
void rs_svd_group_destroy(rs_svd_group* group);
/* Item shards of near-equal ratings over contiguous inner item ids: bounds (n_shards + 1 entries). */
int rs_item_shards(int64_t nnz, const int32_t* items, int32_t n_items, int32_t n_shards, int32_t* bounds);
/* core/svd.go:63-132 (FAST tile schedule) on n_devices GPUs of this process: the items are sharded by
 * rs_item_shards and P rank-blocks rotate (RS_EXCHANGE_ROTATE); with fewer items than users and P rank-blocks
 * of 16 MiB or more the users are cut into ranges of near-equal ratings and the ranks' item moves are
 * all-reduced (RS_EXCHANGE_QDELTA, fp16 wire; n_blocks = merges per epoch, 0 = 16).  As rs_svd_fit otherwise (GlobalBias warm start, host buffers in / out; a fit
 * whose shards leave the fixed-point range, go non-finite or hold a factor past the guard bound is rebuilt and
 * redone from the inputs on half the workgroups and run cap 2, up to three times -- report->refits counts
 * them; RS_ERR_NUMERIC after every shard's values are written). */
int rs_svd_fit_multi(const int32_t* devices, int32_t n_devices, const rs_ratings* r, const rs_sgd_params* p,
                     int32_t n_blocks, double* P, double* Q, double* bu, double* bi, double* gb,
                     rs_report* report /* may be NULL: the refits and the error message of this call */);
/* ---- user-sharded multi-GPU (the dual partition, SURVEY §8e "measured alternative") ---------- *
 * Each rank builds a plan over its user range (local user ids) with ALL items; Q and b_i are
 * replicated, P and b_u are exclusive to the rank.  Per epoch: rs_svd_plan_epoch_qdelta runs the
 * FAST epoch (P in place), writes dQ[i] = w_i (q_i(end) - q_i(start)) (bias column included) and
 * gbsum as rs_svd_plan_epoch_delta, and leaves Q at the epoch start; the caller all-reduces dQ
 * (n_items x ld fp32 -- for U >> I far less than the item-sharded n_users x ld) and gbsum, then
 * rs_svd_plan_apply_qdelta.  w_i = (ratings of i on this rank) / (ratings of i on all ranks). */
int rs_svd_plan_set_item_weights(rs_svd_plan* plan, const float* w /* host, n_items; NULL clears */);
int rs_svd_plan_epoch_qdelta(rs_svd_plan* plan, float lr, float reg, void* dQ, void* gbsum,
                             void* stream);
int rs_svd_plan_apply_qdelta(rs_svd_plan* plan, const void* dQ, const void* gbsum,
                             double inv_total_nnz, void* stream);
/* Device pointers of the resident state (layout above); ld = row stride in floats. */
int rs_svd_plan_device_ptrs(rs_svd_plan* plan, void** P, void** Q, void** gb_f64, int32_t* ld);
/* Per-launch timing: when on, rs_svd_plan_epochs brackets every SGD kernel with HIP events on
 * the stream it runs on (adds one event pair per epoch; leave off for throughput runs). */
int rs_svd_plan_set_timing(rs_svd_plan* plan, int32_t on);
/* Device time of the last rs_svd_plan_epochs call in milliseconds (HIP events on the launch
 * stream).  Timing on: sum over the SGD kernels only, n_launches = epochs.  Timing off: the whole
 * enqueued span (SGD + global-bias fold kernels), n_launches = 2 * epochs. */
int rs_svd_plan_last_kernel_ms(rs_svd_plan* plan, double* ms, int32_t* n_launches);
/* Batched Predict on the plan's device factors (core/svd.go:32-51 per pair, inner ids, -1 = unknown,
 * data.go:129), evaluated in float64 on the fp32 factors; and RMSE / MAE over a test set
 * (core/utils.go:162-180; summed in a fixed order on the device).  SURVEY §8f row 1. */
int rs_svd_plan_predict(rs_svd_plan* plan, int64_t n, const int32_t* users, const int32_t* items,
                        double* out);
int rs_svd_plan_evaluate(rs_svd_plan* plan, int64_t n, const int32_t* users, const int32_t* items,
                         const double* ratings, double* rmse, double* mae);

#ifdef __cplusplus
}
#endif
#endif /* RSGPU_H */
