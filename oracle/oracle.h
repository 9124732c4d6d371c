/*
 * oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Reference: Oneaccount1/recommend-sys @ 2025-08-24, pure Go, package core/.
 * The reference cannot be compiled here (no Go toolchain, gonum v0.9.1 absent, and the package has
 * compile errors at this snapshot: core/eval.go:40,107).  This file restates, in plain C and fp64,
 * the exact arithmetic order of the functions on the hot path.  Every function cites the reference
 * file:line it follows.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - Cosine/MSD/Pearson are pinned by the reference's own known-answer tests core/sim_test.go:10-59
 *     (tests/golden/sim_kat.json, exact values 14/sqrt(205), 1/10, 0).
 *   - SVD / NMF / KNN fits are pinned by the reference's accuracy regressions core/base_test.go:35,43,51
 *     (5-fold CV on ML-100K, RMSE/MAE <= expected + 0.008), evaluated on the restatement.
 *   - SVD++ has no active reference test (core/base_test.go:38-40 is commented out): parity unpinned.
 *   - gonum floats.Dot (third-party, gonum.org/v1/gonum v0.9.1, go.mod:7, not vendored) is restated as
 *     a sequential left-to-right sum; its amd64 asm summation order is unverified (few-ulp effect).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* data.go:131-154 NewTrainSet: inner ids by first appearance over Users, then over Items. */
int or_trainset_ids(int64_t n, const int64_t* users, const int64_t* items,
                    int32_t* inner_u, int32_t* inner_i, int32_t* n_users, int32_t* n_items);

/* svd.go:63-132 SVD.Fit epoch loop, ratings visited in the given (train-set) order.
 * P (U*k), Q (I*k) carry the injected initial factors in and the fitted factors out
 * (svd.go:80-85 draws them; Q4: the draw is unseeded in the reference so parity injects it).
 * bu, bi, gb are in/out (reference starts them at 0: svd.go:77-78, GlobalBias zero value). */
void or_svd_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                int32_t k, int32_t epochs, double lr, double reg,
                double* P, double* Q, double* bu, double* bi, double* gb);

/* The FAST schedules' GlobalBias semantics over explicit work items (segments of the given order),
 * works run one after another: the GPU tile / per-user kernels' own schedule on race-free input. */
void or_svd_fit_works(int64_t n, const int32_t* u, const int32_t* i, const double* r, int64_t n_works,
                      const int64_t* work_off, int32_t k, int32_t epochs, double lr, double reg, double* P,
                      double* Q, double* bu, double* bi, double* gb);
/* The same with the fold chosen: compose = 0 the count-weighted mean of the works' GlobalBias moves (the
 * multi-GPU exchanges; or_svd_fit_works), 1 the works' affine chains composed in work order (the
 * single-GPU tile schedule since round 6). */
void or_svd_fit_works2(int64_t n, const int32_t* u, const int32_t* i, const double* r, int64_t n_works,
                       const int64_t* work_off, int32_t k, int32_t epochs, double lr, double reg, double* P,
                       double* Q, double* bu, double* bi, double* gb, int32_t compose);
/* or_svd_fit_works2 (compose 0 or 2) with the tile schedule's hot-run damping (oracle.c). */
void or_svd_fit_works_damped(int64_t n, const int32_t* u, const int32_t* i, const double* r, int64_t n_works,
                             const int64_t* work_off, const int32_t* deg, double kconc, int32_t k, int32_t epochs,
                             double lr, double reg, double* P, double* Q, double* bu, double* bi, double* gb,
                             int32_t compose);
/* svd.go:32-51 SVD.Predict for inner ids (-1 = unknown, data.go:129 newID). */
void or_svd_predict(int64_t n, const int32_t* u, const int32_t* i, int32_t k,
                    const double* P, const double* Q, const double* bu, const double* bi,
                    double gb, double* out);

/* svd.go:316-427 SVDPP.Fit, literal O(sum |N(u)|^2 k) form.  N(u) = TrainSet.UserRatings()
 * (data.go:185-199: data order).  n_users needed to build N(u). */
void or_svdpp_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                  int32_t n_users, int32_t k, int32_t epochs, double lr, double reg,
                  double* P, double* Q, double* Y, double* bu, double* bi, double* gb);

/* svd.go:271-310 SVDPP.Predict for inner ids. */
void or_svdpp_predict(int64_t n_train, const int32_t* tu, const int32_t* ti, int32_t n_users,
                      int64_t n, const int32_t* u, const int32_t* i, int32_t k,
                      const double* P, const double* Q, const double* Y, const double* bu,
                      const double* bi, double gb, double* out);

/* svd.go:158-251 NMF.Fit.  as_written=1 reproduces svd.go:243-249 literally (Q5: q_i *= itemUp[i]
 * undivided); as_written=0 applies the intended q_i *= itemUp[i]/itemDown[i] (svd.go:242 comment). */
void or_nmf_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                int32_t n_users, int32_t n_items, int32_t k, int32_t epochs, double reg,
                int32_t as_written, double* P, double* Q);

/* svd.go:140-147 NMF.Predict. */
void or_nmf_predict(int64_t n, const int32_t* u, const int32_t* i, int32_t k,
                    const double* P, const double* Q, double* out);

/* sim.go:10-81 Cosine (kind 0), MSD (kind 1), Pearson (kind 2) over ID-ascending lists. */
double or_sim(int32_t kind, int64_t na, const int32_t* a_id, const double* a_r,
              int64_t nb, const int32_t* b_id, const double* b_r);

/* knn.go:189-216 (KNN.Fit pair loop) with nJobs = 1: Sims L x L, NaN where no co-rating, NaN
 * diagonal.  Rows are given as CSR (rowptr int64[L+1], ids, ratings) in data order and sorted by
 * ID here (data.go:236-243 sorts). */
void or_knn_sims(int32_t kind, int32_t L, const int64_t* rowptr, const int32_t* ids,
                 const double* ratings, double* sims);

/* Rows [row_begin, row_end) of the knn.go pair loop against every partner (cpu_baseline sample). */
void or_knn_sims_rows(int32_t kind, int32_t L, const int64_t* rowptr, const int32_t* sorted_ids,
                      const double* sorted_r, int32_t row_begin, int32_t row_end, double* out);

/* knn.go:75-141 KNN.Predict.  The candidates are ordered as Go 1.24's sort.Sort (pdqsort, unstable)
 * orders them (knn.go:107-108), restated call for call in oracle.c -- the tie order among equal
 * similarities, and so the top-k boundary and the summation order, are the reference's.
 * type: 0 basic, 1 centered, 2 zscore, 3 baseline.  right_* is RightRatings CSR in data order. */
void or_knn_predict(int32_t type, int32_t L, const double* sims, const int64_t* right_rowptr,
                    const int32_t* right_ids, const double* right_r, const double* means,
                    const double* stddevs, const double* bias, double global_mean,
                    int32_t k, int32_t min_k, int64_t n, const int32_t* left, const int32_t* right,
                    double* out);
/* The same with ties broken by candidate position (sim desc, position asc): the library's
 * RS_TIE_STABLE option. */
void or_knn_predict_stable(int32_t type, int32_t L, const double* sims, const int64_t* right_rowptr,
                           const int32_t* right_ids, const double* right_r, const double* means,
                           const double* stddevs, const double* bias, double global_mean,
                           int32_t k, int32_t min_k, int64_t n, const int32_t* left, const int32_t* right,
                           double* out);
/* Go's sort.Sort permutation for keys under Less(i, j) = key_i > key_j (perm[t] = input position). */
void or_go_sort_desc(int64_t n, const double* keys, int64_t* perm);

/* base.go:135-163 BaseLine.Fit (bias-only SGD, used by KNN baseline knn.go:179-187). */
void or_baseline_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                     int32_t epochs, double lr, double reg, double* bu, double* bi, double* gb);

/* slope_one.go:47-93 SlopeOne.Fit with nJobs = 1: dev (L x L, L = items) from the item CSR (rows =
 * ItemRatings in data order, user ids; sorted by ID here, slope_one.go:62). */
void or_slope_one_fit(int32_t L, const int64_t* rowptr, const int32_t* ids, const double* ratings,
                      double* dev);

/* slope_one.go:21-45 SlopeOne.Predict for inner ids (-1 = unknown); user CSR = UserRatings in data
 * order; userMeans = means() (data.go:222-235). */
void or_slope_one_predict(int32_t L, const double* dev, int32_t n_users, const int64_t* user_rowptr,
                          const int32_t* user_items, const double* user_ratings, double global_mean,
                          int64_t n, const int32_t* users, const int32_t* items, double* out);

/* ---- restatements of THIS build's own GPU schedules (not of the reference) ---- */

/* Fast-mode SGD schedule of recommend-sys_amd/csrc/sgd.hip, single-threaded: work items are
 * (user, CSR range) chunks; all chunks advance in lock-step rounds (round t processes the t-th
 * rating of every live chunk in chunk order), which is the schedule the GPU runs when every chunk
 * is resident; per-chunk local GlobalBias, folded at epoch end as gb += sum(n_w * dgb_w) / nnz.
 * A split user's P row and bias become the count-weighted average of its pieces' end states
 * (P += sum_pieces len/deg * (p_end - p_start)), applied in piece order.  Used for RMSE-parity
 * studies and for the race-free factor parity test (inputs where no two chunks share an item). */
void or_svd_fit_chunked(int32_t n_users, const int64_t* rowptr, const int32_t* items,
                        const double* r, int32_t chunk, int32_t k, int32_t epochs, double lr,
                        double reg, double* P, double* Q, double* bu, double* bi, double* gb);

/* The FAST schedules' GlobalBias warm start: mean over ratings of (r - b_u - b_i). */
double or_gb_warm_start(int32_t n_users, const int64_t* rowptr, const int32_t* items,
                        const double* r, const double* bu, const double* bi);

/* or_svdpp_fit_userwise in its O(nnz k) lazy affine form (rows without repeated items). */
void or_svdpp_fit_lazy(int32_t n_users, const int64_t* rowptr, const int32_t* items, const double* r,
                       int32_t k, int32_t epochs, double lr, double reg, double* P, double* Q, double* Y,
                       double* bu, double* bi, double* gb);
/* Restatement of the GPU FAST SVD++ schedule (svdpp.hip): user rows processed one after another,
 * each with the literal per-rating reference updates (svd.go:352-424) restricted to that user's row,
 * a user-local GlobalBias copy folded at epoch end as in or_svd_fit_chunked.  Equal to the GPU's
 * lazy-y wave kernel when no two users share an item (race-free input). */
void or_svdpp_fit_userwise(int32_t n_users, const int64_t* rowptr, const int32_t* items,
                           const double* r, int32_t k, int32_t epochs, double lr, double reg,
                           double* P, double* Q, double* Y, double* bu, double* bi, double* gb);

/* CPU baselines with the reference's own goroutine fan-out, restated with OpenMP (bench only). */
void or_svdpp_fit_jobs(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                       int32_t n_users, int32_t k, int32_t epochs, double lr, double reg, double* P,
                       double* Q, double* Y, double* bu, double* bi, double* gb, int32_t n_jobs,
                       int64_t n_visit);
void or_knn_sims_rows_mt(int32_t kind, int32_t L, const int64_t* rowptr, const int32_t* sid,
                         const double* sr, int32_t row_begin, int32_t row_end, int32_t n_jobs, double* out);

#ifdef __cplusplus
}
#endif
#endif
