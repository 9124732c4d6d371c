/*
 * oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY: loaded by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product path.
 * See oracle.h for what each function restates and how the restatement is pinned.
 *
 * Built with -O2 -ffp-contract=off: Go on amd64 never fuses a*b+c, so neither may the oracle.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* open-addressing map int64 -> int32 for first-appearance inner ids (data.go:137-151)          */

typedef struct {
    int64_t* keys;
    int32_t* vals;
    uint8_t* used;
    int64_t cap;
} idmap;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

static int idmap_init(idmap* m, int64_t n) {
    int64_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    m->cap = cap;
    m->keys = (int64_t*)malloc((size_t)cap * sizeof(int64_t));
    m->vals = (int32_t*)malloc((size_t)cap * sizeof(int32_t));
    m->used = (uint8_t*)calloc((size_t)cap, 1);
    return (m->keys && m->vals && m->used) ? 0 : -1;
}

static void idmap_free(idmap* m) {
    free(m->keys);
    free(m->vals);
    free(m->used);
}

/* returns the inner id of key, inserting next_id if absent */
static int32_t idmap_get_or_put(idmap* m, int64_t key, int32_t* next_id) {
    uint64_t h = mix64((uint64_t)key) & (uint64_t)(m->cap - 1);
    while (m->used[h]) {
        if (m->keys[h] == key) return m->vals[h];
        h = (h + 1) & (uint64_t)(m->cap - 1);
    }
    m->used[h] = 1;
    m->keys[h] = key;
    m->vals[h] = (*next_id)++;
    return m->vals[h];
}

int or_trainset_ids(int64_t n, const int64_t* users, const int64_t* items, int32_t* inner_u,
                    int32_t* inner_i, int32_t* n_users, int32_t* n_items) {
    idmap mu, mi;
    if (idmap_init(&mu, n) || idmap_init(&mi, n)) return -1;
    int32_t nu = 0, ni = 0;
    /* data.go:138-143: all users first ... */
    for (int64_t t = 0; t < n; t++) inner_u[t] = idmap_get_or_put(&mu, users[t], &nu);
    /* data.go:146-151: ... then all items */
    for (int64_t t = 0; t < n; t++) inner_i[t] = idmap_get_or_put(&mi, items[t], &ni);
    *n_users = nu;
    *n_items = ni;
    idmap_free(&mu);
    idmap_free(&mi);
    return 0;
}

/* gonum floats.Dot restated as a sequential sum (see oracle.h) */
static double dot(const double* a, const double* b, int32_t k) {
    double s = 0.0;
    for (int32_t f = 0; f < k; f++) s += a[f] * b[f];
    return s;
}

/* ------------------------------------------------------------------------------------------ */
/* SVD                                                                                         */

void or_svd_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r, int32_t k,
                int32_t epochs, double lr, double reg, double* P, double* Q, double* bu,
                double* bi, double* gb) {
    double GB = *gb;
    for (int32_t epoch = 0; epoch < epochs; epoch++) {      /* svd.go:92 */
        for (int64_t t = 0; t < n; t++) {                   /* svd.go:93: train-set order (Q3) */
            const int32_t uu = u[t], ii = i[t];
            const double rating = r[t];
            const double userBias = bu[uu];                 /* svd.go:97-98: pre-update copies */
            const double itemBias = bi[ii];
            double* pu = P + (int64_t)uu * k;               /* svd.go:99-100: ALIASES (Q1) */
            double* qi = Q + (int64_t)ii * k;
            /* svd.go:102 -> Predict svd.go:35-48: ((gb + bu) + bi) + dot(p, q) */
            double pred = GB;
            pred += bu[uu];
            pred += bi[ii];
            pred += dot(pu, qi, k);
            const double diff = pred - rating;
            GB -= lr * diff;                                /* svd.go:105-106 (Q2) */
            bu[uu] -= lr * (diff + reg * userBias);         /* svd.go:108-109 */
            bi[ii] -= lr * (diff + reg * itemBias);         /* svd.go:111-112 */
            /* svd.go:114-120: a = q*diff; b = p*reg; a += b; a *= lr; p -= a */
            for (int32_t f = 0; f < k; f++) {
                double a = qi[f] * diff;
                double b = pu[f] * reg;
                a = a + b;
                a = a * lr;
                pu[f] = pu[f] - a;
            }
            /* svd.go:122-128: same with the ALREADY UPDATED p (Q1) */
            for (int32_t f = 0; f < k; f++) {
                double a = pu[f] * diff;
                double b = qi[f] * reg;
                a = a + b;
                a = a * lr;
                qi[f] = qi[f] - a;
            }
        }
    }
    *gb = GB;
}

/* Restatement of the GPU FAST schedules' GlobalBias semantics over explicit work items: the ratings
 * (in the given order) are cut into n_works consecutive segments [work_off[w], work_off[w+1]); each
 * runs the per-rating updates of svd.go:93-129 with a work-local GlobalBias copy starting from the
 * epoch's value, P/Q/bu/bi updated in place, works one after another; after the epoch
 * GB += sum_w n_w (gb_w - GB) / n (the fixed-order fold of sgd.hip / sgd_tile.hip).  Equal to the GPU
 * kernels when their works do not race (one wave, or works with disjoint users and items). */
/* The FAST schedules' GlobalBias: every work w runs svd.go:102-106's chain gb <- gb - lr (gb + e_j) from the
 * epoch-start value GB on its own ratings, and the works are folded after the epoch.  compose = 0 (the
 * multi-GPU exchanges): GB += sum_w n_w (g_w - GB) / n, the count-weighted mean of the works' moves.
 * compose = 1 (the single-GPU tile schedule, round 6): the works' affine maps g -> a_w g + b_w, a_w = (1 - lr)^n_w,
 * b_w = g_w - a_w GB, composed in work order -- GB' = A GB + sum_w c_w b_w with c_w the product of a_v over the
 * works after w and A over all -- what the sequential chain gives when each work's e_j are its own (sgd.hip
 * svd_epoch_epilogue_kernel evaluates the same sum). */
void or_svd_fit_works2(int64_t n, const int32_t* u, const int32_t* i, const double* r, int64_t n_works,
                       const int64_t* work_off, int32_t k, int32_t epochs, double lr, double reg, double* P,
                       double* Q, double* bu, double* bi, double* gb, int32_t compose) {
    double GB = *gb;
    double* gend = (double*)malloc((size_t)(n_works > 0 ? n_works : 1) * sizeof(double));
    for (int32_t epoch = 0; epoch < epochs; epoch++) {
        double fold = 0.0;
        for (int64_t w = 0; w < n_works; w++) {
            double g = GB;
            for (int64_t t = work_off[w]; t < work_off[w + 1]; t++) {
                const int32_t uu = u[t], ii = i[t];
                const double userBias = bu[uu], itemBias = bi[ii];
                double* pu = P + (int64_t)uu * k;
                double* qi = Q + (int64_t)ii * k;
                double pred = g;
                pred += bu[uu];
                pred += bi[ii];
                pred += dot(pu, qi, k);
                const double diff = pred - r[t];
                g -= lr * diff;
                bu[uu] -= lr * (diff + reg * userBias);
                bi[ii] -= lr * (diff + reg * itemBias);
                for (int32_t f = 0; f < k; f++) pu[f] = pu[f] - (qi[f] * diff + pu[f] * reg) * lr;
                for (int32_t f = 0; f < k; f++) qi[f] = qi[f] - (pu[f] * diff + qi[f] * reg) * lr;
            }
            fold += (double)(work_off[w + 1] - work_off[w]) * (g - GB);
            gend[w] = g;
        }
        if (compose == 2) {
            const double l1 = log1p(-lr);
            double num = 0.0, den = 0.0, later = 0.0;
            for (int64_t w = 0; w < n_works; w++) {
                const double nw = (double)(work_off[w + 1] - work_off[w]);
                const double a = exp(nw * l1);
                num += gend[w] - a * GB;
                den += 1.0 - a;
                later += nw;
            }
            const double A = exp(later * l1);
            if (den > 0.0) GB = A * GB + (1.0 - A) * (num / den);
        } else if (compose) {
            const double l1 = log1p(-lr);
            double acc = 0.0, later = 0.0;  /* sum of c_w b_w; ratings of the works after w */
            for (int64_t w = n_works - 1; w >= 0; w--) {
                const double nw = (double)(work_off[w + 1] - work_off[w]);
                const double b = gend[w] - exp(nw * l1) * GB;
                acc += exp(later * l1) * b;
                later += nw;
            }
            GB = exp(later * l1) * GB + acc;
        } else if (n > 0) {
            GB += fold / (double)n;
        }
    }
    free(gend);
    *gb = GB;
}

void or_svd_fit_works(int64_t n, const int32_t* u, const int32_t* i, const double* r, int64_t n_works,
                      const int64_t* work_off, int32_t k, int32_t epochs, double lr, double reg, double* P,
                      double* Q, double* bu, double* bi, double* gb) {
    or_svd_fit_works2(n, u, i, r, n_works, work_off, k, epochs, lr, reg, P, Q, bu, bi, gb, 0);
}

/* The tile schedule's hot-run damping (round 5, sgd_tile.hip; a rule of this build, not of svd.go) on top of
 * or_svd_fit_works2: a run is a maximal stretch of one item's ratings inside a work (the kernel's (item, tile)
 * run when runs are not cut).  The run trains as svd.go:93-128 does; at its end, where the item's runs in flight
 * R = deg[item] x kconc reach 4, its closing fractions f_q = 1 - exp(-lr (sum |p_u|^2 + n reg)) (|p_u|^2 over the
 * factor columns, before each rating's update) and f_b = 1 - (1 - lr (1 + reg))^n give weights
 * w = min(1, 1 / (R f)), and the item row keeps only w of the run's move: q = q0 + w_q (q - q0),
 * b_i = b0 + w_b (b_i - b0).  P, b_u and GlobalBias are not damped. */
void or_svd_fit_works_damped(int64_t n, const int32_t* u, const int32_t* i, const double* r, int64_t n_works,
                             const int64_t* work_off, const int32_t* deg, double kconc, int32_t k, int32_t epochs,
                             double lr, double reg, double* P, double* Q, double* bu, double* bi, double* gb,
                             int32_t compose) {
    double GB = *gb;
    double* gend = (double*)malloc((size_t)(n_works > 0 ? n_works : 1) * sizeof(double));
    double* q0 = (double*)malloc((size_t)(k > 0 ? k : 1) * sizeof(double));
    const double l1 = log1p(-lr);
    for (int32_t epoch = 0; epoch < epochs; epoch++) {
        double fold = 0.0;
        for (int64_t w = 0; w < n_works; w++) {
            double g = GB, hp = 0.0, b0 = 0.0;
            int64_t nrun = 0;
            for (int64_t t = work_off[w]; t < work_off[w + 1]; t++) {
                const int32_t uu = u[t], ii = i[t];
                double* pu = P + (int64_t)uu * k;
                double* qi = Q + (int64_t)ii * k;
                if (t == work_off[w] || i[t - 1] != ii) {  /* a run starts */
                    memcpy(q0, qi, (size_t)k * sizeof(double));
                    b0 = bi[ii];
                    hp = 0.0;
                    nrun = 0;
                }
                const double userBias = bu[uu], itemBias = bi[ii];
                double pred = g;
                pred += bu[uu];
                pred += bi[ii];
                pred += dot(pu, qi, k);
                const double diff = pred - r[t];
                hp += dot(pu, pu, k);
                nrun++;
                g -= lr * diff;
                bu[uu] -= lr * (diff + reg * userBias);
                bi[ii] -= lr * (diff + reg * itemBias);
                for (int32_t f = 0; f < k; f++) pu[f] = pu[f] - (qi[f] * diff + pu[f] * reg) * lr;
                for (int32_t f = 0; f < k; f++) qi[f] = qi[f] - (pu[f] * diff + qi[f] * reg) * lr;
                if (t + 1 == work_off[w + 1] || i[t + 1] != ii) {  /* the run ends: its move, damped */
                    const double R = (double)deg[ii] * kconc;
                    if (R >= 4.0) {
                        const double fq = 1.0 - exp(-lr * (hp + (double)nrun * reg));
                        const double fb = 1.0 - exp((double)nrun * log(1.0 - lr * (1.0 + reg)));
                        const double wq = fmin(1.0, 1.0 / (R * fq)), wb = fmin(1.0, 1.0 / (R * fb));
                        for (int32_t f = 0; f < k; f++) qi[f] = q0[f] + wq * (qi[f] - q0[f]);
                        bi[ii] = b0 + wb * (bi[ii] - b0);
                    }
                }
            }
            fold += (double)(work_off[w + 1] - work_off[w]) * (g - GB);
            gend[w] = g;
        }
        if (compose == 2) {
            double num = 0.0, den = 0.0, later = 0.0;
            for (int64_t w = 0; w < n_works; w++) {
                const double nw = (double)(work_off[w + 1] - work_off[w]);
                const double a = exp(nw * l1);
                num += gend[w] - a * GB;
                den += 1.0 - a;
                later += nw;
            }
            const double A = exp(later * l1);
            if (den > 0.0) GB = A * GB + (1.0 - A) * (num / den);
        } else if (n > 0) {
            GB += fold / (double)n;
        }
    }
    free(q0);
    free(gend);
    *gb = GB;
}

void or_svd_predict(int64_t n, const int32_t* u, const int32_t* i, int32_t k, const double* P,
                    const double* Q, const double* bu, const double* bi, double gb, double* out) {
    for (int64_t t = 0; t < n; t++) {
        const int32_t uu = u[t], ii = i[t];
        double ret = gb;                                    /* svd.go:35 */
        if (uu >= 0) ret += bu[uu];                         /* svd.go:37-39 */
        if (ii >= 0) ret += bi[ii];                         /* svd.go:41-43 */
        if (uu >= 0 && ii >= 0) ret += dot(P + (int64_t)uu * k, Q + (int64_t)ii * k, k);
        out[t] = ret;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* SVD++                                                                                       */

/* data.go:185-199 UserRatings: per inner user, (item, position) in data order -> CSR */
static void build_user_csr(int64_t n, const int32_t* u, int32_t n_users, int64_t** rowptr_out,
                           int64_t** pos_out) {
    int64_t* rowptr = (int64_t*)calloc((size_t)n_users + 1, sizeof(int64_t));
    int64_t* pos = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    for (int64_t t = 0; t < n; t++) rowptr[u[t] + 1]++;
    for (int32_t x = 0; x < n_users; x++) rowptr[x + 1] += rowptr[x];
    int64_t* fill = (int64_t*)malloc(((size_t)n_users + 1) * sizeof(int64_t));
    memcpy(fill, rowptr, ((size_t)n_users + 1) * sizeof(int64_t));
    for (int64_t t = 0; t < n; t++) pos[fill[u[t]]++] = t;
    free(fill);
    *rowptr_out = rowptr;
    *pos_out = pos;
}

/* svd.go:271-282 ensembleImplFactors: e = (sum_j Y[j]) / sqrt(|N(u)|), floats.Add in N(u) order */
static void ensemble(const int64_t* rowptr, const int64_t* pos, const int32_t* items, int32_t uu,
                     int32_t k, const double* Y, double* e) {
    for (int32_t f = 0; f < k; f++) e[f] = 0.0;
    int64_t count = 0;
    for (int64_t x = rowptr[uu]; x < rowptr[uu + 1]; x++) {
        const double* y = Y + (int64_t)items[pos[x]] * k;
        for (int32_t f = 0; f < k; f++) e[f] = e[f] + y[f];
        count++;
    }
    const double s = sqrt((double)count);
    for (int32_t f = 0; f < k; f++) e[f] /= s;              /* utils.go:63-67 divConst */
}

void or_svdpp_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                  int32_t n_users, int32_t k, int32_t epochs, double lr, double reg, double* P,
                  double* Q, double* Y, double* bu, double* bi, double* gb) {
    int64_t *rowptr, *pos;
    build_user_csr(n, u, n_users, &rowptr, &pos);           /* svd.go:342 */
    double* e = (double*)malloc((size_t)k * sizeof(double));
    double GB = *gb;
    for (int32_t epoch = 0; epoch < epochs; epoch++) {      /* svd.go:350 */
        for (int64_t t = 0; t < n; t++) {                   /* svd.go:352 */
            const int32_t uu = u[t], ii = i[t];
            const double rating = r[t];
            const double userBias = bu[uu];                 /* svd.go:358-361 (aliases) */
            const double itemBias = bi[ii];
            double* pu = P + (int64_t)uu * k;
            double* qi = Q + (int64_t)ii * k;
            /* svd.go:363 internalPredict svd.go:290-305 */
            double pred = GB;
            pred += bu[uu];
            pred += bi[ii];
            ensemble(rowptr, pos, i, uu, k, Y, e);
            double s = 0.0;                                 /* tmp = 0 + p + e; dot(tmp, q) */
            for (int32_t f = 0; f < k; f++) {
                double tmp = 0.0;
                tmp = tmp + pu[f];
                tmp = tmp + e[f];
                s += tmp * qi[f];
            }
            pred += s;
            const double diff = pred - rating;              /* svd.go:364 */
            GB -= lr * diff;                                /* svd.go:366-367 */
            bu[uu] -= lr * (diff + reg * userBias);         /* svd.go:370-371 */
            bi[ii] -= lr * (diff + reg * itemBias);         /* svd.go:374-375 */
            for (int32_t f = 0; f < k; f++) {               /* svd.go:378-384, old q */
                double a = qi[f] * diff;
                double b = pu[f] * reg;
                a = a + b;
                a = a * lr;
                pu[f] = pu[f] - a;
            }
            for (int32_t f = 0; f < k; f++) {               /* svd.go:387-396, NEW p plus e */
                double a = pu[f];
                a = a + e[f];                               /* len(emImpFactor) > 0 (L388) */
                a = a * diff;
                double b = qi[f] * reg;
                a = a + b;
                a = a * lr;
                qi[f] = qi[f] - a;
            }
            /* svd.go:399-422: every j in N(u), with the NEW q_i (alias) */
            const double sq = sqrt((double)(rowptr[uu + 1] - rowptr[uu]));
            for (int64_t x = rowptr[uu]; x < rowptr[uu + 1]; x++) {
                double* y = Y + (int64_t)i[pos[x]] * k;
                for (int32_t f = 0; f < k; f++) {
                    double a = qi[f] * diff;                /* L410-411 */
                    a = a / sq;                             /* L412 divConst */
                    double b = y[f] * reg;                  /* L413-414 */
                    a = a + b;                              /* L415 */
                    a = a * lr;                             /* L416 */
                    y[f] = y[f] - a;                        /* L417 */
                }
            }
        }
    }
    *gb = GB;
    free(e);
    free(rowptr);
    free(pos);
}

/* or_svdpp_fit with the reference's own parallelism (CPU baseline only): svd.go:399-422 splits the
 * y-update loop of EVERY rating over nJobs goroutines (contiguous ranges [nRating*j/nJobs,
 * nRating*(j+1)/nJobs)) and waits for them (wg.Wait) before the next rating; restated as one OpenMP
 * fork/join per rating with the same static contiguous split.  Same arithmetic per element.  Each epoch
 * visits the first n_visit ratings (n_visit = n: the whole epoch; less: a timed slice of it, N(u) still
 * over all n ratings). */
void or_svdpp_fit_jobs(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                       int32_t n_users, int32_t k, int32_t epochs, double lr, double reg, double* P,
                       double* Q, double* Y, double* bu, double* bi, double* gb, int32_t n_jobs,
                       int64_t n_visit) {
    int64_t *rowptr, *pos;
    build_user_csr(n, u, n_users, &rowptr, &pos);
    double* e = (double*)malloc((size_t)k * sizeof(double));
    double GB = *gb;
    if (n_visit > n) n_visit = n;
    for (int32_t epoch = 0; epoch < epochs; epoch++) {
        for (int64_t t = 0; t < n_visit; t++) {
            const int32_t uu = u[t], ii = i[t];
            const double userBias = bu[uu], itemBias = bi[ii];
            double* pu = P + (int64_t)uu * k;
            double* qi = Q + (int64_t)ii * k;
            double pred = GB;
            pred += bu[uu];
            pred += bi[ii];
            ensemble(rowptr, pos, i, uu, k, Y, e);
            double s = 0.0;
            for (int32_t f = 0; f < k; f++) {
                double tmp = 0.0;
                tmp = tmp + pu[f];
                tmp = tmp + e[f];
                s += tmp * qi[f];
            }
            pred += s;
            const double diff = pred - r[t];
            GB -= lr * diff;
            bu[uu] -= lr * (diff + reg * userBias);
            bi[ii] -= lr * (diff + reg * itemBias);
            for (int32_t f = 0; f < k; f++) pu[f] = pu[f] - (qi[f] * diff + pu[f] * reg) * lr;
            for (int32_t f = 0; f < k; f++) qi[f] = qi[f] - ((pu[f] + e[f]) * diff + qi[f] * reg) * lr;
            const int64_t b0 = rowptr[uu], nr = rowptr[uu + 1] - b0;
            const double sq = sqrt((double)nr);
#pragma omp parallel for num_threads(n_jobs) schedule(static)
            for (int32_t j = 0; j < n_jobs; j++) {          /* svd.go:402-420: one goroutine per job */
                for (int64_t x = b0 + nr * j / n_jobs; x < b0 + nr * (j + 1) / n_jobs; x++) {
                    double* y = Y + (int64_t)i[pos[x]] * k;
                    for (int32_t f = 0; f < k; f++) {
                        double a = qi[f] * diff;
                        a = a / sq;
                        double b = y[f] * reg;
                        a = a + b;
                        a = a * lr;
                        y[f] = y[f] - a;
                    }
                }
            }
        }
    }
    *gb = GB;
    free(e);
    free(rowptr);
    free(pos);
}

void or_svdpp_predict(int64_t n_train, const int32_t* tu, const int32_t* ti, int32_t n_users,
                      int64_t n, const int32_t* u, const int32_t* i, int32_t k, const double* P,
                      const double* Q, const double* Y, const double* bu, const double* bi,
                      double gb, double* out) {
    int64_t *rowptr, *pos;
    build_user_csr(n_train, tu, n_users, &rowptr, &pos);
    double* e = (double*)malloc((size_t)k * sizeof(double));
    for (int64_t t = 0; t < n; t++) {
        const int32_t uu = u[t], ii = i[t];
        double ret = gb;
        if (uu >= 0) ret += bu[uu];
        if (ii >= 0) ret += bi[ii];
        if (uu >= 0 && ii >= 0) {
            ensemble(rowptr, pos, ti, uu, k, Y, e);
            const double* pu = P + (int64_t)uu * k;
            const double* qi = Q + (int64_t)ii * k;
            double s = 0.0;
            for (int32_t f = 0; f < k; f++) {
                double tmp = 0.0;
                tmp = tmp + pu[f];
                tmp = tmp + e[f];
                s += tmp * qi[f];
            }
            ret += s;
        }
        out[t] = ret;
    }
    free(e);
    free(rowptr);
    free(pos);
}

/* ------------------------------------------------------------------------------------------ */
/* NMF                                                                                         */

void or_nmf_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r, int32_t n_users,
                int32_t n_items, int32_t k, int32_t epochs, double reg, int32_t as_written,
                double* P, double* Q) {
    const size_t su = (size_t)n_users * k, si = (size_t)n_items * k;
    double* userUp = (double*)malloc(su * sizeof(double));  /* svd.go:173-176 */
    double* userDown = (double*)malloc(su * sizeof(double));
    double* itemUp = (double*)malloc(si * sizeof(double));
    double* itemDown = (double*)malloc(si * sizeof(double));
    double* buffer = (double*)malloc((size_t)k * sizeof(double));
    for (int32_t epoch = 0; epoch < epochs; epoch++) {      /* svd.go:178 */
        memset(userUp, 0, su * sizeof(double));             /* svd.go:180-183 */
        memset(userDown, 0, su * sizeof(double));
        memset(itemUp, 0, si * sizeof(double));
        memset(itemDown, 0, si * sizeof(double));
        for (int64_t t = 0; t < n; t++) {                   /* svd.go:186 */
            const int32_t uu = u[t], ii = i[t];
            const double rating = r[t];
            const double* pu = P + (int64_t)uu * k;
            const double* qi = Q + (int64_t)ii * k;
            const double prediction = dot(pu, qi, k);       /* svd.go:190 -> 144 */
            double* uup = userUp + (int64_t)uu * k;
            double* udn = userDown + (int64_t)uu * k;
            double* iup = itemUp + (int64_t)ii * k;
            double* idn = itemDown + (int64_t)ii * k;
            for (int32_t f = 0; f < k; f++) uup[f] = uup[f] + qi[f] * rating;      /* L193-197 */
            for (int32_t f = 0; f < k; f++) udn[f] = udn[f] + qi[f] * prediction;  /* L200-204 */
            for (int32_t f = 0; f < k; f++) udn[f] = udn[f] + pu[f] * reg;         /* L206-210 */
            for (int32_t f = 0; f < k; f++) iup[f] = iup[f] + pu[f] * rating;      /* L214-218 */
            for (int32_t f = 0; f < k; f++) idn[f] = idn[f] + pu[f] * prediction;  /* L221-225 */
            for (int32_t f = 0; f < k; f++) idn[f] = idn[f] + qi[f] * reg;         /* L227-231 */
        }
        for (int32_t x = 0; x < n_users; x++) {             /* svd.go:236-241 */
            double* pu = P + (int64_t)x * k;
            for (int32_t f = 0; f < k; f++) {
                buffer[f] = userUp[(int64_t)x * k + f];
                buffer[f] = buffer[f] / userDown[(int64_t)x * k + f];
                pu[f] = pu[f] * buffer[f];
            }
        }
        for (int32_t x = 0; x < n_items; x++) {             /* svd.go:243-249 */
            double* qi = Q + (int64_t)x * k;
            for (int32_t f = 0; f < k; f++) {
                const int64_t o = (int64_t)x * k + f;
                buffer[f] = itemUp[o];                      /* L244: copy BEFORE the divide */
                itemUp[o] = itemUp[o] / itemDown[o];        /* L246: divides itemUp in place */
                qi[f] = qi[f] * (as_written ? buffer[f] : itemUp[o]); /* L248 (Q5) */
            }
        }
    }
    free(userUp);
    free(userDown);
    free(itemUp);
    free(itemDown);
    free(buffer);
}

void or_nmf_predict(int64_t n, const int32_t* u, const int32_t* i, int32_t k, const double* P,
                    const double* Q, double* out) {
    for (int64_t t = 0; t < n; t++) {                       /* svd.go:140-147 */
        if (u[t] >= 0 && i[t] >= 0)
            out[t] = dot(P + (int64_t)u[t] * k, Q + (int64_t)i[t] * k, k);
        else
            out[t] = 0.0;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Similarities                                                                                */

static double sim_cosine(int64_t na, const int32_t* a_id, const double* a_r, int64_t nb,
                         const int32_t* b_id, const double* b_r) {
    double m = 0.0, n = 0.0, l = 0.0;                       /* sim.go:11 */
    int64_t ptr = 0;
    for (int64_t x = 0; x < na; x++) {                      /* sim.go:13 */
        while (ptr < nb && b_id[ptr] < a_id[x]) ptr++;      /* sim.go:14-16 */
        if (ptr < nb && b_id[ptr] == a_id[x]) {             /* sim.go:17 */
            const double ra = a_r[x], rb = b_r[ptr];
            m += ra * ra;                                   /* sim.go:19-21 */
            n += rb * rb;
            l += ra * rb;
        }
    }
    return l / (sqrt(m) * sqrt(n));                         /* sim.go:24 */
}

static double sim_msd(int64_t na, const int32_t* a_id, const double* a_r, int64_t nb,
                      const int32_t* b_id, const double* b_r) {
    double count = 0.0, sum = 0.0;                          /* sim.go:29 */
    int64_t ptr = 0;
    for (int64_t x = 0; x < na; x++) {
        while (ptr < nb && b_id[ptr] < a_id[x]) ptr++;
        if (ptr < nb && b_id[ptr] == a_id[x]) {
            const double d = a_r[x] - b_r[ptr];
            sum += d * d;                                   /* sim.go:37 */
            count++;
        }
    }
    return 1.0 / (sum / count + 1.0);                       /* sim.go:43 */
}

static double sim_pearson(int64_t na, const int32_t* a_id, const double* a_r, int64_t nb,
                          const int32_t* b_id, const double* b_r) {
    double count = 0.0, sum = 0.0;                          /* sim.go:49-54: mean over ALL of a */
    for (int64_t x = 0; x < na; x++) {
        sum += a_r[x];
        count += 1;
    }
    const double meanA = sum / count;
    count = 0.0;                                            /* sim.go:57-62 */
    sum = 0.0;
    for (int64_t x = 0; x < nb; x++) {
        sum += b_r[x];
        count += 1;
    }
    const double meanB = sum / count;
    double m = 0.0, n = 0.0, l = 0.0;                       /* sim.go:65-79 */
    int64_t ptr = 0;
    for (int64_t x = 0; x < na; x++) {
        while (ptr < nb && b_id[ptr] < a_id[x]) ptr++;
        if (ptr < nb && b_id[ptr] == a_id[x]) {
            const double ra = a_r[x] - meanA;
            const double rb = b_r[ptr] - meanB;
            m += ra * ra;
            n += rb * rb;
            l += ra * rb;
        }
    }
    return l / (sqrt(m) * sqrt(n));                         /* sim.go:80 */
}

double or_sim(int32_t kind, int64_t na, const int32_t* a_id, const double* a_r, int64_t nb,
              const int32_t* b_id, const double* b_r) {
    switch (kind) {
        case 0: return sim_cosine(na, a_id, a_r, nb, b_id, b_r);
        case 1: return sim_msd(na, a_id, a_r, nb, b_id, b_r);
        default: return sim_pearson(na, a_id, a_r, nb, b_id, b_r);
    }
}

typedef struct {
    int32_t id;
    double r;
} idr;

static int cmp_idr(const void* x, const void* y) {
    const idr* a = (const idr*)x;
    const idr* b = (const idr*)y;
    return (a->id > b->id) - (a->id < b->id);
}

void or_knn_sims(int32_t kind, int32_t L, const int64_t* rowptr, const int32_t* ids,
                 const double* ratings, double* sims) {
    const int64_t nnz = rowptr[L];
    int32_t* sid = (int32_t*)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int32_t));
    double* sr = (double*)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(double));
    idr* tmp = (idr*)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(idr));
    /* data.go:236-243 sorts(): each row sorted by ID (unique IDs: any sort gives this order) */
    for (int32_t x = 0; x < L; x++) {
        const int64_t b = rowptr[x], e = rowptr[x + 1];
        for (int64_t t = b; t < e; t++) {
            tmp[t - b].id = ids[t];
            tmp[t - b].r = ratings[t];
        }
        qsort(tmp, (size_t)(e - b), sizeof(idr), cmp_idr);
        for (int64_t t = b; t < e; t++) {
            sid[t] = tmp[t - b].id;
            sr[t] = tmp[t - b].r;
        }
    }
    free(tmp);
    const int64_t LL = (int64_t)L * L;
    for (int64_t t = 0; t < LL; t++) sims[t] = NAN;         /* knn.go:157/161 newNanMatrix */
    for (int32_t a = 0; a < L; a++) {                       /* knn.go:199 (nJobs = 1) */
        for (int32_t b = 0; b < L; b++) {                   /* knn.go:201 */
            if (a == b) continue;                           /* knn.go:202: diagonal stays NaN */
            if (!isnan(sims[(int64_t)a * L + b])) continue; /* knn.go:203 */
            const double v = or_sim(kind, rowptr[a + 1] - rowptr[a], sid + rowptr[a],
                                    sr + rowptr[a], rowptr[b + 1] - rowptr[b], sid + rowptr[b],
                                    sr + rowptr[b]);
            if (!isnan(v)) {                                /* knn.go:205-208 */
                sims[(int64_t)a * L + b] = v;
                sims[(int64_t)b * L + a] = v;
            }
        }
    }
    free(sid);
    free(sr);
}

void or_knn_sims_rows(int32_t kind, int32_t L, const int64_t* rowptr, const int32_t* sid,
                      const double* sr, int32_t row_begin, int32_t row_end, double* out) {
    for (int32_t a = row_begin; a < row_end; a++)
        for (int32_t b = 0; b < L; b++)
            out[(int64_t)(a - row_begin) * L + b] =
                a == b ? NAN
                       : or_sim(kind, rowptr[a + 1] - rowptr[a], sid + rowptr[a], sr + rowptr[a],
                                rowptr[b + 1] - rowptr[b], sid + rowptr[b], sr + rowptr[b]);
}

/* or_knn_sims_rows on n_jobs threads (CPU baseline only): the rows split into contiguous ranges as
 * knn.go:192-216 splits them over its nJobs goroutines, every row against every partner. */
void or_knn_sims_rows_mt(int32_t kind, int32_t L, const int64_t* rowptr, const int32_t* sid,
                         const double* sr, int32_t row_begin, int32_t row_end, int32_t n_jobs, double* out) {
#pragma omp parallel for num_threads(n_jobs) schedule(static)
    for (int32_t a = row_begin; a < row_end; a++)
        for (int32_t b = 0; b < L; b++)
            out[(int64_t)(a - row_begin) * L + b] =
                a == b ? NAN
                       : or_sim(kind, rowptr[a + 1] - rowptr[a], sid + rowptr[a], sr + rowptr[a],
                                rowptr[b + 1] - rowptr[b], sid + rowptr[b], sr + rowptr[b]);
}

/* ------------------------------------------------------------------------------------------ */
/* KNN.Predict                                                                                 */

static const double* g_sim_row; /* comparator context (single-threaded oracle) */

typedef struct {
    int32_t id;
    double r;
    int64_t pos;
} cand;

static int cmp_cand(const void* x, const void* y) {
    const cand* a = (const cand*)x;
    const cand* b = (const cand*)y;
    const double sa = g_sim_row[a->id], sb = g_sim_row[b->id];
    if (sa > sb) return -1;                                 /* knn.go:43-45: desc by sim */
    if (sa < sb) return 1;
    return (a->pos > b->pos) - (a->pos < b->pos);           /* documented tie rule */
}

/* Go 1.24 sort.Sort (knn.go:107-108 sorts the CandidateSet with it; go.mod:3 pins go 1.24): pdqsort as in
 * the standard library's sort/zsortinterface.go, restated here call for call -- the same Less / Swap
 * sequence, so the same permutation of tied candidates (sort.Sort is not stable).  Less(i, j) =
 * sims[c_i] > sims[c_j] (knn.go:43-45), Swap exchanges two candidates (knn.go:46-48).  Restated from the
 * published algorithm of that release; no Go toolchain exists here or on the GPU boxes to run the
 * original, so the tie order is pinned by this restatement only. */
typedef struct {
    cand* c;
    const double* s;
} gosort;
static int g_less(const gosort* d, int64_t i, int64_t j) { return d->s[d->c[i].id] > d->s[d->c[j].id]; }
static void g_swap(gosort* d, int64_t i, int64_t j) {
    const cand t = d->c[i];
    d->c[i] = d->c[j];
    d->c[j] = t;
}
static int g_bits_len(uint64_t x) { /* math/bits.Len */
    int n = 0;
    while (x) {
        n++;
        x >>= 1;
    }
    return n;
}
static void g_insertion(gosort* d, int64_t a, int64_t b) {
    for (int64_t i = a + 1; i < b; i++)
        for (int64_t j = i; j > a && g_less(d, j, j - 1); j--) g_swap(d, j, j - 1);
}
static void g_sift_down(gosort* d, int64_t lo, int64_t hi, int64_t first) {
    int64_t root = lo;
    for (;;) {
        int64_t child = 2 * root + 1;
        if (child >= hi) return;
        if (child + 1 < hi && g_less(d, first + child, first + child + 1)) child++;
        if (!g_less(d, first + root, first + child)) return;
        g_swap(d, first + root, first + child);
        root = child;
    }
}
static void g_heap_sort(gosort* d, int64_t a, int64_t b) {
    const int64_t first = a, lo = 0, hi = b - a;
    for (int64_t i = (hi - 1) / 2; i >= 0; i--) g_sift_down(d, i, hi, first);
    for (int64_t i = hi - 1; i >= 0; i--) {
        g_swap(d, first, first + i);
        g_sift_down(d, lo, i, first);
    }
}
enum { G_UNKNOWN = 0, G_INCREASING = 1, G_DECREASING = 2 };
static void g_order2(gosort* d, int64_t* a, int64_t* b, int* swaps) {
    if (g_less(d, *b, *a)) {
        const int64_t t = *a;
        *a = *b;
        *b = t;
        (*swaps)++;
    }
}
static int64_t g_median(gosort* d, int64_t a, int64_t b, int64_t c, int* swaps) {
    g_order2(d, &a, &b, swaps);
    g_order2(d, &b, &c, swaps);
    g_order2(d, &a, &b, swaps);
    return b;
}
static int64_t g_median_adjacent(gosort* d, int64_t a, int* swaps) { return g_median(d, a - 1, a, a + 1, swaps); }
static int64_t g_choose_pivot(gosort* d, int64_t a, int64_t b, int* hint) {
    const int64_t l = b - a;
    int swaps = 0;
    int64_t i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
        if (l >= 50) { /* Tukey ninther */
            i = g_median_adjacent(d, i, &swaps);
            j = g_median_adjacent(d, j, &swaps);
            k = g_median_adjacent(d, k, &swaps);
        }
        j = g_median(d, i, j, k, &swaps);
    }
    *hint = swaps == 0 ? G_INCREASING : (swaps == 12 ? G_DECREASING : G_UNKNOWN);
    return j;
}
static void g_reverse(gosort* d, int64_t a, int64_t b) {
    for (int64_t i = a, j = b - 1; i < j; i++, j--) g_swap(d, i, j);
}
static int g_partial_insertion(gosort* d, int64_t a, int64_t b) {
    int64_t i = a + 1;
    for (int step = 0; step < 5; step++) {
        while (i < b && !g_less(d, i, i - 1)) i++;
        if (i == b) return 1;
        if (b - a < 50) return 0;
        g_swap(d, i, i - 1);
        if (i - a >= 2)
            for (int64_t j = i - 1; j >= 1; j--) {
                if (!g_less(d, j, j - 1)) break;
                g_swap(d, j, j - 1);
            }
        if (b - i >= 2)
            for (int64_t j = i + 1; j < b; j++) {
                if (!g_less(d, j, j - 1)) break;
                g_swap(d, j, j - 1);
            }
    }
    return 0;
}
static void g_break_patterns(gosort* d, int64_t a, int64_t b) {
    const int64_t length = b - a;
    if (length >= 8) {
        uint64_t r = (uint64_t)length; /* xorshift seeded with the length */
        const uint64_t modulus = (uint64_t)1 << g_bits_len((uint64_t)length);
        const int64_t idx = a + (length / 4) * 2 - 1;
        for (int t = 0; t < 3; t++) {
            r ^= r << 13;
            r ^= r >> 7;
            r ^= r << 17;
            int64_t other = (int64_t)(r & (modulus - 1));
            if (other >= length) other -= length;
            g_swap(d, idx - 1 + t, a + other);
        }
    }
}
static int64_t g_partition_equal(gosort* d, int64_t a, int64_t b, int64_t pivot) {
    g_swap(d, a, pivot);
    int64_t i = a + 1, j = b - 1;
    for (;;) {
        while (i <= j && !g_less(d, a, i)) i++;
        while (i <= j && g_less(d, a, j)) j--;
        if (i > j) break;
        g_swap(d, i, j);
        i++;
        j--;
    }
    return i;
}
static int64_t g_partition(gosort* d, int64_t a, int64_t b, int64_t pivot, int* already) {
    g_swap(d, a, pivot);
    int64_t i = a + 1, j = b - 1;
    while (i <= j && g_less(d, i, a)) i++;
    while (i <= j && !g_less(d, j, a)) j--;
    if (i > j) {
        g_swap(d, j, a);
        *already = 1;
        return j;
    }
    g_swap(d, i, j);
    i++;
    j--;
    for (;;) {
        while (i <= j && g_less(d, i, a)) i++;
        while (i <= j && !g_less(d, j, a)) j--;
        if (i > j) break;
        g_swap(d, i, j);
        i++;
        j--;
    }
    g_swap(d, j, a);
    *already = 0;
    return j;
}
static void g_pdqsort(gosort* d, int64_t a, int64_t b, int limit) {
    int was_balanced = 1, was_partitioned = 1;
    for (;;) {
        const int64_t length = b - a;
        if (length <= 12) {
            g_insertion(d, a, b);
            return;
        }
        if (limit == 0) {
            g_heap_sort(d, a, b);
            return;
        }
        if (!was_balanced) {
            g_break_patterns(d, a, b);
            limit--;
        }
        int hint;
        int64_t pivot = g_choose_pivot(d, a, b, &hint);
        if (hint == G_DECREASING) {
            g_reverse(d, a, b);
            pivot = (b - 1) - (pivot - a);
            hint = G_INCREASING;
        }
        if (was_balanced && was_partitioned && hint == G_INCREASING)
            if (g_partial_insertion(d, a, b)) return;
        if (a > 0 && !g_less(d, a - 1, pivot)) {
            a = g_partition_equal(d, a, b, pivot);
            continue;
        }
        int already = 0;
        const int64_t mid = g_partition(d, a, b, pivot, &already);
        was_partitioned = already;
        const int64_t left_len = mid - a, right_len = b - mid, threshold = length / 8;
        if (left_len < right_len) {
            was_balanced = left_len >= threshold;
            g_pdqsort(d, a, mid, limit);
            a = mid + 1;
        } else {
            was_balanced = right_len >= threshold;
            g_pdqsort(d, mid + 1, b, limit);
            b = mid;
        }
    }
}
static void go_sort_candidates(cand* c, int64_t n, const double* srow) {
    if (n <= 1) return;
    gosort d = {c, srow};
    g_pdqsort(&d, 0, n, g_bits_len((uint64_t)n));
}

/* Test helper: the permutation Go's sort.Sort leaves for keys under Less(i, j) = key_i > key_j (perm[t] =
 * the input position at output t). */
void or_go_sort_desc(int64_t n, const double* keys, int64_t* perm) {
    cand* c = (cand*)malloc((size_t)(n > 0 ? n : 1) * sizeof(cand));
    for (int64_t t = 0; t < n; t++) {
        c[t].id = (int32_t)t;
        c[t].r = 0.0;
        c[t].pos = t;
    }
    go_sort_candidates(c, n, keys);
    for (int64_t t = 0; t < n; t++) perm[t] = c[t].pos;
    free(c);
}

static void knn_predict_impl(int go_order, int32_t type, int32_t L, const double* sims, const int64_t* right_rowptr,
                             const int32_t* right_ids, const double* right_r, const double* means,
                             const double* stddevs, const double* bias, double global_mean, int32_t k,
                             int32_t min_k, int64_t n, const int32_t* left, const int32_t* right,
                             double* out) {
    int64_t maxdeg = 1;
    for (int64_t x = 0; x < n; x++) {
        if (right[x] < 0) continue;
        const int64_t d = right_rowptr[right[x] + 1] - right_rowptr[right[x]];
        if (d > maxdeg) maxdeg = d;
    }
    cand* c = (cand*)malloc((size_t)maxdeg * sizeof(cand));
    for (int64_t x = 0; x < n; x++) {
        const int32_t li = left[x], ri = right[x];
        if (li < 0 || ri < 0) {                             /* knn.go:89-91 */
            out[x] = global_mean;
            continue;
        }
        const double* srow = sims + (int64_t)li * L;
        int64_t nc = 0;
        for (int64_t t = right_rowptr[ri]; t < right_rowptr[ri + 1]; t++) { /* knn.go:95-99 */
            if (!isnan(srow[right_ids[t]])) {
                c[nc].id = right_ids[t];
                c[nc].r = right_r[t];
                c[nc].pos = nc;
                nc++;
            }
        }
        if (nc <= min_k) {                                  /* knn.go:102-104 */
            out[x] = global_mean;
            continue;
        }
        if (go_order) {
            go_sort_candidates(c, nc, srow);                /* knn.go:107-108: sort.Sort */
        } else {
            g_sim_row = srow;
            qsort(c, (size_t)nc, sizeof(cand), cmp_cand);   /* stable tie rule (position) */
        }
        const int64_t nn = nc < k ? nc : k;                 /* knn.go:111-114 */
        double weightSum = 0.0, weightRating = 0.0;
        for (int64_t t = 0; t < nn; t++) {                  /* knn.go:118-130 */
            weightSum += srow[c[t].id];
            double rating = c[t].r;
            if (type == 1) rating -= means[c[t].id];
            else if (type == 2) rating = (rating - means[c[t].id]) / stddevs[c[t].id];
            else if (type == 3) rating -= bias[c[t].id];
            weightRating += srow[c[t].id] * rating;
        }
        double prediction = weightRating / weightSum;       /* knn.go:131-139 */
        if (type == 1) prediction += means[li];
        else if (type == 3) prediction += bias[li];
        else if (type == 2) {
            prediction *= stddevs[li];
            prediction += means[li];
        }
        out[x] = prediction;
    }
    free(c);
}

/* KNN.Predict (knn.go:75-141) with the reference's tie order (Go sort.Sort, restated above) */
void or_knn_predict(int32_t type, int32_t L, const double* sims, const int64_t* right_rowptr,
                    const int32_t* right_ids, const double* right_r, const double* means,
                    const double* stddevs, const double* bias, double global_mean, int32_t k,
                    int32_t min_k, int64_t n, const int32_t* left, const int32_t* right,
                    double* out) {
    knn_predict_impl(1, type, L, sims, right_rowptr, right_ids, right_r, means, stddevs, bias, global_mean, k,
                     min_k, n, left, right, out);
}

/* The same with ties kept in candidate (RightRatings) order: the library's RS_TIE_STABLE option */
void or_knn_predict_stable(int32_t type, int32_t L, const double* sims, const int64_t* right_rowptr,
                           const int32_t* right_ids, const double* right_r, const double* means,
                           const double* stddevs, const double* bias, double global_mean, int32_t k,
                           int32_t min_k, int64_t n, const int32_t* left, const int32_t* right,
                           double* out) {
    knn_predict_impl(0, type, L, sims, right_rowptr, right_ids, right_r, means, stddevs, bias, global_mean, k,
                     min_k, n, left, right, out);
}

void or_baseline_fit(int64_t n, const int32_t* u, const int32_t* i, const double* r,
                     int32_t epochs, double lr, double reg, double* bu, double* bi, double* gb) {
    double GB = *gb;
    for (int32_t epoch = 0; epoch < epochs; epoch++) {      /* base.go:145 */
        for (int64_t t = 0; t < n; t++) {
            const int32_t uu = u[t], ii = i[t];
            const double userBias = bu[uu], itemBias = bi[ii];
            double pred = GB;                               /* base.go:122-133 */
            pred += bu[uu];
            pred += bi[ii];
            const double diff = pred - r[t];
            GB -= lr * diff;                                /* base.go:158-160 */
            bu[uu] -= lr * (diff + reg * userBias);
            bi[ii] -= lr * (diff + reg * itemBias);
        }
    }
    *gb = GB;
}

/* ------------------------------------------------------------------------------------------ */
/* Restatement of the GPU fast-mode schedule (sgd.hip), see oracle.h                           */

void or_svd_fit_chunked(int32_t n_users, const int64_t* rowptr, const int32_t* items,
                        const double* r, int32_t chunk, int32_t k, int32_t epochs, double lr,
                        double reg, double* P, double* Q, double* bu, double* bi, double* gb) {
    /* work items: each user row split into ceil(deg / chunk) near-equal pieces */
    int64_t nw = 0;
    for (int32_t x = 0; x < n_users; x++) {
        const int64_t d = rowptr[x + 1] - rowptr[x];
        nw += d > 0 ? (d + chunk - 1) / chunk : 0;
    }
    int32_t* wu = (int32_t*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(int32_t));
    int64_t* wb = (int64_t*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(int64_t));
    int64_t* we = (int64_t*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(int64_t));
    int32_t* wsplit = (int32_t*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(int32_t));
    int64_t w = 0, maxlen = 0;
    for (int32_t x = 0; x < n_users; x++) {
        const int64_t d = rowptr[x + 1] - rowptr[x];
        if (d == 0) continue;
        const int64_t pieces = (d + chunk - 1) / chunk;
        for (int64_t p = 0; p < pieces; p++) {
            wu[w] = x;
            wb[w] = rowptr[x] + d * p / pieces;
            we[w] = rowptr[x] + d * (p + 1) / pieces;
            wsplit[w] = pieces > 1;
            if (we[w] - wb[w] > maxlen) maxlen = we[w] - wb[w];
            w++;
        }
    }
    double* lp = (double*)malloc((size_t)(nw > 0 ? nw : 1) * k * sizeof(double));
    double* lp0 = (double*)malloc((size_t)(nw > 0 ? nw : 1) * k * sizeof(double));
    double* lbu = (double*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(double));
    double* lbu0 = (double*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(double));
    double* lgb = (double*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(double));
    int64_t nnz = rowptr[n_users];
    double GB = *gb;
    for (int32_t epoch = 0; epoch < epochs; epoch++) {
        for (int64_t x = 0; x < nw; x++) {
            memcpy(lp + x * k, P + (int64_t)wu[x] * k, (size_t)k * sizeof(double));
            memcpy(lp0 + x * k, P + (int64_t)wu[x] * k, (size_t)k * sizeof(double));
            lbu[x] = lbu0[x] = bu[wu[x]];
            lgb[x] = GB;
        }
        for (int64_t t = 0; t < maxlen; t++) {
            for (int64_t x = 0; x < nw; x++) {
                const int64_t pos = wb[x] + t;
                if (pos >= we[x]) continue;
                const int32_t ii = items[pos];
                double* pu = lp + x * k;
                double* qi = Q + (int64_t)ii * k;
                const double ub = lbu[x], ib = bi[ii];
                double pred = lgb[x];
                pred += ub;
                pred += ib;
                pred += dot(pu, qi, k);
                const double diff = pred - r[pos];
                lgb[x] -= lr * diff;
                lbu[x] = ub - lr * (diff + reg * ub);
                bi[ii] = ib - lr * (diff + reg * ib);
                for (int32_t f = 0; f < k; f++) pu[f] = pu[f] - (qi[f] * diff + pu[f] * reg) * lr;
                for (int32_t f = 0; f < k; f++) qi[f] = qi[f] - (pu[f] * diff + qi[f] * reg) * lr;
            }
        }
        double gsum = 0.0;
        for (int64_t x = 0; x < nw; x++) {
            const int32_t uu = wu[x];
            if (!wsplit[x]) {
                memcpy(P + (int64_t)uu * k, lp + x * k, (size_t)k * sizeof(double));
                bu[uu] = lbu[x];
            } else {  /* split user: count-weighted average of the pieces' end states */
                const double wgt = (double)(we[x] - wb[x]) / (double)(rowptr[uu + 1] - rowptr[uu]);
                for (int32_t f = 0; f < k; f++)
                    P[(int64_t)uu * k + f] += wgt * (lp[x * k + f] - lp0[x * k + f]);
                bu[uu] += wgt * (lbu[x] - lbu0[x]);
            }
            gsum += (double)(we[x] - wb[x]) * (lgb[x] - GB);
        }
        if (nnz > 0) GB += gsum / (double)nnz;
    }
    *gb = GB;
    free(wu);
    free(wb);
    free(we);
    free(wsplit);
    free(lp);
    free(lp0);
    free(lbu);
    free(lbu0);
    free(lgb);
}

void or_svdpp_fit_userwise(int32_t n_users, const int64_t* rowptr, const int32_t* items,
                           const double* r, int32_t k, int32_t epochs, double lr, double reg,
                           double* P, double* Q, double* Y, double* bu, double* bi, double* gb) {
    const int64_t nnz = rowptr[n_users];
    int32_t* uu = (int32_t*)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int32_t));
    for (int32_t x = 0; x < n_users; x++)
        for (int64_t t = rowptr[x]; t < rowptr[x + 1]; t++) uu[t] = x;
    double GB = *gb;
    for (int32_t epoch = 0; epoch < epochs; epoch++) {
        double gsum = 0.0;
        for (int32_t x = 0; x < n_users; x++) {
            const int64_t b = rowptr[x], e = rowptr[x + 1];
            if (e == b) continue;
            /* the user's row as its own train set: N(x) = the row, in row order */
            double g = GB;
            or_svdpp_fit(e - b, uu + b, items + b, r + b, x + 1, k, 1, lr, reg, P, Q, Y, bu, bi, &g);
            gsum += (double)(e - b) * (g - GB);
        }
        if (nnz > 0) GB += gsum / (double)nnz;
    }
    *gb = GB;
    free(uu);
}

/* The same schedule as or_svdpp_fit_userwise in O(nnz k) per epoch: inside a user's row every y-step
 * of svd.go:408-418 is one affine map for all j in N(u), y_j <- a y_j - b_t q_i (a = 1 - lr reg,
 * b_t = lr diff_t / sqrt|N(u)|), so y_j = A y_j0 - C with A = a^t and C = a C + b_t q_i, the implicit
 * sum of svd.go:271-282 is (A S0 - n C) / sqrt n with S0 = sum y_j0, and the rows are written once at
 * the user's end (equal to the literal form up to rounding for rows without repeated
 * items).  Used as the checker at BASELINE configs[2] scale, where the literal form is O(sum |N|^2 k). */
void or_svdpp_fit_lazy(int32_t n_users, const int64_t* rowptr, const int32_t* items, const double* r,
                       int32_t k, int32_t epochs, double lr, double reg, double* P, double* Q, double* Y,
                       double* bu, double* bi, double* gb) {
    const int64_t nnz = rowptr[n_users];
    double* S0 = (double*)malloc((size_t)k * sizeof(double));
    double* Cv = (double*)malloc((size_t)k * sizeof(double));
    double* e = (double*)malloc((size_t)k * sizeof(double));
    const double al = 1.0 - lr * reg;
    double GB = *gb;
    for (int32_t epoch = 0; epoch < epochs; epoch++) {
        double gsum = 0.0;
        for (int32_t x = 0; x < n_users; x++) {
            const int64_t b = rowptr[x], en = rowptr[x + 1];
            if (en == b) continue;
            const double n = (double)(en - b), sq = sqrt(n);
            for (int32_t f = 0; f < k; f++) {
                S0[f] = 0.0;
                Cv[f] = 0.0;
            }
            for (int64_t t = b; t < en; t++)
                for (int32_t f = 0; f < k; f++) S0[f] += Y[(int64_t)items[t] * k + f];
            double A = 1.0, g = GB;
            double* pu = P + (int64_t)x * k;
            for (int64_t t = b; t < en; t++) {
                const int32_t ii = items[t];
                double* qi = Q + (int64_t)ii * k;
                const double userBias = bu[x], itemBias = bi[ii];
                double pred = g;
                pred += bu[x];
                pred += bi[ii];
                double s = 0.0;
                for (int32_t f = 0; f < k; f++) {
                    e[f] = (A * S0[f] - n * Cv[f]) / sq;
                    s += (pu[f] + e[f]) * qi[f];
                }
                pred += s;
                const double diff = pred - r[t];
                g -= lr * diff;
                bu[x] -= lr * (diff + reg * userBias);
                bi[ii] -= lr * (diff + reg * itemBias);
                for (int32_t f = 0; f < k; f++) pu[f] = pu[f] - (qi[f] * diff + pu[f] * reg) * lr;
                for (int32_t f = 0; f < k; f++) qi[f] = qi[f] - ((pu[f] + e[f]) * diff + qi[f] * reg) * lr;
                const double bt = lr * diff / sq;
                for (int32_t f = 0; f < k; f++) Cv[f] = al * Cv[f] + bt * qi[f];
                A *= al;
            }
            for (int64_t t = b; t < en; t++) {
                double* y = Y + (int64_t)items[t] * k;
                for (int32_t f = 0; f < k; f++) y[f] = A * y[f] - Cv[f];
            }
            gsum += n * (g - GB);
        }
        if (nnz > 0) GB += gsum / (double)nnz;
    }
    *gb = GB;
    free(S0);
    free(Cv);
    free(e);
}

double or_gb_warm_start(int32_t n_users, const int64_t* rowptr, const int32_t* items,
                        const double* r, const double* bu, const double* bi) {
    const int64_t nnz = rowptr[n_users];
    if (nnz <= 0) return 0.0;
    double s = 0.0;
    for (int32_t x = 0; x < n_users; x++)
        for (int64_t t = rowptr[x]; t < rowptr[x + 1]; t++) s += r[t] - bu[x] - bi[items[t]];
    return s / (double)nnz;
}

/* ------------------------------------------------------------------------------------------ */
/* SlopeOne                                                                                    */

void or_slope_one_fit(int32_t L, const int64_t* rowptr, const int32_t* ids, const double* ratings,
                      double* dev) {
    const int64_t nnz = rowptr[L];
    int32_t* sid = (int32_t*)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int32_t));
    double* sr = (double*)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(double));
    idr* tmp = (idr*)malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(idr));
    /* slope_one.go:62 sorts(itemRatings) (data.go:236-243): each item's list by user ID */
    for (int32_t x = 0; x < L; x++) {
        const int64_t b = rowptr[x], e = rowptr[x + 1];
        for (int64_t t = b; t < e; t++) {
            tmp[t - b].id = ids[t];
            tmp[t - b].r = ratings[t];
        }
        qsort(tmp, (size_t)(e - b), sizeof(idr), cmp_idr);
        for (int64_t t = b; t < e; t++) {
            sid[t] = tmp[t - b].id;
            sr[t] = tmp[t - b].r;
        }
    }
    free(tmp);
    const int64_t LL = (int64_t)L * L;
    for (int64_t t = 0; t < LL; t++) dev[t] = 0.0;           /* slope_one.go:59 newZeroMatrix */
    for (int32_t i = 0; i < L; i++) {                        /* slope_one.go:75 (nJobs = 1) */
        const int64_t bi = rowptr[i], ni = rowptr[i + 1] - bi;
        for (int32_t j = 0; j < i; j++) {                    /* slope_one.go:76 */
            const int64_t bj = rowptr[j], nj = rowptr[j + 1] - bj;
            double count = 0.0, sum = 0.0;
            int64_t ptr = 0;
            for (int64_t k = 0; k < ni && ptr < nj; k++) {   /* slope_one.go:78-87 */
                const int32_t uid = sid[bi + k];
                while (ptr < nj && sid[bj + ptr] < uid) ptr++;
                if (ptr < nj && sid[bj + ptr] == uid) {
                    count++;
                    sum += sr[bi + k] - sr[bj + ptr];
                }
            }
            if (count > 0) {                                 /* slope_one.go:88-91 */
                dev[(int64_t)i * L + j] = sum / count;
                dev[(int64_t)j * L + i] = -dev[(int64_t)i * L + j];
            }
        }
    }
    free(sid);
    free(sr);
}

void or_slope_one_predict(int32_t L, const double* dev, int32_t n_users, const int64_t* user_rowptr,
                          const int32_t* user_items, const double* user_ratings, double global_mean,
                          int64_t n, const int32_t* users, const int32_t* items, double* out) {
    for (int64_t q = 0; q < n; q++) {
        const int32_t u = users[q], i = items[q];
        const int ku = u >= 0 && u < n_users, ki = i >= 0 && i < L;
        double prediction = 0.0;
        if (ku) {                                            /* slope_one.go:26-30 */
            double sum = 0.0, count = 0.0;                   /* means(), data.go:222-235 */
            for (int64_t t = user_rowptr[u]; t < user_rowptr[u + 1]; t++) {
                sum += user_ratings[t];
                count++;
            }
            prediction = sum / count;
        } else {
            prediction = global_mean;
        }
        if (ki && ku) {                                      /* slope_one.go:32-42 */
            double sum = 0.0, count = 0.0;
            for (int64_t t = user_rowptr[u]; t < user_rowptr[u + 1]; t++) {
                sum += dev[(int64_t)i * L + user_items[t]];
                count++;
            }
            if (count > 0) prediction += sum / count;
        }
        out[q] = prediction;
    }
}
