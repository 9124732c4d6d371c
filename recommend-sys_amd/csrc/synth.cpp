// synth.cpp -- deterministic synthetic rating sets straight into inner-id user-CSR (BASELINE
// configs[4]: 10M users x 1M items x ~1B ratings; SURVEY §8d "generated directly in inner-ID CSR by
// the C++ generator, bypassing Go maps").  Benchmark-data plumbing, not a reference function: the
// reference downloads MovieLens files (core/data.go:270-284), which this environment cannot.
//
// Shape:
//   user degree  lognormal(mu, sigma) with mean mean_deg, clamped to [min_deg, max_deg]
//   items        Zipf(s) popularity over a seeded permutation of the item ids ("hashed ids": an item
//                range shard gets a balanced share), no duplicate (u, i) within a user
//   ratings      integers 1..5 from a planted model: 3.6 + b_u + b_i + x_u . y_i (rank 4) + noise
// Every value is a pure function of (seed, user, draw) through counter-based hashing, so the set is
// independent of the thread count, and a shard [item_lo, item_hi) is exactly the full set's ratings
// of those items, in the same order (each rank of an item-sharded run generates its own shard).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <vector>

#include "common.hpp"

namespace rs {
int32_t clamp_threads(int32_t n_threads);
void parallel_run(int32_t n, const std::function<void(int32_t)>& fn);
}  // namespace rs

struct rs_synth {
    int32_t n_users = 0, n_items = 0;
    int64_t nnz = 0;
    std::vector<int64_t> rowptr;
    std::vector<int32_t> cols;
    std::vector<float> vals;
};

namespace rs {
namespace {

inline uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
inline uint64_t hash3(uint64_t a, uint64_t b, uint64_t c) {
    return splitmix(splitmix(splitmix(a) ^ b) ^ c);
}
inline double unit(uint64_t h) { return (static_cast<double>(h >> 11) + 0.5) * (1.0 / 9007199254740992.0); }
inline double normal(uint64_t h) {  // Box-Muller on two halves of one stream
    const double u1 = unit(h), u2 = unit(splitmix(h));
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

}  // namespace

static void synth_build(const int32_t n_users, const int32_t n_items, double mean_deg, double sigma,
                        int32_t min_deg, int32_t max_deg, double zipf_s, uint64_t seed, int32_t item_lo,
                        int32_t item_hi, int32_t user_lo, int32_t user_hi, int32_t n_threads,
                        rs_synth* out) {
    const int32_t n_rows = user_hi - user_lo;  // rows of the output CSR: users [user_lo, user_hi)
    const int32_t T = clamp_threads(n_threads);
    // Zipf CDF over ranks and the rank -> item permutation (Fisher-Yates on the seed)
    std::vector<double> cdf(n_items);
    double acc = 0.0;
    for (int32_t r = 0; r < n_items; ++r) cdf[r] = (acc += std::pow(static_cast<double>(r + 1), -zipf_s));
    for (double& c : cdf) c /= acc;
    // guide table: ranks with cdf <= g / n_items lie below guide[g], so a draw searches one bucket
    std::vector<int32_t> guide(static_cast<size_t>(n_items) + 1);
    for (int32_t g = 0, r = 0; g <= n_items; ++g) {
        const double x = static_cast<double>(g) / n_items;
        while (r < n_items && cdf[r] <= x) ++r;
        guide[g] = r;
    }
    std::vector<int32_t> perm(n_items);
    for (int32_t x = 0; x < n_items; ++x) perm[x] = x;
    for (int32_t x = n_items - 1; x > 0; --x)
        std::swap(perm[x], perm[static_cast<int32_t>(hash3(seed, 7, x) % static_cast<uint64_t>(x + 1))]);
    // planted item terms: b_i and y_i (rank 4)
    constexpr int kRank = 4;
    std::vector<float> item_t(static_cast<size_t>(n_items) * (kRank + 1));
    for (int32_t x = 0; x < n_items; ++x) {
        float* t = item_t.data() + static_cast<size_t>(x) * (kRank + 1);
        t[0] = static_cast<float>(0.4 * normal(hash3(seed, 2, x)));
        for (int f = 0; f < kRank; ++f) t[1 + f] = static_cast<float>(0.6 * normal(hash3(seed, 3 + f, x)));
    }
    const double mu = std::log(mean_deg) - 0.5 * sigma * sigma;
    // thread t generates rows [n_rows t / T, n_rows (t + 1) / T) into its own buffers
    std::vector<std::vector<int32_t>> tc(T);
    std::vector<std::vector<float>> tv(T);
    out->rowptr.assign(static_cast<size_t>(n_rows) + 1, 0);
    parallel_run(T, [&](int32_t t) {
        const int32_t u0 = user_lo + static_cast<int32_t>(static_cast<int64_t>(n_rows) * t / T);
        const int32_t u1 = user_lo + static_cast<int32_t>(static_cast<int64_t>(n_rows) * (t + 1) / T);
        std::vector<int32_t> stamp(n_items, -1);  // user that last drew the item (dedup)
        std::vector<int32_t>& cols = tc[t];
        std::vector<float>& vals = tv[t];
        cols.reserve(static_cast<size_t>((u1 - u0) * mean_deg * (item_hi - item_lo) / std::max(1, n_items) * 1.1) + 64);
        vals.reserve(cols.capacity());
        for (int32_t u = u0; u < u1; ++u) {
            const uint64_t hu = hash3(seed, 1, u);
            double d = std::exp(mu + sigma * normal(hu));
            int32_t deg = static_cast<int32_t>(std::llround(d));
            deg = std::max(min_deg, std::min(deg, std::min(max_deg, n_items)));
            const float bu = static_cast<float>(0.4 * normal(hash3(seed, 10, u)));
            float xu[kRank];
            for (int f = 0; f < kRank; ++f) xu[f] = static_cast<float>(0.6 * normal(hash3(seed, 11 + f, u)));
            int32_t kept = 0;
            for (int32_t j = 0; j < deg; ++j) {
                int32_t item = -1;
                for (int32_t a = 0; a < 64 && item < 0; ++a) {  // Zipf draws, redrawn on a repeat
                    const double x = unit(hash3(hu, j, a));
                    const int32_t g = std::min(static_cast<int32_t>(x * n_items), n_items - 1);
                    const auto lo = cdf.begin() + guide[g], hi = cdf.begin() + std::min(n_items, guide[g + 1] + 1);
                    const int32_t r = static_cast<int32_t>(std::upper_bound(lo, hi, x) - cdf.begin());
                    const int32_t it = perm[std::min(r, n_items - 1)];
                    if (stamp[it] != u) item = it;
                }
                if (item < 0) {  // saturated head: the next unused id after a uniform start
                    int32_t it = static_cast<int32_t>(hash3(hu, j, 99) % static_cast<uint64_t>(n_items));
                    while (stamp[it] == u) it = it + 1 == n_items ? 0 : it + 1;
                    item = it;
                }
                stamp[item] = u;
                if (item < item_lo || item >= item_hi) continue;
                const float* ti = item_t.data() + static_cast<size_t>(item) * (kRank + 1);
                double s = 3.6 + bu + ti[0] + 0.5 * normal(hash3(hu, j, 1000));
                for (int f = 0; f < kRank; ++f) s += xu[f] * ti[1 + f];
                cols.push_back(item);
                vals.push_back(static_cast<float>(std::min(5.0, std::max(1.0, std::nearbyint(s)))));
                ++kept;
            }
            out->rowptr[static_cast<size_t>(u - user_lo) + 1] = kept;
        }
    });
    for (int32_t x = 0; x < n_rows; ++x) out->rowptr[x + 1] += out->rowptr[x];
    out->nnz = out->rowptr[n_rows];
    out->cols.resize(static_cast<size_t>(out->nnz));
    out->vals.resize(static_cast<size_t>(out->nnz));
    parallel_run(T, [&](int32_t t) {
        const int32_t x0 = static_cast<int32_t>(static_cast<int64_t>(n_rows) * t / T);
        const int64_t o = out->rowptr[x0];
        std::memcpy(out->cols.data() + o, tc[t].data(), tc[t].size() * sizeof(int32_t));
        std::memcpy(out->vals.data() + o, tv[t].data(), tv[t].size() * sizeof(float));
        std::vector<int32_t>().swap(tc[t]);
        std::vector<float>().swap(tv[t]);
    });
    out->n_users = n_rows;
    out->n_items = n_items;
}

}  // namespace rs

extern "C" int rs_synth_create(int32_t n_users, int32_t n_items, double mean_deg, double sigma,
                               int32_t min_deg, int32_t max_deg, double zipf_s, uint64_t seed,
                               int32_t item_lo, int32_t item_hi, int32_t user_lo, int32_t user_hi,
                               int32_t n_threads, rs_synth** out) {
    return rs_guard(nullptr, [&]() -> int {
        if (!out) return rs::set_error(nullptr, RS_ERR_INVALID, "out is NULL");
        *out = nullptr;
        if (n_users < 1 || n_items < 1 || !(mean_deg >= 1.0) || !(sigma >= 0.0) || min_deg < 1 ||
            max_deg < min_deg || !(zipf_s >= 0.0) || item_lo < 0 || item_hi > n_items || item_lo >= item_hi ||
            user_lo < 0 || user_hi > n_users || user_lo >= user_hi)
            return rs::set_error(nullptr, RS_ERR_INVALID, "rs_synth_create: bad arguments");
        auto* s = new rs_synth();
        try {
            rs::synth_build(n_users, n_items, mean_deg, sigma, min_deg, max_deg, zipf_s, seed, item_lo,
                            item_hi, user_lo, user_hi, n_threads, s);
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
        return RS_OK;
    });
}

extern "C" int rs_synth_csr(const rs_synth* s, int64_t* nnz, const int64_t** rowptr, const int32_t** cols,
                            const float** vals) {
    if (!s || !nnz || !rowptr || !cols || !vals) return rs::set_error(nullptr, RS_ERR_INVALID, "bad arguments");
    *nnz = s->nnz;
    *rowptr = s->rowptr.data();
    *cols = s->cols.data();
    *vals = s->vals.data();
    return RS_OK;
}

extern "C" void rs_synth_destroy(rs_synth* s) { delete s; }
