// ingest.cpp -- host-side TrainSet construction for the GPU path, C++ threads.
//
// The reference builds its TrainSet with Go maps (core/data.go:131-154: inner ids in first-appearance
// order, users then items) and per-user adjacency lists in data order (data.go:185-216).  At the
// 1e9-rating shape of BASELINE configs[4] that map work dominates the host, so the
// drop-in path does it here, in parallel, with results identical to the sequential definition:
//
//   rs_trainset_ids    inner ids by first appearance (== data.go:137-151 for any thread count)
//   rs_csr_build       stable counting sort of COO rows -> CSR (== data.go:185-199 row order)
//   rs_global_mean     stat.Mean of the ratings (data.go:134), fixed-order chunked sum
//
// None of these touch the GPU; they run on the caller's thread plus n_threads - 1 pooled threads.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <cmath>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"

namespace rs {

int32_t clamp_threads(int32_t n_threads) {
    if (n_threads > 0) return std::min(n_threads, 256);
    const unsigned hw = std::thread::hardware_concurrency();
    return static_cast<int32_t>(std::max(1u, std::min(hw, 16u)));
}

namespace {

// Persistent workers for parallel_run: creating threads costs tens of microseconds each on the GPU boxes'
// hosts, which made a 16-thread, four-pass CSR build slower than one thread (3.0 ms against 2.0 ms for
// 1M ratings).  Workers are created on first use, then sleep on a condition variable between jobs.  One
// job at a time: a caller that finds the pool busy (another host thread, e.g. a shard of a multi-GPU fit)
// spawns its own threads as before.  A nested call -- from inside a pool job, on a worker or on the
// caller's own t = 0 -- never touches the pool's mutex (try_lock on a mutex the thread already holds is
// undefined behaviour): the thread-local flag sends it to the spawned-threads path.
thread_local bool in_pool_job = false;

class WorkerPool {
  public:
    bool try_run(int32_t n, const std::function<void(int32_t)>& fn, std::vector<std::exception_ptr>& err) {
        if (in_pool_job) return false;
        std::unique_lock<std::mutex> busy(busy_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> g(m_);
            while (static_cast<int32_t>(workers_.size()) < n - 1) {
                const int32_t id = static_cast<int32_t>(workers_.size()) + 1;
                workers_.emplace_back([this, id] { loop(id); });
            }
            job_ = &fn;
            err_ = &err;
            n_ = n;
            left_ = n - 1;
            ++gen_;
        }
        cv_.notify_all();
        in_pool_job = true;
        try {
            fn(0);
        } catch (...) {
            err[0] = std::current_exception();
        }
        in_pool_job = false;
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return left_ == 0; });
        job_ = nullptr;
        return true;
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : workers_) t.join();
    }

  private:
    void loop(int32_t id) {
        in_pool_job = true;  // a worker only ever runs pool jobs
        uint64_t seen = 0;
        std::unique_lock<std::mutex> l(m_);
        for (;;) {
            cv_.wait(l, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            if (id >= n_) continue;
            const std::function<void(int32_t)>* fn = job_;
            std::vector<std::exception_ptr>* err = err_;
            l.unlock();
            try {
                (*fn)(id);
            } catch (...) {
                (*err)[id] = std::current_exception();
            }
            l.lock();
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::mutex busy_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int32_t)>* job_ = nullptr;
    std::vector<std::exception_ptr>* err_ = nullptr;
    int32_t n_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

WorkerPool& pool() {
    static WorkerPool p;
    return p;
}

}  // namespace

// Runs fn(t) for t in [0, n) on n threads (the caller runs t = 0); rethrows the first exception.
void parallel_run(int32_t n, const std::function<void(int32_t)>& fn) {
    if (n <= 1) {
        fn(0);
        return;
    }
    std::vector<std::exception_ptr> err(n);
    if (!pool().try_run(n, fn, err)) {
        std::vector<std::thread> th;
        th.reserve(n - 1);
        for (int32_t t = 1; t < n; ++t)
            th.emplace_back([&, t]() {
                try {
                    fn(t);
                } catch (...) {
                    err[t] = std::current_exception();
                }
            });
        try {
            fn(0);
        } catch (...) {
            err[0] = std::current_exception();
        }
        for (auto& x : th) x.join();
    }
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

namespace {

uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

// Open-addressing int64 -> int64 map owned by one thread (no locking).
struct IdMap {
    std::vector<int64_t> keys, vals;
    std::vector<uint8_t> used;
    uint64_t mask = 0;
    int64_t size = 0;
    void init(int64_t expect) {
        uint64_t cap = 64;
        while (cap < static_cast<uint64_t>(2 * expect + 64)) cap <<= 1;
        keys.assign(cap, 0);
        vals.assign(cap, 0);
        used.assign(cap, 0);
        mask = cap - 1;
        size = 0;
    }
    void grow() {
        IdMap n;
        n.init(static_cast<int64_t>(keys.size()));  // doubles the capacity
        for (size_t s = 0; s < keys.size(); ++s)
            if (used[s]) *n.slot_put(keys[s], vals[s]) = vals[s];
        *this = std::move(n);
    }
    // value slot of key, inserting val if absent
    int64_t* slot_put(int64_t key, int64_t val) {
        uint64_t h = mix64(static_cast<uint64_t>(key)) & mask;
        while (used[h]) {
            if (keys[h] == key) return &vals[h];
            h = (h + 1) & mask;
        }
        used[h] = 1;
        keys[h] = key;
        vals[h] = val;
        ++size;
        return &vals[h];
    }
    int64_t get(int64_t key) const {
        uint64_t h = mix64(static_cast<uint64_t>(key)) & mask;
        while (used[h]) {
            if (keys[h] == key) return vals[h];
            h = (h + 1) & mask;
        }
        return -1;
    }
};

// Key k belongs to thread (mix64(k ^ c) >> 40) % n (independent of the map hash
// bits used for probing, which are the low ones).
inline int32_t owner_of(int64_t key, int32_t n) {
    return static_cast<int32_t>((mix64(static_cast<uint64_t>(key) ^ 0x9e3779b97f4a7c15ULL) >> 40) % n);
}

}  // namespace

// Inner ids of a column of outer ids, in first-appearance order (data.go:137-151).
// Each thread owns the keys hashing to it and scans the whole column in order, so its map records the
// first position of each owned key; first positions are flagged, a prefix count over the flags gives
// the ids (id = number of distinct keys whose first position comes earlier), and a second owner scan
// writes every position's id.  Result is independent of n_threads.
void trainset_ids(int64_t n, const int64_t* outer, int32_t n_threads, int32_t* inner,
                  int64_t* outer_of_inner, int32_t* n_unique) {
    const int32_t T = clamp_threads(n_threads);
    std::vector<IdMap> maps(T);
    std::vector<uint8_t> first(static_cast<size_t>(std::max<int64_t>(n, 1)), 0);
    std::vector<uint8_t> owner(static_cast<size_t>(std::max<int64_t>(n, 1)), 0);
    parallel_run(T, [&](int32_t t) {  // owner of every position, hashed once
        for (int64_t p = n * t / T, e = n * (t + 1) / T; p < e; ++p)
            owner[p] = static_cast<uint8_t>(owner_of(outer[p], T));
    });
    parallel_run(T, [&](int32_t t) {
        IdMap& m = maps[t];
        m.init(std::min<int64_t>(n / T + 64, int64_t{1} << 22));
        for (int64_t p = 0; p < n; ++p) {
            if (owner[p] != t) continue;
            const int64_t k = outer[p];
            if (2 * (m.size + 1) > static_cast<int64_t>(m.keys.size())) m.grow();
            int64_t* v = m.slot_put(k, p);
            if (*v == p) first[p] = 1;
        }
    });
    // prefix count over the flags in T contiguous ranges
    std::vector<int64_t> base(T + 1, 0);
    parallel_run(T, [&](int32_t t) {
        const int64_t lo = n * t / T, hi = n * (t + 1) / T;
        int64_t c = 0;
        for (int64_t p = lo; p < hi; ++p) c += first[p];
        base[t + 1] = c;
    });
    for (int32_t t = 0; t < T; ++t) base[t + 1] += base[t];
    if (base[T] > INT32_MAX) throw std::invalid_argument("more than 2^31 - 1 distinct ids");
    *n_unique = static_cast<int32_t>(base[T]);
    parallel_run(T, [&](int32_t t) {  // id at every first position
        const int64_t lo = n * t / T, hi = n * (t + 1) / T;
        int64_t id = base[t];
        for (int64_t p = lo; p < hi; ++p)
            if (first[p]) {
                inner[p] = static_cast<int32_t>(id);
                if (outer_of_inner) outer_of_inner[id] = outer[p];
                ++id;
            }
    });
    parallel_run(T, [&](int32_t t) {  // map values: first position -> id; then every position
        IdMap& m = maps[t];
        for (size_t s = 0; s < m.keys.size(); ++s)
            if (m.used[s]) m.vals[s] = inner[m.vals[s]];
        for (int64_t p = 0; p < n; ++p)
            if (owner[p] == t && !first[p]) inner[p] = static_cast<int32_t>(m.get(outer[p]));
    });
}

// Stable CSR of COO rows (data order inside a row, data.go:185-199): per-thread histograms over T
// contiguous chunks, exclusive offsets per (row, thread), ordered scatter.
void csr_build(int64_t nnz, int32_t n_rows, const int32_t* rows, const int32_t* cols,
               const double* vals, int32_t n_threads, int64_t* rowptr, int32_t* cols_out,
               float* vals_out) {
    int32_t T = clamp_threads(n_threads);
    // per-thread histograms cost T * n_rows words: fall back to fewer threads for tiny inputs
    while (T > 1 && nnz < static_cast<int64_t>(T) * 4096) T /= 2;
    std::vector<std::vector<int64_t>> cnt(T);
    parallel_run(T, [&](int32_t t) {
        std::vector<int64_t>& c = cnt[t];
        c.assign(static_cast<size_t>(n_rows), 0);
        const int64_t lo = nnz * t / T, hi = nnz * (t + 1) / T;
        for (int64_t p = lo; p < hi; ++p) {
            const int32_t r = rows[p];
            if (r < 0 || r >= n_rows) throw std::invalid_argument("row id out of range at " + std::to_string(p));
            c[r]++;
        }
    });
    // rowptr and per-thread start offsets (cnt[t][r] becomes thread t's next slot in row r)
    std::vector<int64_t> part(T + 1, 0);
    parallel_run(T, [&](int32_t t) {
        const int64_t lo = static_cast<int64_t>(n_rows) * t / T, hi = static_cast<int64_t>(n_rows) * (t + 1) / T;
        int64_t s = 0;
        for (int64_t r = lo; r < hi; ++r)
            for (int32_t x = 0; x < T; ++x) s += cnt[x][r];
        part[t + 1] = s;
    });
    for (int32_t t = 0; t < T; ++t) part[t + 1] += part[t];
    parallel_run(T, [&](int32_t t) {
        const int64_t lo = static_cast<int64_t>(n_rows) * t / T, hi = static_cast<int64_t>(n_rows) * (t + 1) / T;
        int64_t off = part[t];
        for (int64_t r = lo; r < hi; ++r) {
            rowptr[r] = off;
            for (int32_t x = 0; x < T; ++x) {
                const int64_t c = cnt[x][r];
                cnt[x][r] = off;
                off += c;
            }
        }
    });
    rowptr[n_rows] = nnz;
    parallel_run(T, [&](int32_t t) {
        std::vector<int64_t>& c = cnt[t];
        const int64_t lo = nnz * t / T, hi = nnz * (t + 1) / T;
        for (int64_t p = lo; p < hi; ++p) {
            const int64_t d = c[rows[p]]++;
            cols_out[d] = cols[p];
            if (vals_out) vals_out[d] = static_cast<float>(vals[p]);
        }
    });
}

// gonum stat.Mean(x, nil) = sum / n (data.go:134).  Summed in fixed 2^20-element chunks combined in
// order, so the value does not depend on n_threads (it can differ from a single running sum by a few
// ulp; the reference's own floats.Sum order is gonum's asm kernel, unpinned here).
double global_mean(int64_t n, const double* r, int32_t n_threads) {
    if (n <= 0) return std::nan("");
    constexpr int64_t kChunk = int64_t{1} << 20;
    const int64_t nc = (n + kChunk - 1) / kChunk;
    std::vector<double> part(nc, 0.0);
    const int32_t T = clamp_threads(n_threads);
    std::atomic<int64_t> next{0};
    parallel_run(T, [&](int32_t) {
        for (int64_t c; (c = next.fetch_add(1)) < nc;) {
            double s = 0.0;
            for (int64_t p = c * kChunk, e = std::min(n, (c + 1) * kChunk); p < e; ++p) s += r[p];
            part[c] = s;
        }
    });
    double s = 0.0;
    for (double x : part) s += x;
    return s / static_cast<double>(n);
}

}  // namespace rs

extern "C" int rs_trainset_ids(int64_t n, const int64_t* outer, int32_t n_threads, int32_t* inner,
                               int64_t* outer_of_inner, int32_t* n_unique) {
    return rs_guard(nullptr, [&]() -> int {
        if (n < 0 || !n_unique || (n > 0 && (!outer || !inner)))
            return rs::set_error(nullptr, RS_ERR_INVALID, "rs_trainset_ids: bad arguments");
        rs::trainset_ids(n, outer, n_threads, inner, outer_of_inner, n_unique);
        return RS_OK;
    });
}

extern "C" int rs_csr_build(int64_t nnz, int32_t n_rows, const int32_t* rows, const int32_t* cols,
                            const double* vals, int32_t n_threads, int64_t* rowptr, int32_t* cols_out,
                            float* vals_out) {
    return rs_guard(nullptr, [&]() -> int {
        if (nnz < 0 || n_rows < 0 || !rowptr || (nnz > 0 && (!rows || !cols || !cols_out)) ||
            (vals_out && nnz > 0 && !vals))
            return rs::set_error(nullptr, RS_ERR_INVALID, "rs_csr_build: bad arguments");
        rs::csr_build(nnz, n_rows, rows, cols, vals, n_threads, rowptr, cols_out, vals_out);
        return RS_OK;
    });
}

extern "C" int rs_global_mean(int64_t n, const double* ratings, int32_t n_threads, double* mean) {
    return rs_guard(nullptr, [&]() -> int {
        if (n < 0 || !mean || (n > 0 && !ratings))
            return rs::set_error(nullptr, RS_ERR_INVALID, "rs_global_mean: bad arguments");
        *mean = rs::global_mean(n, ratings, n_threads);
        return RS_OK;
    });
}
