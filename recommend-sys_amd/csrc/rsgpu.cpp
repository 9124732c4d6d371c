// rsgpu.cpp -- context management and host-side helpers of the C-ABI (include/rsgpu.h).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"

namespace rs {

std::string& tls_error() {
    static thread_local std::string e;
    return e;
}

int set_error(rs_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    tls_error() = msg;
    return code;
}

void pack_rows_f32(const double* src, int64_t rows, int32_t k, int32_t ld, std::vector<float>& dst) {
    dst.assign(static_cast<size_t>(rows) * ld, 0.f);
    for (int64_t r = 0; r < rows; ++r)
        for (int32_t f = 0; f < k; ++f) dst[r * ld + f] = static_cast<float>(src[r * k + f]);
}

void unpack_rows_f64(const std::vector<float>& src, int64_t rows, int32_t k, int32_t ld, double* dst) {
    for (int64_t r = 0; r < rows; ++r)
        for (int32_t f = 0; f < k; ++f) dst[r * k + f] = static_cast<double>(src[r * ld + f]);
}

void build_csr(int64_t nnz, int32_t n_rows, const int32_t* rows, const int32_t* cols,
               const double* vals, UserCSR& out) {  // stable: data order within a row (ingest.cpp)
    out.rowptr.resize(static_cast<size_t>(n_rows) + 1);
    out.cols.resize(static_cast<size_t>(nnz));
    out.vals.resize(static_cast<size_t>(nnz));
    csr_build(nnz, n_rows, rows, cols, vals, 0, out.rowptr.data(), out.cols.data(), out.vals.data());
}

// The buffer is sized to the request rounded up to 1 MiB (callers cap requests at 256 MiB, sgd_tile.hip).
void* pinned_staging(rs_ctx* ctx, size_t bytes, int slot) {
    rs_ctx::Pinned& b = ctx->pinned[slot & 1];
    if (b.n < bytes) {
        if (b.p) (void)hipHostFree(b.p);
        b.p = nullptr;
        b.n = 0;
        const size_t n = (bytes + (size_t{1} << 20) - 1) & ~((size_t{1} << 20) - 1);
        RS_HIP(hipHostMalloc(&b.p, n, hipHostMallocPortable));
        b.n = n;
    }
    return b.p;
}

void* pinned_small(rs_ctx* ctx, int slot) {
    if (!ctx->pinned_small_p) RS_HIP(hipHostMalloc(&ctx->pinned_small_p, 256, hipHostMallocPortable));
    return static_cast<char*>(ctx->pinned_small_p) + 64 * slot;
}

void release_pinned(rs_ctx* ctx) {  // (after the ctx stream is synchronised: no copy is in flight)
    for (rs_ctx::Pinned& b : ctx->pinned) {
        if (b.p) (void)hipHostFree(b.p);
        b.p = nullptr;
        b.n = 0;
    }
    if (ctx->pinned_small_p) (void)hipHostFree(ctx->pinned_small_p);
    ctx->pinned_small_p = nullptr;
}

void fill_report(rs_report* rep, int status, int32_t refits) {
    if (!rep) return;
    rep->refits = refits;
    const std::string& e = status == RS_OK ? std::string() : tls_error();
    const size_t n = std::min(e.size(), sizeof(rep->error) - 1);
    std::memcpy(rep->error, e.data(), n);
    rep->error[n] = '\0';
}

// mean(r - b_u - b_i) over fixed 2^16-rating chunks summed in order (independent of the thread count)
double gb_warm_start(const rs_ratings* r, const double* bu, const double* bi) {
    if (r->nnz <= 0) return 0.0;
    constexpr int64_t kChunk = int64_t{1} << 16;
    const int64_t nc = (r->nnz + kChunk - 1) / kChunk;
    std::vector<double> part(static_cast<size_t>(nc), 0.0);
    const int32_t T = static_cast<int32_t>(std::min<int64_t>(clamp_threads(0), nc));
    parallel_run(T, [&](int32_t th) {
        for (int64_t c = th; c < nc; c += T) {
            double s = 0.0;
            for (int64_t t = c * kChunk, e = std::min(r->nnz, (c + 1) * kChunk); t < e; ++t)
                s += r->ratings[t] - bu[r->users[t]] - bi[r->items[t]];
            part[c] = s;
        }
    });
    double s = 0.0;
    for (double x : part) s += x;
    return s / static_cast<double>(r->nnz);
}

int check_ratings(rs_ctx* ctx, const rs_ratings* r) {
    if (!r) return set_error(ctx, RS_ERR_INVALID, "ratings is NULL");
    if (r->nnz < 0 || r->n_users < 0 || r->n_items < 0)
        return set_error(ctx, RS_ERR_INVALID, "negative size");
    if (r->nnz > 0 && (!r->users || !r->items || !r->ratings))
        return set_error(ctx, RS_ERR_INVALID, "ratings arrays are NULL");
    // the first offending position (the same message whatever the thread count)
    const int32_t T = static_cast<int32_t>(std::max<int64_t>(1, std::min<int64_t>(clamp_threads(0), r->nnz >> 16)));
    std::vector<int64_t> bad(static_cast<size_t>(T), -1);
    parallel_run(T, [&](int32_t th) {
        for (int64_t t = r->nnz * th / T, e = r->nnz * (th + 1) / T; t < e; ++t)
            if (static_cast<uint32_t>(r->users[t]) >= static_cast<uint32_t>(r->n_users) ||
                static_cast<uint32_t>(r->items[t]) >= static_cast<uint32_t>(r->n_items)) {
                bad[th] = t;
                return;
            }
    });
    for (int64_t t : bad) {
        if (t < 0) continue;
        if (r->users[t] < 0 || r->users[t] >= r->n_users)
            return set_error(ctx, RS_ERR_INVALID, "user id out of range at " + std::to_string(t));
        return set_error(ctx, RS_ERR_INVALID, "item id out of range at " + std::to_string(t));
    }
    return RS_OK;
}

}  // namespace rs

extern "C" int32_t rs_version(void) { return 1; }

extern "C" int rs_device_count(int32_t* n) {
    return rs_guard(nullptr, [&]() -> int {
        if (!n) return rs::set_error(nullptr, RS_ERR_INVALID, "n is NULL");
        int c = 0;
        hipError_t e = hipGetDeviceCount(&c);
        if (e != hipSuccess) {
            *n = 0;
            return rs::set_error(nullptr, RS_ERR_NO_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
        }
        *n = c;
        return RS_OK;
    });
}

extern "C" int rs_open(int32_t device, rs_ctx** out) {
    return rs_guard(nullptr, [&]() -> int {
        if (!out) return rs::set_error(nullptr, RS_ERR_INVALID, "out is NULL");
        *out = nullptr;
        int c = 0;
        const hipError_t ce = hipGetDeviceCount(&c);
        if (ce != hipSuccess || c == 0)
            return rs::set_error(nullptr, RS_ERR_NO_DEVICE,
                                 std::string("no HIP device visible (hipGetDeviceCount: ") + hipGetErrorString(ce) + ")");
        if (device < 0 || device >= c) return rs::set_error(nullptr, RS_ERR_INVALID, "device out of range");
        hipDeviceProp_t prop;
        RS_HIP(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return rs::set_error(nullptr, RS_ERR_NO_DEVICE,
                                 std::string("librsgpu is built for gfx950 only; device is ") + prop.gcnArchName);
        RS_HIP(hipSetDevice(device));
        auto* ctx = new rs_ctx();
        ctx->device = device;
        hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete ctx;
            return rs::set_error(nullptr, RS_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
        }
        if (hipEventCreate(&ctx->k0) != hipSuccess || hipEventCreate(&ctx->k1) != hipSuccess) {
            (void)hipStreamDestroy(ctx->stream);
            delete ctx;
            return rs::set_error(nullptr, RS_ERR_HIP, "hipEventCreate failed");
        }
        *out = ctx;
        return RS_OK;
    });
}

extern "C" void rs_close(rs_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamDestroy(ctx->stream);
    }
    if (ctx->k0) (void)hipEventDestroy(ctx->k0);
    if (ctx->k1) (void)hipEventDestroy(ctx->k1);
    ctx->svd_fit_cache.reset();  // a cached plan frees its device buffers on this device
    ctx->staging.reset();
    rs::release_pinned(ctx);
    delete ctx;
}

extern "C" int rs_open_r(int32_t device, rs_ctx** out, rs_report* report) {
    const int st = rs_open(device, out);  // (its ctx-less error is this thread's: copied before returning)
    rs::fill_report(report, st, 0);
    return st;
}

extern "C" const char* rs_last_error(const rs_ctx* ctx) {
    return ctx ? ctx->err.c_str() : rs::tls_error().c_str();
}

extern "C" int rs_last_kernel_ms(const rs_ctx* ctx, double* ms) {
    if (!ctx || !ms) return rs::set_error(nullptr, RS_ERR_INVALID, "NULL argument");
    *ms = ctx->last_kernel_ms;
    return RS_OK;
}

extern "C" int rs_synchronize(rs_ctx* ctx) {
    if (!ctx) return rs::set_error(ctx, RS_ERR_INVALID, "ctx is NULL");
    return rs_guard(ctx, [&]() -> int {
        RS_HIP(hipStreamSynchronize(ctx->stream));
        return RS_OK;
    });
}
