// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths of the SGD tile kernel
// (MI355X_MICROARCH.md §HBM: only 16-B/lane streaming reads and float atomics are calibrated).
// Each kernel touches a known byte count once (coalesced, one dword per lane):
//   load_b32_sc1   buffer_load_dword with sc1 (the tile kernel's q-row loads)
//   load_b128      16-B/lane loads (the guide's calibrated case, FETCH_SIZE = 1/2 of the bytes)
//   atomic_add_i32 buffer_atomic_add (no return; the tile kernel's run-end q deltas)
//   store_b32      dword stores
// over a 1 GiB buffer (past the 256 MiB MALL) and over a 2 MiB buffer touched 64 times (the
// ML-1M Q matrix's size: resident on die).  Build: hipcc --offload-arch=gfx950 -O3 pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__device__ inline __amdgpu_buffer_rsrc_t rsrc(void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, bytes, 0x00020000);
}

// n_dw dwords per pass, `passes` passes over the same range (offset wraps at range_dw)
__global__ void load_b32_sc1(int32_t* buf, uint32_t range_dw, uint64_t n_dw, int32_t* sink) {
    auto r = rsrc(buf, range_dw * 4u);
    int32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_dw; i += gridDim.x * 256ull)
        acc += __builtin_amdgcn_raw_buffer_load_b32(r, static_cast<uint32_t>(i % range_dw) * 4u, 0, 16);
    if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ void load_b128(int4* buf, uint32_t range_v, uint64_t n_v, int32_t* sink) {
    int32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_v; i += gridDim.x * 256ull) {
        int4 v = buf[i % range_v];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ void atomic_add_i32(int32_t* buf, uint32_t range_dw, uint64_t n_dw) {
    auto r = rsrc(buf, range_dw * 4u);
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_dw; i += gridDim.x * 256ull)
        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, r, static_cast<uint32_t>(i % range_dw) * 4u, 0, 0);
}

__global__ void store_b32(int32_t* buf, uint32_t range_dw, uint64_t n_dw) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_dw; i += gridDim.x * 256ull)
        buf[i % range_dw] = static_cast<int32_t>(i);
}

int main() {
    const uint64_t big = 1ull << 28;       // dwords: 1 GiB
    const uint32_t small = 1u << 19;       // dwords: 2 MiB
    int32_t *buf, *sink;
    CK(hipMalloc(&buf, big * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, big * 4));
    const int grid = 256 * 32;
    for (int rep = 0; rep < 2; ++rep) {
        load_b32_sc1<<<grid, 256>>>(buf, static_cast<uint32_t>(big), big, sink);
        load_b128<<<grid, 256>>>(reinterpret_cast<int4*>(buf), static_cast<uint32_t>(big / 4), big / 4, sink);
        atomic_add_i32<<<grid, 256>>>(buf, static_cast<uint32_t>(big), big);
        store_b32<<<grid, 256>>>(buf, static_cast<uint32_t>(big), big);
        // small range touched 64 times: 128 MiB of requests against a 2 MiB footprint
        load_b32_sc1<<<grid, 256>>>(buf, small, 64ull * small, sink);
        atomic_add_i32<<<grid, 256>>>(buf, small, 64ull * small);
    }
    CK(hipDeviceSynchronize());
    std::printf("bytes per launch: big %llu (1 GiB), small-range %llu (64 x 2 MiB)\n",
                static_cast<unsigned long long>(big * 4), static_cast<unsigned long long>(64ull * small * 4));
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
