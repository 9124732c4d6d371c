// exp_lds_atomics.hip -- microbenchmark (not part of the library): LDS atomic row-add throughput on
// gfx950, the cost of combining a CU's q_i deltas in LDS before one memory-side atomic per (item, CU).
// 256 blocks x NT threads (one block per CU).  Each wave repeatedly picks a pseudo-random row of a
// ROWS x 128-dword LDS table and adds 2 dwords per lane (lane l -> dwords l and 64 + l: conflict-free,
// the layout of a k = 100 row).  MODE 0 ds_add_u32, 1 ds_add_f32, 2 ds_write_b32 (baseline),
// 3 ds_add_rtn_u32, 4 ds_read_b32 x2 + ds_add_u32 x2 (read q + acc, add delta).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

constexpr int ROWS = 256;

template <int MODE, int NT>
__global__ __launch_bounds__(NT) void lds_atomic(int iters, unsigned* out) {
    __shared__ unsigned tab[ROWS * 128];
    for (int x = threadIdx.x; x < ROWS * 128; x += NT) tab[x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned s = 1234567u * (w + 1) + 7919u * blockIdx.x;
    unsigned acc = 0;
    float facc = 0.f;
    for (int t = 0; t < iters; ++t) {
        s = s * 1664525u + 1013904223u;
        const int row = __builtin_amdgcn_readfirstlane((s >> 12) & (ROWS - 1));
        unsigned* r = tab + row * 128;
        if constexpr (MODE == 0) {
            __hip_atomic_fetch_add(r + lane, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(r + 64 + lane, s ^ 5u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if constexpr (MODE == 1) {
            float* f = reinterpret_cast<float*>(r);
            __hip_atomic_fetch_add(f + lane, 1e-3f * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(f + 64 + lane, 2e-3f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if constexpr (MODE == 2) {
            r[lane] = s;
            r[64 + lane] = s ^ 5u;
        } else if constexpr (MODE == 3) {
            acc += __hip_atomic_fetch_add(r + lane, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            acc += __hip_atomic_fetch_add(r + 64 + lane, s ^ 5u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            const unsigned a = r[lane], b = r[64 + lane];
            acc += a ^ b;
            __hip_atomic_fetch_add(r + lane, s + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(r + 64 + lane, s + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    out[blockIdx.x * NT + threadIdx.x] = acc + tab[threadIdx.x] + (unsigned)facc;
}

template <int MODE, int NT>
void run(const char* name, unsigned* out) {
    const int iters = 20000;
    hipLaunchKernelGGL((lds_atomic<MODE, NT>), dim3(256), dim3(NT), 0, 0, iters, out);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((lds_atomic<MODE, NT>), dim3(256), dim3(NT), 0, 0, iters, out);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double rows = double(iters) * (NT / 64);
    std::printf("%-22s NT=%4d  %7.2f ns per 512-B row op per CU  (%6.1f cycles at 2.4 GHz)\n", name, NT,
                ms * 1e6 / rows, ms * 1e6 / rows * 2.4);
}

int main() {
    unsigned* out;
    CHECK(hipMalloc(&out, 256 * 1024 * sizeof(unsigned)));
    run<0, 256>("ds_add_u32", out);
    run<0, 512>("ds_add_u32", out);
    run<0, 1024>("ds_add_u32", out);
    run<1, 256>("ds_add_f32", out);
    run<1, 1024>("ds_add_f32", out);
    run<2, 256>("ds_write_b32", out);
    run<2, 1024>("ds_write_b32", out);
    run<3, 256>("ds_add_rtn_u32", out);
    run<3, 1024>("ds_add_rtn_u32", out);
    run<4, 256>("read2+add2 u32", out);
    run<4, 1024>("read2+add2 u32", out);
    return 0;
}
