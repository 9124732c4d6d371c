// exp_hotlines.hip -- microbenchmark (not part of the library): does a hot 512-B row serialise
// because its eight 64-B lines share one memory channel?  Every wave repeatedly adds one value per
// dword of a row picked among H hot rows (2 f32 atomics per lane, like one Q-row delta of the SGD
// kernel).  Layout "contig": row = 512 contiguous bytes.  Layout "spread S": line c of row r sits at
// c * S + r * 64 (the row's lines S bytes apart).  Reports ns per row update (chip-wide).
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

__global__ __launch_bounds__(256) void hot(float* tab, int n_hot, long spread, int iters) {
    const int lane = threadIdx.x & 63;
    unsigned s = 2654435761u * (blockIdx.x * 4 + (threadIdx.x >> 6) + 1);
    // lane l covers dwords l and l + 64 of the row: lines (l >> 4) and 4 + (l >> 4)
    const long c0 = lane >> 4, c1 = 4 + (lane >> 4), w = lane & 15;
    for (int t = 0; t < iters; ++t) {
        s = s * 1664525u + 1013904223u;
        const int row = __builtin_amdgcn_readfirstlane((s >> 8) % n_hot);
        long a0, a1;
        if (spread == 0) {
            a0 = (long)row * 128 + lane;
            a1 = a0 + 64;
        } else {
            a0 = (c0 * spread + (long)row * 64) / 4 + w;
            a1 = (c1 * spread + (long)row * 64) / 4 + w;
        }
        atomicAdd(tab + a0, 1.0f);
        atomicAdd(tab + a1, 1.0f);
    }
}

int main() {
    float* tab;
    const size_t bytes = size_t(64) << 20;
    CHECK(hipMalloc(&tab, bytes));
    CHECK(hipMemset(tab, 0, bytes));
    const int blocks = 1024, iters = 200;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const long spreads[] = {0, 4096, 65536, 1 << 20, 4 << 20};
    const int hots[] = {1, 4, 16, 64, 256};
    for (int h : hots)
        for (long sp : spreads) {
            hipLaunchKernelGGL(hot, dim3(blocks), dim3(256), 0, 0, tab, h, sp, 10);
            CHECK(hipEventRecord(a, 0));
            hipLaunchKernelGGL(hot, dim3(blocks), dim3(256), 0, 0, tab, h, sp, iters);
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double rows = double(blocks) * 4 * iters;
            std::printf("hot=%4d spread=%8ld  %8.3f ms  %7.2f ns/row-update chip  %7.1f ns/update per hot row\n",
                        h, sp, ms, ms * 1e6 / rows, ms * 1e6 / rows * h);
            std::fflush(stdout);
        }
    return 0;
}
