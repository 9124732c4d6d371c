// exp_atomics.hip -- microbenchmark (not part of the library): where and how fast row-shaped
// read-modify-writes run on gfx950, for the SGD item-row write-back (K1).
// 1024 blocks x 256 threads; every wave repeatedly picks a 512-B row (128 dwords) of a table and
// adds one value per dword (2 instructions per lane), like one Q-row delta of svd_epoch_fast_kernel.
//   rows: "all"  -- uniform over the whole table (every XCD touches every row)
//         "xcd"  -- uniform over the 1/8 of the table owned by this block's XCD (HW_REG_XCC_ID)
//         "hot4" -- all waves into 4 rows (same-line serialisation)
//   op:   f32 atomic add | u32 atomic add | sc1 load + plain store (racy RMW, rate only)
// After each u32 run the table sum is compared with the number of adds: a shortfall on "all" means
// the op executed in a (non-coherent) XCD L2.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

enum { OP_F32 = 0, OP_U32 = 1, OP_RMW = 2 };
enum { ROWS_ALL = 0, ROWS_XCD = 1, ROWS_HOT = 2 };

template <int OP, int ROWS>
__global__ __launch_bounds__(256) void rmw(unsigned* tab, int n_rows, int iters) {
    const int lane = threadIdx.x & 63;
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    unsigned s = 2654435761u * (blockIdx.x * 4 + (threadIdx.x >> 6) + 1);
    const int per = n_rows / 8;
    for (int t = 0; t < iters; ++t) {
        s = s * 1664525u + 1013904223u;
        const unsigned h = __builtin_amdgcn_readfirstlane(s >> 8);
        int row;
        if (ROWS == ROWS_ALL) row = h % n_rows;
        else if (ROWS == ROWS_XCD) row = xcc * per + h % per;
        else row = h & 3;
        unsigned* r = tab + static_cast<size_t>(row) * 128;
        if (OP == OP_F32) {
            atomicAdd(reinterpret_cast<float*>(r) + lane, 1.0f);
            atomicAdd(reinterpret_cast<float*>(r) + lane + 64, 1.0f);
        } else if (OP == OP_U32) {
            atomicAdd(r + lane, 1u);
            atomicAdd(r + lane + 64, 1u);
        } else {
            const unsigned a = __hip_atomic_load(r + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned b = __hip_atomic_load(r + lane + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            r[lane] = a + 1;
            r[lane + 64] = b + 1;
        }
    }
}

template <int OP, int ROWS>
void run(const char* name, unsigned* tab, int n_rows, int iters) {
    const int blocks = 1024;
    CHECK(hipMemset(tab, 0, size_t(n_rows) * 512));
    hipLaunchKernelGGL((rmw<OP, ROWS>), dim3(blocks), dim3(256), 0, 0, tab, n_rows, iters / 8);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(tab, 0, size_t(n_rows) * 512));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((rmw<OP, ROWS>), dim3(blocks), dim3(256), 0, 0, tab, n_rows, iters);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double rows = double(blocks) * 4 * iters;
    std::printf("%-26s rows=%6d  %8.3f ms  %6.2f ns/row chip  %6.3f TB/s of row bytes", name, n_rows, ms,
                ms * 1e6 / rows, rows * 512 / (ms * 1e-3) / 1e12);
    if (OP != OP_RMW) {
        std::vector<unsigned> h(size_t(n_rows) * 128);
        CHECK(hipMemcpy(h.data(), tab, h.size() * 4, hipMemcpyDeviceToHost));
        double sum = 0;
        for (unsigned v : h) sum += OP == OP_F32 ? double(reinterpret_cast<float&>(v)) : double(v);
        std::printf("  adds %.0f / %.0f", sum, rows * 128);
    }
    std::printf("\n");
    std::fflush(stdout);
}

int main() {
    unsigned* tab;
    const int n_rows = 8 * 464;  // ~ML-1M item count, 512-B rows (k=100 padded to 128)
    CHECK(hipMalloc(&tab, size_t(8 * 65536) * 512));
    const int it = 2000;
    run<OP_F32, ROWS_ALL>("f32 atomic, all rows", tab, n_rows, it);
    run<OP_F32, ROWS_XCD>("f32 atomic, xcd rows", tab, n_rows, it);
    run<OP_U32, ROWS_ALL>("u32 atomic, all rows", tab, n_rows, it);
    run<OP_U32, ROWS_XCD>("u32 atomic, xcd rows", tab, n_rows, it);
    run<OP_RMW, ROWS_ALL>("sc1 ld + st, all rows", tab, n_rows, it);
    run<OP_RMW, ROWS_XCD>("sc1 ld + st, xcd rows", tab, n_rows, it);
    run<OP_F32, ROWS_HOT>("f32 atomic, 4 hot rows", tab, n_rows, it / 8);
    run<OP_U32, ROWS_HOT>("u32 atomic, 4 hot rows", tab, n_rows, it / 8);
    run<OP_RMW, ROWS_HOT>("sc1 ld + st, 4 hot rows", tab, n_rows, it / 8);
    run<OP_F32, ROWS_XCD>("f32 atomic, xcd rows (big)", tab, 8 * 65536, it);
    run<OP_U32, ROWS_XCD>("u32 atomic, xcd rows (big)", tab, 8 * 65536, it);
    return 0;
}
