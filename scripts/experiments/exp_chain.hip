// exp_chain.hip -- microbenchmark for the SGD write-back design (not part of the library).
// One wave per "user" walks L random item rows of a Q table (128 floats per row, k=100 shape) with
// the FAST kernel's arithmetic, ring-prefetching D rows ahead.  Write-back modes:
//   0 float-atomic deltas (memory side)        1 sc1 stores (write-through)
//   2 plain stores                             3 Q table in LDS, ds_add_f32 deltas (rows < 256)
//   4 loads only (no write-back: the chain without store acks)
// Reports ns per rating for a single wave (chain latency) and for U waves (throughput).
#include <hip/hip_runtime.h>

#include <chrono>
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

constexpr int kOut = 0x7FFFFFF0;


template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float x) {
    x += dpp<0xB1>(x);
    x += dpp<0x4E>(x);
    x += dpp<0x141>(x);
    x += dpp<0x140>(x);
    auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
    auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

template <int MODE, int D>
__global__ __launch_bounds__(256) void chain(const int* __restrict__ items, int L, int n_users, float* Q,
                                             int q_bytes, float* out, float lr, float reg) {
#pragma clang fp contract(fast)
    constexpr int E = 2;
    __shared__ float lq[MODE == 3 ? 96 * 128 : 1];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + (threadIdx.x >> 6));
    if (MODE == 3) {
        for (int x = threadIdx.x; x < 96 * 128; x += 256) lq[x] = Q[x];
        __syncthreads();
    }
    if (w >= n_users) return;
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(Q, 0, q_bytes, 0x00020000);
    const int* it = items + static_cast<long>(w) * L;
    float p[E] = {0.01f * lane, 0.02f};
    float ring[D][E];
    const float a = 1.f - lr * reg;
    auto load = [&](float (&q)[E], int j) {
        const int item = j < L ? it[j] : 0;
        if constexpr (MODE == 3) {
#pragma unroll
            for (int x = 0; x < E; ++x) q[x] = lq[item * 128 + lane + 64 * x];
        } else {
            const int row = j < L ? item * 512 : kOut;
#pragma unroll
            for (int x = 0; x < E; ++x)
                q[x] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rq, row + lane * 4 + 256 * x, 0, 16));
        }
    };
#pragma unroll
    for (int s = 0; s < D; ++s) load(ring[s], s);
    float gb = 3.5f;
    for (int j0 = 0; j0 < L; j0 += D) {
#pragma unroll
        for (int s = 0; s < D; ++s) {
            const int j = j0 + s;
            if (j < L) {
                float* q = ring[s];
                const int item = it[j];
                float acc = p[0] * q[0] + p[1] * q[1];
                acc = wave_sum(acc);
                const float diff = gb + acc - 3.f;
                const float c = lr * diff;
                gb -= c;
                float qn[E];
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    p[x] = __builtin_fmaf(-c, q[x], p[x] * a);
                    qn[x] = __builtin_fmaf(-c, p[x], q[x] * a);
                }
                const int row = item * 512;
#pragma unroll
                for (int x = 0; x < E; ++x) {
                    if constexpr (MODE == 0)
                        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(qn[x] - q[x], rq, row + lane * 4 + 256 * x, 0, 0);
                    else if constexpr (MODE == 1)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(qn[x]), rq, row + lane * 4 + 256 * x, 0, 16);
                    else if constexpr (MODE == 2)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(qn[x]), rq, row + lane * 4 + 256 * x, 0, 0);
                    else if constexpr (MODE == 3)
                        atomicAdd(&lq[item * 128 + lane + 64 * x], qn[x] - q[x]);
                }
            }
            load(ring[s], j + D);
        }
    }
    out[w * 64 + lane] = p[0] + p[1] + gb;
}

template <int MODE, int D>
double run(const int* items, int L, int U, float* Q, int qb, float* out) {
    const int blocks = (U + 3) / 4;
    hipLaunchKernelGGL((chain<MODE, D>), dim3(blocks), dim3(256), 0, 0, items, L, U, Q, qb, out, 0.005f, 0.02f);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int reps = 5;
    CHECK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((chain<MODE, D>), dim3(blocks), dim3(256), 0, 0, items, L, U, Q, qb, out, 0.005f, 0.02f);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <int MODE, int D>
void row(const char* name, int* d_one, int* d_many, int n_items, float* Q, float* out) {
    const int qb = n_items * 512;
    const double t1 = run<MODE, D>(d_one, 2314, 1, Q, qb, out);
    const double tu = run<MODE, D>(d_many, 165, 6040, Q, qb, out);
    std::printf("%-28s D=%2d  chain %7.1f ns/rating (1 wave x 2314)   many %8.1f us (6040 x 165 = %.2f ns/rating chip)\n",
                name, D, t1 * 1e6 / 2314, tu * 1e3, tu * 1e6 / (6040.0 * 165));
}

int main() {
    const int I_glob = 3706, I_lds = 96;
    std::vector<int> one(2314), many(6040L * 165);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
    for (auto& x : one) x = rnd() % I_lds;
    for (auto& x : many) x = rnd() % I_lds;
    std::vector<int> one_g(2314), many_g(6040L * 165);
    for (auto& x : one_g) x = rnd() % I_glob;
    for (auto& x : many_g) x = rnd() % I_glob;
    int *d1, *dm, *d1g, *dmg;
    float *Q, *out;
    CHECK(hipMalloc(&d1, one.size() * 4));
    CHECK(hipMalloc(&dm, many.size() * 4));
    CHECK(hipMalloc(&d1g, one.size() * 4));
    CHECK(hipMalloc(&dmg, many.size() * 4));
    CHECK(hipMalloc(&Q, I_glob * 512));
    CHECK(hipMalloc(&out, 6040 * 64 * 4));
    CHECK(hipMemcpy(d1, one.data(), one.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dm, many.data(), many.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d1g, one_g.data(), one.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dmg, many_g.data(), many.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemset(Q, 0, I_glob * 512));
    row<0, 8>("atomic (global rows)", d1g, dmg, I_glob, Q, out);
    row<0, 16>("atomic (global rows)", d1g, dmg, I_glob, Q, out);
    row<1, 8>("sc1 store (global rows)", d1g, dmg, I_glob, Q, out);
    row<1, 16>("sc1 store (global rows)", d1g, dmg, I_glob, Q, out);
    row<2, 8>("plain store (global rows)", d1g, dmg, I_glob, Q, out);
    row<2, 16>("plain store (global rows)", d1g, dmg, I_glob, Q, out);
    row<4, 8>("loads only (global rows)", d1g, dmg, I_glob, Q, out);
    row<4, 16>("loads only (global rows)", d1g, dmg, I_glob, Q, out);
    row<3, 2>("LDS ds_add (96 rows)", d1, dm, I_lds, Q, out);
    row<3, 4>("LDS ds_add (96 rows)", d1, dm, I_lds, Q, out);
    return 0;
}
