// exp_lds.hip -- microbenchmark (not part of the library): LDS row read-modify-write rates on gfx950.
// 256 blocks x NT threads, one block per CU, a 64-row x 128-float table in LDS.  Each 16-lane group
// repeatedly reads a pseudo-random row (2 x ds_read_b128 per lane), computes a dot product +
// group reduction, and writes the row back as
//   MODE 0: ds_add_f32 deltas (8 per lane)     MODE 1: ds_write_b128 (2 per lane)
//   MODE 2: no write-back (reads + reduction only)
//   MODE 3: ds_add_f32 deltas, interleaved layout (col = lane + 16 x, row stride 144 floats)
// Prints ns per row-update per CU (throughput) and per group chain (one group alone).
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

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

template <int MODE, int NT>
__global__ __launch_bounds__(NT) void lds_rmw(const float4* __restrict__ init, int iters, int active_groups,
                                             float* out) {
#pragma clang fp contract(fast)
    __shared__ float4 tab[64 * 36];
    for (int x = threadIdx.x; x < 64 * 32; x += NT) tab[x] = init[x];
    __syncthreads();
    const int g = threadIdx.x >> 4, gl = threadIdx.x & 15;
    if (g >= active_groups) return;
    float4 p0 = make_float4(0.01f * gl, 0.02f, 0.03f, 0.04f), p1 = p0;
    unsigned s = 1234567u * (g + 1) + blockIdx.x;
    float gb = 0.f;
    for (int t = 0; t < iters; ++t) {
        s = s * 1664525u + 1013904223u;
        const int row = (s >> 10) & 63;
        float4* r = tab + row * 32;
        const float4 q0 = r[gl], q1 = r[16 + gl];
        float d = p0.x * q0.x + p0.y * q0.y + p0.z * q0.z + p0.w * q0.w + p1.x * q1.x + p1.y * q1.y +
                  p1.z * q1.z + p1.w * q1.w;
        d += dpp<0xB1>(d);
        d += dpp<0x4E>(d);
        d += dpp<0x141>(d);
        d += dpp<0x140>(d);
        const float c = 0.005f * (d + gb - 3.f);
        gb -= c;
        p0.x -= c * q0.x; p0.y -= c * q0.y; p0.z -= c * q0.z; p0.w -= c * q0.w;
        p1.x -= c * q1.x; p1.y -= c * q1.y; p1.z -= c * q1.z; p1.w -= c * q1.w;
        if constexpr (MODE == 3) {
            float* f = reinterpret_cast<float*>(tab) + row * 144;
            const float dq = -c;
#pragma unroll
            for (int x = 0; x < 8; ++x) atomicAdd(f + gl + 16 * x, dq * (x + 1));
        } else if constexpr (MODE == 0) {
            float* f = reinterpret_cast<float*>(r);
            atomicAdd(f + 4 * gl + 0, -c * p0.x);
            atomicAdd(f + 4 * gl + 1, -c * p0.y);
            atomicAdd(f + 4 * gl + 2, -c * p0.z);
            atomicAdd(f + 4 * gl + 3, -c * p0.w);
            atomicAdd(f + 64 + 4 * gl + 0, -c * p1.x);
            atomicAdd(f + 64 + 4 * gl + 1, -c * p1.y);
            atomicAdd(f + 64 + 4 * gl + 2, -c * p1.z);
            atomicAdd(f + 64 + 4 * gl + 3, -c * p1.w);
        } else if constexpr (MODE == 1) {
            r[gl] = make_float4(q0.x - c * p0.x, q0.y - c * p0.y, q0.z - c * p0.z, q0.w - c * p0.w);
            r[16 + gl] = make_float4(q1.x - c * p1.x, q1.y - c * p1.y, q1.z - c * p1.z, q1.w - c * p1.w);
        }
    }
    out[(blockIdx.x * NT + threadIdx.x)] = p0.x + p1.y + gb;
}

template <int MODE, int NT>
void run(const char* name, const float4* init, float* out) {
    const int iters = 4000;
    for (int full = 1; full >= 0; --full) {
        const int groups = full ? NT / 16 : 1;
        hipLaunchKernelGGL((lds_rmw<MODE, NT>), dim3(256), dim3(NT), 0, 0, init, iters, groups, out);
        CHECK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((lds_rmw<MODE, NT>), dim3(256), dim3(NT), 0, 0, init, iters, groups, out);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (full)
            std::printf("%-18s NT=%4d  throughput %6.2f ns per row-update per CU (%d groups)\n", name, NT,
                        ms * 1e6 / (double(iters) * groups), groups);
        else
            std::printf("%-18s NT=%4d  chain      %6.1f ns per row-update (1 group)\n", name, NT,
                        ms * 1e6 / iters);
    }
}

int main() {
    float4* init;
    float* out;
    CHECK(hipMalloc(&init, 64 * 32 * sizeof(float4)));
    CHECK(hipMemset(init, 0, 64 * 32 * sizeof(float4)));
    CHECK(hipMalloc(&out, 256 * 1024 * sizeof(float)));
    run<0, 256>("ds_add_f32", init, out);
    run<0, 512>("ds_add_f32", init, out);
    run<0, 1024>("ds_add_f32", init, out);
    run<1, 256>("ds_write_b128", init, out);
    run<1, 512>("ds_write_b128", init, out);
    run<1, 1024>("ds_write_b128", init, out);
    run<3, 256>("ds_add interleaved", init, out);
    run<3, 1024>("ds_add interleaved", init, out);
    run<2, 256>("read only", init, out);
    run<2, 1024>("read only", init, out);
    return 0;
}
