// Experiment (round 5): the QDELTA merge pass (csrc/multi.hip qdelta_merge_kernel<16>) at configs[4] size --
// 1M item rows of 260 int32 (k = 256) -- in several shapes, to find what holds it at 4.2 TB/s (22 B per
// element: Q, Q0 read + written, the fp16 moves written, the previous merge's fp16 sum and moves read).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o qdelta_merge_bench qdelta_merge_bench.hip
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ inline float hb(uint32_t h) {
    const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, sign = (h & 0x8000u) << 16;
    uint32_t bits;
    if (e == 0) bits = __float_as_uint(static_cast<float>(m) * 5.9604644775390625e-8f);
    else if (e == 31) bits = 0x7f800000u | (m << 13);
    else bits = ((e + 112u) << 23) | (m << 13);
    return __uint_as_float(bits | sign);
}
__device__ inline int fxd(uint32_t h, float fx) { return __float2int_rn(hb(h) * fx); }
__device__ inline uint32_t pack(float a, float b) {
    const __half2 x = __floats2half2_rn(a, b);
    return __builtin_bit_cast(uint32_t, x);
}

struct Step {
    int4 v;
    uint2 d;
};
__device__ inline Step step(int4 q, int4 q0, uint2 ps, uint2 pd, float w, float fx, float fxi, bool prev) {
    const float s = w * fxi;
    Step o;
    o.d = make_uint2(pack(s * (q.x - q0.x), s * (q.y - q0.y)), pack(s * (q.z - q0.z), s * (q.w - q0.w)));
    int4 v = make_int4(q0.x + fxd(o.d.x & 0xffff, fx), q0.y + fxd(o.d.x >> 16, fx), q0.z + fxd(o.d.y & 0xffff, fx),
                       q0.w + fxd(o.d.y >> 16, fx));
    if (prev) {
        v.x += fxd(ps.x & 0xffff, fx) - fxd(pd.x & 0xffff, fx);
        v.y += fxd(ps.x >> 16, fx) - fxd(pd.x >> 16, fx);
        v.z += fxd(ps.y & 0xffff, fx) - fxd(pd.y & 0xffff, fx);
        v.w += fxd(ps.y >> 16, fx) - fxd(pd.y >> 16, fx);
    }
    o.v = v;
    return o;
}

// A: the library's shape (64-bit index and division, one vector per iteration)
__global__ __launch_bounds__(256) void kA(int4* Q, int4* Q0, const float* w, uint2* dq, const uint2* ps, const uint2* pd,
                                          int64_t n4, int32_t l4, float fx, float fxi) {
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; t < n4; t += static_cast<int64_t>(gridDim.x) * 256) {
        const Step o = step(Q[t], Q0[t], ps[t], pd[t], w[t / l4], fx, fxi, true);
        dq[t] = o.d;
        Q[t] = o.v;
        Q0[t] = o.v;
    }
}
// B: 32-bit index, U vectors per thread per iteration (loads first)
template <int U>
__global__ __launch_bounds__(256) void kB(int4* Q, int4* Q0, const float* w, uint2* dq, const uint2* ps, const uint2* pd,
                                          uint32_t n4, uint32_t l4, float fx, float fxi) {
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t t0 = blockIdx.x * 256u + threadIdx.x; t0 < n4; t0 += stride * U) {
        int4 q[U], z[U];
        uint2 a[U], b[U];
        float ww[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = t0 + u * stride;
            if (t < n4) {
                q[u] = Q[t]; z[u] = Q0[t]; a[u] = ps[t]; b[u] = pd[t]; ww[u] = w[t / l4];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = t0 + u * stride;
            if (t < n4) {
                const Step o = step(q[u], z[u], a[u], b[u], ww[u], fx, fxi, true);
                dq[t] = o.d;
                Q[t] = o.v;
                Q0[t] = o.v;
            }
        }
    }
}
// C: as B<2> with nontemporal stores
__global__ __launch_bounds__(256) void kC(int4* Q, int4* Q0, const float* w, uint2* dq, const uint2* ps, const uint2* pd,
                                          uint32_t n4, uint32_t l4, float fx, float fxi) {
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < n4; t += stride) {
        const Step o = step(Q[t], Q0[t], ps[t], pd[t], w[t / l4], fx, fxi, true);
        __builtin_nontemporal_store(o.d.x, &dq[t].x);
        __builtin_nontemporal_store(o.d.y, &dq[t].y);
        Q[t] = o.v;
        __builtin_nontemporal_store(o.v.x, &Q0[t].x);
        __builtin_nontemporal_store(o.v.y, &Q0[t].y);
        __builtin_nontemporal_store(o.v.z, &Q0[t].z);
        __builtin_nontemporal_store(o.v.w, &Q0[t].w);
    }
}
// D: copy of the same bytes (22 B per element: 12 read, 10 written) as the ceiling
__global__ __launch_bounds__(256) void kD(int4* Q, int4* Q0, uint2* dq, const uint2* ps, const uint2* pd, uint32_t n4) {
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < n4; t += stride) {
        int4 q = Q[t], z = Q0[t];
        const uint2 a = ps[t], b = pd[t];
        q.x += z.x + a.x; q.y += b.y;
        dq[t] = make_uint2(a.x ^ b.x, a.y ^ b.y);
        Q[t] = q;
        Q0[t] = z;
    }
}

// E: the library's compact layout (Q0 / wire rows of l4c = 65 vectors, Q rows of ld4 = 80), one vector per thread
__global__ __launch_bounds__(256) void kE(int4* Q, int4* Q0, const float* w, uint2* dq, const uint2* ps, const uint2* pd,
                                          uint32_t n4, uint32_t l4, uint32_t ld4, float fx, float fxi) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t < n4) {
        const uint32_t i = t / l4;
        int4& qv = Q[size_t(i) * ld4 + (t - i * l4)];
        const Step o = step(qv, Q0[t], ps[t], pd[t], w[i], fx, fxi, true);
        dq[t] = o.d;
        qv = o.v;
        Q0[t] = o.v;
    }
}
// H: one wave per row: lanes take vectors 0..63, lane 0 also the row's last vector (l4 = 65)
__global__ __launch_bounds__(256) void kH(int4* Q, int4* Q0, const float* w, uint2* dq, const uint2* ps, const uint2* pd,
                                          uint32_t ni, uint32_t l4, uint32_t ld4, float fx, float fxi) {
    const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (i >= ni) return;
    const float wi = w[i];
    for (uint32_t c = lane; c < l4; c += 64) {
        const size_t t = size_t(i) * l4 + c;
        int4& qv = Q[size_t(i) * ld4 + c];
        const Step o = step(qv, Q0[t], ps[t], pd[t], wi, fx, fxi, true);
        dq[t] = o.d;
        qv = o.v;
        Q0[t] = o.v;
    }
}

int main() {
    const uint32_t ni = 1000000, ld = 260, l4 = ld / 4;
    const uint32_t n4 = ni * l4;
    int4 *Q, *Q0;
    uint2 *dq, *ps, *pd;
    float* w;
    CK(hipMalloc(&Q, size_t(n4) * 16));
    CK(hipMalloc(&Q0, size_t(n4) * 16));
    CK(hipMalloc(&dq, size_t(n4) * 8));
    CK(hipMalloc(&ps, size_t(n4) * 8));
    CK(hipMalloc(&pd, size_t(n4) * 8));
    CK(hipMalloc(&w, size_t(ni) * 4));
    CK(hipMemset(Q, 1, size_t(n4) * 16));
    CK(hipMemset(Q0, 0, size_t(n4) * 16));
    CK(hipMemset(ps, 0, size_t(n4) * 8));
    CK(hipMemset(pd, 0, size_t(n4) * 8));
    CK(hipMemset(w, 0, size_t(ni) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 22.0 * 4 * n4;
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-34s %8.3f ms  %6.2f TB/s\n", name, ms / 10, bytes / (ms / 10 * 1e-3) / 1e12);
    };
    const float fx = 16777216.f, fxi = 1.f / fx;
    for (int g : {4096, 2048, 1024, 8192}) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "A lib shape grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL(kA, dim3(g), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, (int64_t)n4, (int32_t)l4, fx, fxi); });
        std::snprintf(nm, sizeof nm, "B<1> grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL(kB<1>, dim3(g), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, n4, l4, fx, fxi); });
        std::snprintf(nm, sizeof nm, "B<2> grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL(kB<2>, dim3(g), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, n4, l4, fx, fxi); });
        std::snprintf(nm, sizeof nm, "B<4> grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL(kB<4>, dim3(g), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, n4, l4, fx, fxi); });
        std::snprintf(nm, sizeof nm, "C nt stores grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL(kC, dim3(g), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, n4, l4, fx, fxi); });
        std::snprintf(nm, sizeof nm, "D copy ceiling grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL(kD, dim3(g), dim3(256), 0, 0, Q, Q0, dq, ps, pd, n4); });
    }
    const uint32_t full = (n4 + 255) / 256;
    {
        const uint32_t l4c = 65, nc = ni * l4c;
        const double cb = 22.0 * 4 * nc;
        auto runc = [&](const char* name, auto launch) {
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int r = 0; r < 10; ++r) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("%-34s %8.3f ms  %6.2f TB/s (compact bytes)\n", name, ms / 10, cb / (ms / 10 * 1e-3) / 1e12);
        };
        runc("E compact, vector per thread", [&] { hipLaunchKernelGGL(kE, dim3((nc + 255) / 256), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, nc, l4c, l4, fx, fxi); });
        runc("H compact, wave per row", [&] { hipLaunchKernelGGL(kH, dim3((ni + 3) / 4), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, ni, l4c, l4, fx, fxi); });
        runc("E compact, vector per thread", [&] { hipLaunchKernelGGL(kE, dim3((nc + 255) / 256), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, nc, l4c, l4, fx, fxi); });
    }
    run("B<1> one vector per thread", [&] { hipLaunchKernelGGL(kB<1>, dim3(full), dim3(256), 0, 0, Q, Q0, w, dq, ps, pd, n4, l4, fx, fxi); });
    run("D copy one vector per thread", [&] { hipLaunchKernelGGL(kD, dim3(full), dim3(256), 0, 0, Q, Q0, dq, ps, pd, n4); });
    return 0;
}
