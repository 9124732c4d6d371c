// wave.hpp -- wavefront-level primitives for gfx950 (64-lane waves, DPP within 16-lane rows).
#pragma once

#include <hip/hip_runtime.h>

namespace rs {

// DPP controls (GFX9 encoding): quad_perm xor1 / xor2, row_half_mirror, row_mirror.
constexpr int DPP_QUAD_XOR1 = 0xB1;    // [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;    // [2,3,0,1]
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_ROW_MIRROR = 0x140;

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Sum over an aligned group of G lanes (G = 4, 8 or 16) inside a DPP row.  Every lane of the group
// ends with the bitwise-identical total (each stage adds a value and its mirror; fp add commutes).
template <int G>
__device__ __forceinline__ float group_sum(float x) {
    static_assert(G == 4 || G == 8 || G == 16, "group must sit inside one 16-lane DPP row");
    x += dpp_mov<DPP_QUAD_XOR1>(x);
    x += dpp_mov<DPP_QUAD_XOR2>(x);
    if constexpr (G >= 8) x += dpp_mov<DPP_ROW_HALF_MIRROR>(x);
    if constexpr (G >= 16) x += dpp_mov<DPP_ROW_MIRROR>(x);
    return x;
}

__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
    return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

}  // namespace rs
