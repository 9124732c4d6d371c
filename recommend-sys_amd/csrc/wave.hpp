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

// Wave sum ending in lane 63 (GFX9 DPP row broadcasts): the in-row tree gives every lane its row's
// sum, row_bcast:15 adds row 0 / 2's sum into rows 1 / 3, row_bcast:31 adds rows 0-1 into rows 2-3.
// Six VALU ops and a v_readlane, against ten for the all-lanes form (the value is needed as a scalar).
__device__ __forceinline__ float wave_sum_l63(float x) {
    x = group_sum<16>(x);
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xA, 0xF, false));  // row_bcast:15
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

// floor(x + 0.5) as int32 in one VALU op (v_cvt_rpi_i32_f32; __float2int_rn is rndne + cvt)
__device__ __forceinline__ int32_t cvt_rpi(float x) {
    int32_t r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

}  // namespace rs
