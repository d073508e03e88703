// Wave-level helpers shared by the SBR / PS kernels (one wave64 owns one unit of work and hands
// values between its lanes through LDS, ds_bpermute, DPP or v_permlane*_swap).
#pragma once
#include <hip/hip_runtime.h>

namespace jaad {
namespace {

// LDS hand-off between lanes of one wave: in-order LDS queue + no compiler motion across
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// (every control used here has a source lane in the row for every lane: no old value is read, so
// none is materialised -- update_dpp(0, ...) cost a v_mov 0 per exchange)
template <int kCtrl>
__device__ __forceinline__ float dpp_mov(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kCtrl, 0xF, 0xF, true));
}
// value held by lane ^ kXor inside a 16-lane row (DPP, no LDS)
template <int kXor>
__device__ __forceinline__ float swz(float v)
{
    static_assert(kXor == 1 || kXor == 2 || kXor == 4 || kXor == 8, "row-local exchanges only");
    if constexpr (kXor == 1) return dpp_mov<0xB1>(v);                       // quad_perm [1,0,3,2]
    else if constexpr (kXor == 2) return dpp_mov<0x4E>(v);                  // quad_perm [2,3,0,1]
    else if constexpr (kXor == 4) return dpp_mov<0x1B>(dpp_mov<0x141>(v));  // row_half_mirror, quad_perm [3,2,1,0]
    else return dpp_mov<0x128>(v);                                          // row_ror:8
}
// value held by lane (row base) + 15 - (lane & 15) (DPP row_mirror)
__device__ __forceinline__ float mirror16(float v) { return dpp_mov<0x140>(v); }
// value held by lane ^ 16 / lane ^ 32: v_permlane16_swap / v_permlane32_swap of v with itself
__device__ __forceinline__ float xor16(float v, int lane)
{
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float((lane & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor32(float v, int lane)
{
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float((lane & 32) ? r[0] : r[1]);
}
__device__ __forceinline__ int bitrev5(int e) { return (int)(__builtin_bitreverse32((uint32_t)e) >> 27); }
__device__ __forceinline__ float shfl(float v, int src_lane)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}

}  // namespace
}  // namespace jaad
