// Wave-level helpers shared by the SBR / PS kernels (one wave64 owns one unit of work and hands
// values between its lanes through LDS or ds_swizzle / ds_bpermute).
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

template <int kXor>
__device__ __forceinline__ float swz(float v)
{
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (kXor << 10)));
}
__device__ __forceinline__ float shfl(float v, int src_lane)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}

}  // namespace
}  // namespace jaad
