// PS mixing step (PSImpl.ps_mix_phase, A/ = aac/src/main/java/net/sourceforge/jaad/aac/,
// A/ps/PSImpl.java:592-679) used by ps_mix_kernel (jaad_ps.hip), kept apart so that any other kernel
// mixing rows (the round-4 fusion experiments) performs the same binary32 operations in
// the same order (-ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jaad {

// QMF band 3..63 -> its group 10..21 of the T20 map (group borders 3, 4, 5, 6, 7, 8, 9, 11, 14,
// 18, 23, 35, 64)
__device__ __forceinline__ int ps_qmf_group(int band)
{
    constexpr int lo[12] = {3, 4, 5, 6, 7, 8, 9, 11, 14, 18, 23, 35};
    int g = 10;
#pragma unroll
    for (int i = 1; i < 12; i++)
        if (band >= lo[i]) g = 10 + i;
    return g;
}

// H of one group through the slots of a frame, in slot order: at each envelope border H restarts
// from the envelope's start row, then every slot advances it by the delta (the imaginary parts
// only with rot), as the Java interpolates.  hbf: the frame's rows [env][22 groups][16] (start re 4,
// im 4, delta re 4, im 4); bw: border_position[0..5] as bytes.
struct PsHWalk {
    float H[8], D[8];
    int env, next;
    __device__ __forceinline__ void begin()
    {
        env = 0;
        next = 0;
    }
    __device__ __forceinline__ void step(const float* hbf, uint64_t bw, int gr, bool rot, int n)
    {
        if (n == next) {  // uniform: the borders are per frame
            const float* hv = hbf + (env * 22 + gr) * 16;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                H[k] = hv[k];
                D[k] = hv[8 + k];
            }
            env++;
            next = (int)((bw >> (8 * env)) & 255u);
        }
#pragma unroll
        for (int k = 0; k < 4; k++) H[k] += D[k];
        if (rot)
#pragma unroll
            for (int k = 4; k < 8; k++) H[k] += D[k];
    }
};

// One slot of one (sub)band: H (h11, h12, h21, h22 real parts, then imaginary parts, advanced to
// this slot), X_left x, all-pass output r0, transient gain G -> (left, right) (PSImpl.java:640-673:
// r = G r0, l' = h11 x + h21 r, r' = h12 x + h22 r, + the IPD/OPD imaginary terms when rot)
__device__ __forceinline__ void ps_mix_slot(const float (&H)[8], bool rot, float2 x, float2 r0, float G, float2& ol,
                                            float2& orr)
{
    const float2 r = make_float2((G * r0.x), (G * r0.y));
    ol = make_float2((H[0] * x.x) + (H[2] * r.x), (H[0] * x.y) + (H[2] * r.y));
    orr = make_float2((H[1] * x.x) + (H[3] * r.x), (H[1] * x.y) + (H[3] * r.y));
    if (rot) {
        ol.x -= (H[4] * x.y) + (H[6] * r.y);
        ol.y += (H[4] * x.x) + (H[6] * r.x);
        orr.x -= (H[5] * x.y) + (H[7] * r.y);
        orr.y += (H[5] * x.x) + (H[7] * r.x);
    }
}

}  // namespace jaad
