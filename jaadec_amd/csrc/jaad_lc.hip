// AAC-LC DSP kernel for gfx950 (CDNA4).
//
// Replaces, per channel-frame, the reference's
//   ICStream.decodeSpectralData IQ/PNS half   A/syntax/ICStream.java:222-275
//   MS.process / IS.process                   A/tools/MS.java:17-41, A/tools/IS.java:17-53
//   TNS.process (no-op in the reference)      A/tools/TNS.java:63-68  (+ ISO 4.6.9 "spec" mode)
//   FilterBank.process / MDCT / FFT           A/filterbank/FilterBank.java:39-123, MDCT.java:36-81, FFT.java:48-135
//   SampleBuffer.accept PCM packing           S/SampleBuffer.java:168-209
// in ONE pass over HBM: quantised int16 spectra in, interleaved PCM out.
//
// Work decomposition: one wave64 decodes a chunk of up to kChunkFrames consecutive frames of one
// stream; the 1024-sample IMDCT overlap of every channel stays in VGPRs between frames (lane u
// owns output positions {2u+128j} U {1023-2u-128j}); a chunk that does not start its stream
// re-decodes the previous frame to rebuild the overlap.  Each frame's 512-point complex IFFT is
// held as 8 complex values per lane and done in three register passes (bit-reversed radix-4 +
// one radix-2 stage, then 3+3 radix-2 stages) with two LDS transposes.  The butterflies,
// twiddles (the reference's float32 recurrence tables) and evaluation order are those of the
// Java code, and the file is compiled with -ffp-contract=off, so results are bit-exact.
#include <hip/hip_runtime.h>

#include "jaad_lc.h"

namespace jaad {

struct alignas(16) LdsWave {
    float buf[1024];      // spectrum / FFT transpose (float2[512]) / short-window OLA time buffer
    float gain[2][128];   // per band: +-SCALEFACTOR_TABLE[...] as ICStream.scaleFactors holds it
    uint32_t code[128];   // per band: cb_L | cb_R << 4 | ms_used << 8
};

__device__ __forceinline__ void wave_sync()
{
    // LDS traffic of one wave executes in order; this only stops the compiler from moving LDS
    // accesses across the point (lanes exchange data through LDS inside one wave).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Lane id through a volatile asm: keeps the compiler from hoisting every lane-dependent LDS
// address out of the frame loop (which otherwise costs >100 VGPRs and all occupancy).
__device__ __forceinline__ int lane_id()
{
    int v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    return v;
}

// bit-reversal of 3 bits; element r of a bit-reversed 8-block lives in register BR3[r]
__device__ constexpr int BR3[8] = {0, 4, 2, 6, 1, 5, 3, 7};

// FFT.java:113-130 radix-2 butterfly (inverse twiddle = column 1 = +sin)
__device__ __forceinline__ void bfly(float& r0, float& i0, float& r1, float& i1, float wr, float wi)
{
    float zRe = r1 * wr - i1 * wi;
    float zIm = r1 * wi + i1 * wr;
    r1 = r0 - zRe;
    i1 = i0 - zIm;
    r0 = r0 + zRe;
    i0 = i0 + zIm;
}

// FFT.java:69-108 bottom radix-4 round, inverse direction
__device__ __forceinline__ void radix4_inv(float& r0, float& i0, float& r1, float& i1, float& r2, float& i2,
                                           float& r3, float& i3)
{
    float aRe = r0 + r1, aIm = i0 + i1;
    float bRe = r2 + r3, bIm = i2 + i3;
    float cRe = r0 - r1, cIm = i0 - i1;
    float dRe = r2 - r3, dIm = i2 - i3;
    r0 = aRe + bRe;
    i0 = aIm + bIm;
    r2 = aRe - bRe;
    i2 = aIm - bIm;
    r1 = cRe - dIm;
    i1 = cIm + dRe;
    r3 = cRe + dIm;
    i3 = cIm - dRe;
}

// Pass 1 on a lane's 8 elements held in bit-reversed order r <-> register BR3[r]:
// radix-4 on r=0..3 and r=4..7, then the i=4 radix-2 stage (roots[k*m1], k=0..3).
__device__ __forceinline__ void fft_pass1(float (&re)[8], float (&im)[8], const float (*roots)[2], int m1)
{
    radix4_inv(re[BR3[0]], im[BR3[0]], re[BR3[1]], im[BR3[1]], re[BR3[2]], im[BR3[2]], re[BR3[3]], im[BR3[3]]);
    radix4_inv(re[BR3[4]], im[BR3[4]], re[BR3[5]], im[BR3[5]], re[BR3[6]], im[BR3[6]], re[BR3[7]], im[BR3[7]]);
#pragma unroll
    for (int k = 0; k < 4; k++)
        bfly(re[BR3[k]], im[BR3[k]], re[BR3[k + 4]], im[BR3[k + 4]], roots[k * m1][0], roots[k * m1][1]);
}

// Three radix-2 stages on elements base + b + B*s (s = 0..7, B = 8 or 64): strides B, 2B, 4B.
// Stage with half-size i = B*2^j has twiddle roots[k * m] with k = (element mod 2i) and
// m = n / (2i); here m = mB, mB/2, mB/4.
__device__ __forceinline__ void fft_pass3stages(float (&re)[8], float (&im)[8], const float (*roots)[2], int b,
                                                int B, int mB)
{
#pragma unroll
    for (int s = 0; s < 8; s += 2) {
        int k = b;
        bfly(re[s], im[s], re[s + 1], im[s + 1], roots[k * mB][0], roots[k * mB][1]);
    }
#pragma unroll
    for (int s0 = 0; s0 < 8; s0 += 4) {
#pragma unroll
        for (int t = 0; t < 2; t++) {
            int s = s0 + t;
            int k = b + B * (s & 1);
            bfly(re[s], im[s], re[s + 2], im[s + 2], roots[k * (mB >> 1)][0], roots[k * (mB >> 1)][1]);
        }
    }
#pragma unroll
    for (int s = 0; s < 4; s++) {
        int k = b + B * (s & 3);
        bfly(re[s], im[s], re[s + 4], im[s + 4], roots[k * (mB >> 2)][0], roots[k * (mB >> 2)][1]);
    }
}

// Math.round(float) (ties toward +inf, NaN -> 0) followed by the short clamp of
// SampleBuffer.accept (S/SampleBuffer.java:193-206); clamping first is equivalent.
__device__ __forceinline__ int java_round16(float x)
{
    if (x != x) return 0;
    x = fminf(fmaxf(x, -32768.0f), 32767.0f);
    float r = __builtin_rintf(x);
    r = (x - r == 0.5f) ? r + 1.0f : r;
    return (int)r;
}

__device__ __forceinline__ uint32_t pack16(int v, bool big_endian)
{
    uint32_t u = (uint32_t)v & 0xffffu;
    return big_endian ? (((u & 0xffu) << 8) | (u >> 8)) : u;
}

// position of FFT slot (s, half) for lane u: see file header / MDCT.java:56-80
__device__ __forceinline__ int long_pos(int u, int s, int h)
{
    int k = u + 64 * s;
    if (s < 4) return h ? 512 + 2 * k : 511 - 2 * k;
    return h ? 1535 - 2 * k : 2 * k - 512;
}

struct FrameCtx {
    int seq, shape, shape_prev;
};

// ------------------------------------------------------------------------------------------
// IMDCT (MDCT.process, N = 2048) + FilterBank window/overlap-add for long window sequences.
// Reads the channel spectrum from lw.buf, updates ov[] (overlap at long_pos), writes out[].
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void imdct_long(LdsWave& lw, const LdsTables& T, float (&re)[8], float (&im)[8])
{
    const int u = lane_id();
    // pre-IFFT complex multiplication (MDCT.java:39-42) for k = u + 64 s
#pragma unroll
    for (int s = 0; s < 8; s++) {
        int k = u + 64 * s;
        float in0 = lw.buf[2 * k];
        float in1 = lw.buf[1023 - 2 * k];
        float c = T.mdct_l[k][0], sn = T.mdct_l[k][1];
        im[s] = (in0 * c) + (in1 * sn);
        re[s] = (in1 * c) - (in0 * sn);
    }
    wave_sync();
    // pass 1: this lane is logical FFT row t = bitrev6(u): rev[8t+r] = buf[u + 64*bitrev3(r)]
    fft_pass1(re, im, T.roots_l, 64);
    float2* X = reinterpret_cast<float2*>(lw.buf);
    const int t = (int)(__builtin_bitreverse32((uint32_t)u) >> 26);
#pragma unroll
    for (int r = 0; r < 8; r++) X[8 * t + r] = make_float2(re[BR3[r]], im[BR3[r]]);
    wave_sync();
    // pass 2: elements 64a + b + 8s, stages i = 8, 16, 32 (m = 32, 16, 8)
    const int a = u >> 3, b = u & 7;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float2 v = X[64 * a + b + 8 * s];
        re[s] = v.x;
        im[s] = v.y;
    }
    fft_pass3stages(re, im, T.roots_l, b, 8, 32);
#pragma unroll
    for (int s = 0; s < 8; s++) X[64 * a + b + 8 * s] = make_float2(re[s], im[s]);
    wave_sync();
    // pass 3: elements u + 64 s, stages i = 64, 128, 256 (m = 4, 2, 1)
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float2 v = X[u + 64 * s];
        re[s] = v.x;
        im[s] = v.y;
    }
    wave_sync();
    fft_pass3stages(re, im, T.roots_l, u, 64, 4);
    // post-IFFT complex multiplication (MDCT.java:48-53)
#pragma unroll
    for (int s = 0; s < 8; s++) {
        int k = u + 64 * s;
        float c = T.mdct_l[k][0], sn = T.mdct_l[k][1];
        float t0 = re[s], t1 = im[s];
        im[s] = (t1 * c) + (t0 * sn);
        re[s] = (t0 * c) - (t1 * sn);
    }
}

// FilterBank.process for ONLY_LONG / LONG_START / LONG_STOP (FilterBank.java:41-70, 102-119)
__device__ __forceinline__ void ola_long(const LdsTables& T, const FrameCtx& fc, const float (&re)[8],
                                         const float (&im)[8], float (&ov)[16], float (&out)[16])
{
    const int u = lane_id();
    const float* LWp = T.win_long[fc.shape_prev];
    const float* LWc = T.win_long[fc.shape];
    const float* SWp = T.win_short[fc.shape_prev];
    const float* SWc = T.win_short[fc.shape];
#pragma unroll
    for (int s = 0; s < 8; s++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int P = long_pos(u, s, h);
            // first-half (buf[P]) and second-half (buf[1024+P]) IMDCT samples of this slot
            float f, g;
            if (s < 4) {
                f = h ? re[s] : -re[s];
                g = -im[s];
            } else {
                f = h ? -im[s] : im[s];
                g = re[s];
            }
            const int o = 2 * s + h;
            float o_v, n_v;
            if (fc.seq == JAAD_LONG_STOP_SEQUENCE) {
                if (P < 448) o_v = ov[o];
                else if (P < 576) o_v = ov[o] + (f * SWp[P - 448]);
                else o_v = ov[o] + f;
            } else {
                o_v = ov[o] + (f * LWp[P]);
            }
            if (fc.seq == JAAD_LONG_START_SEQUENCE) {
                if (P < 448) n_v = g;
                else if (P < 576) n_v = g * SWc[127 - (P - 448)];
                else n_v = 0.0f;
            } else {
                n_v = g * LWc[1023 - P];
            }
            out[o] = o_v;
            ov[o] = n_v;
        }
    }
}

// ------------------------------------------------------------------------------------------
// EIGHT_SHORT_SEQUENCE: 8 x MDCT(256) (64-point IFFTs), FilterBank.java:71-101.
// Lane (w = u>>3, b = u&7) holds window w's elements b + 8s.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void imdct_short(LdsWave& lw, const LdsTables& T, float (&re)[8], float (&im)[8])
{
    const int u = lane_id();
    const int w = u >> 3, b = u & 7;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        int k = b + 8 * s;
        float in0 = lw.buf[128 * w + 2 * k];
        float in1 = lw.buf[128 * w + 127 - 2 * k];
        float c = T.mdct_s[k][0], sn = T.mdct_s[k][1];
        im[s] = (in0 * c) + (in1 * sn);
        re[s] = (in1 * c) - (in0 * sn);
    }
    wave_sync();
    fft_pass1(re, im, T.roots_s, 8);
    float2* X = reinterpret_cast<float2*>(lw.buf);
    const int t = (int)(__builtin_bitreverse32((uint32_t)b) >> 29);
#pragma unroll
    for (int r = 0; r < 8; r++) X[64 * w + 8 * t + r] = make_float2(re[BR3[r]], im[BR3[r]]);
    wave_sync();
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float2 v = X[64 * w + b + 8 * s];
        re[s] = v.x;
        im[s] = v.y;
    }
    wave_sync();
    fft_pass3stages(re, im, T.roots_s, b, 8, 4);
#pragma unroll
    for (int s = 0; s < 8; s++) {
        int k = b + 8 * s;
        float c = T.mdct_s[k][0], sn = T.mdct_s[k][1];
        float t0 = re[s], t1 = im[s];
        im[s] = (t1 * c) + (t0 * sn);
        re[s] = (t0 * c) - (t1 * sn);
    }
}

// window position n (0..255) of short slot (s, j), j = 0..3, and its IMDCT value
__device__ __forceinline__ void short_slot(int b, int s, int j, const float (&re)[8], const float (&im)[8], int& n,
                                           float& v)
{
    int k = b + 8 * s;
    if (s < 4) {  // k < 32
        if (j == 0) { n = 63 - 2 * k; v = -re[s]; }
        else if (j == 1) { n = 64 + 2 * k; v = re[s]; }
        else if (j == 2) { n = 191 - 2 * k; v = -im[s]; }
        else { n = 192 + 2 * k; v = -im[s]; }
    } else {
        if (j == 0) { n = 2 * k - 64; v = im[s]; }
        else if (j == 1) { n = 191 - 2 * k; v = -im[s]; }
        else if (j == 2) { n = 2 * k + 64; v = re[s]; }
        else { n = 319 - 2 * k; v = re[s]; }
    }
}

// Overlap-add of the 8 short windows in Java's evaluation order ((ov + A) + B, A = previous
// window's falling half, B = this window's rising half) through an LDS time buffer, in two
// halves of 576 samples (out: t in [448,1024), new overlap: t in [1024,1600)).
__device__ __forceinline__ void ola_short(LdsWave& lw, const LdsTables& T, const FrameCtx& fc, const float (&re)[8],
                                          const float (&im)[8], float (&ov)[16], float (&out)[16])
{
    const int u = lane_id();
    const int w = u >> 3, b = u & 7;
    const float* SWc = T.win_short[fc.shape];
    const float* SWr = T.win_short[w == 0 ? fc.shape_prev : fc.shape];
    float* Tb = lw.buf;
#pragma unroll
    for (int half = 0; half < 2; half++) {
        const int t0 = half ? 1024 : 448;
        // init: out half <- overlap, overlap half <- -0.0 (so that -0 + A == A exactly)
        if (half == 0) {
#pragma unroll
            for (int o = 0; o < 16; o++) {
                int P = long_pos(u, o >> 1, o & 1);
                if (P >= 448) Tb[P - 448] = ov[o];
            }
        } else {
#pragma unroll
            for (int i = 0; i < 9; i++) Tb[u + 64 * i] = -0.0f;
        }
        wave_sync();
#pragma unroll
        for (int phase = 0; phase < 2; phase++) {  // 0: falling halves (A), 1: rising halves (B)
#pragma unroll
            for (int s = 0; s < 8; s++) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    int n;
                    float v;
                    short_slot(b, s, j, re, im, n, v);
                    const bool rising = n < 128;
                    if (rising != (phase == 1)) continue;
                    int t = 448 + 128 * w + n;
                    if ((t >= 1024) != (half == 1)) continue;
                    float c = rising ? v * SWr[n] : v * SWc[255 - n];
                    Tb[t - t0] = Tb[t - t0] + c;
                }
            }
            wave_sync();
        }
#pragma unroll
        for (int o = 0; o < 16; o++) {
            int P = long_pos(u, o >> 1, o & 1);
            if (half == 0) out[o] = (P >= 448) ? Tb[P - 448] : ov[o];
            else ov[o] = (P < 576) ? Tb[P] : 0.0f;
        }
        wave_sync();
    }
}

// ------------------------------------------------------------------------------------------
// TNS, spec mode (ISO/IEC 14496-3 4.6.9.3), in place on lw.buf; one lane per filter.
// The reference parses TNS (A/tools/TNS.java:35-61) but its process() is a no-op.
// ------------------------------------------------------------------------------------------
__device__ void tns_spec(LdsWave& lw, const LdsTables& T, const jaad_ics_info& info, const jaad_tns* tp)
{
    const int u = lane_id();
    const bool is_short = info.window_sequence == JAAD_EIGHT_SHORT_SEQUENCE;
    const int nswb = is_short ? T.nswb_s : T.nswb_l;
    const int16_t* offs = is_short ? T.swb_s : T.swb_l;
    const int tns_max = is_short ? T.tns_max_s : T.tns_max_l;
    const int nf = tp->n_filters;
    float* scratch = &lw.gain[0][0];  // 384 floats: 8 filters x 48 (band info is dead here)
    if (u < nf && u < 8) {
        const jaad_tns_filter& F = tp->filt[u];
        // top/bottom band of this filter: walk the filters of the same window parsed before it
        int top = nswb, bottom = nswb;
        for (int f = 0; f <= u; f++) {
            const jaad_tns_filter& G = tp->filt[f];
            if (G.window != F.window) continue;
            top = bottom;
            bottom = top - G.length;
            if (bottom < 0) bottom = 0;
        }
        const int order = F.order > 20 ? 20 : F.order;
        float* a = scratch + 48 * u;  // a[0..20], b[21..41], tmp2 -> reuse b region
        const float* tab = T.tns_coef[2 * ((F.flags >> 2) & 1) + ((F.flags >> 1) & 1)];
        a[0] = 1.0f;
        for (int m = 1; m <= order; m++) {
            float tm = -tab[F.coef[m - 1] & 15];
            for (int i = 1; i < m; i++) a[21 + i] = a[i] + tm * a[m - i];
            for (int i = 1; i < m; i++) a[i] = a[21 + i];
            a[m] = tm;
        }
        int s = bottom < tns_max ? bottom : tns_max;
        if (s > info.max_sfb) s = info.max_sfb;
        int e = top < tns_max ? top : tns_max;
        if (e > info.max_sfb) e = info.max_sfb;
        int start = offs[s], end = offs[e];
        int size = end - start;
        if (order > 0 && size > 0) {
            int inc = 1;
            if (F.flags & 1) {
                inc = -1;
                start = end - 1;
            }
            float* x = lw.buf + (is_short ? 128 * F.window : 0) + start;
            for (int n = 0; n < size; n++) {
                float y = x[n * inc];
                for (int j = 0; j < order; j++) {
                    float st = (n - 1 - j >= 0) ? x[(n - 1 - j) * inc] : 0.0f;
                    y -= st * a[j + 1];
                }
                x[n * inc] = y;
            }
        }
    }
    wave_sync();
}

// ------------------------------------------------------------------------------------------
// PNS slow path (ICStream.java:241-257): lane 0 replays the static LCG in parse order.
// ------------------------------------------------------------------------------------------
__device__ void pns_fill(LdsWave& lw, const LdsTables& T, const jaad_ics_info& info, int c, const uint8_t* cbrow)
{
    if (lane_id() == 0) {
        const bool is_short = info.window_sequence == JAAD_EIGHT_SHORT_SEQUENCE;
        const int16_t* offs = is_short ? T.swb_s : T.swb_l;
        int glen[8], ng = 1;
        glen[0] = 1;
        if (is_short)
            for (int i = 0; i < 7; i++) {
                if (info.grouping & (1u << i)) glen[ng - 1]++;
                else glen[ng++] = 1;
            }
        uint32_t rs = info.pns_state;
        const int maxSFB = info.max_sfb;
        for (int g = 0, idx = 0, groupOff = 0; g < ng; g++) {
            for (int sfb = 0; sfb < maxSFB; sfb++, idx++) {
                if (cbrow[idx] != JAAD_NOISE_HCB) continue;
                int off = groupOff + offs[sfb];
                int width = offs[sfb + 1] - offs[sfb];
                float sfv = lw.gain[c][idx];
                for (int w = 0; w < glen[g]; w++, off += 128) {
                    float energy = 0.0f;
                    for (int k = 0; k < width; k++) {
                        rs = 1664525u * rs + 1013904223u;
                        float v = (float)(int32_t)rs;
                        lw.buf[off + k] = v;
                        energy += v * v;
                    }
                    float scale = (float)((double)sfv / sqrt((double)energy));
                    for (int k = 0; k < width; k++) lw.buf[off + k] *= scale;
                }
            }
            groupOff += glen[g] << 7;
        }
    }
    wave_sync();
}

// band index of the quad of bins starting at position p (4-aligned) for this ICS, or -1
__device__ __forceinline__ int band_of(const LdsTables& T, const jaad_ics_info& info, int p)
{
    int sfb, g = 0;
    if (info.window_sequence == JAAD_EIGHT_SHORT_SEQUENCE) {
        int w = p >> 7;
        sfb = T.quad2band_s[(p & 127) >> 2];
        g = w - __builtin_popcount(info.grouping & ((1u << w) - 1u));
    } else {
        sfb = T.quad2band_l[p >> 2];
    }
    if (sfb >= info.max_sfb) return -1;
    return g * info.max_sfb + sfb;
}

__device__ __forceinline__ float iq_value(const LdsTables& T, const float* __restrict__ iq_table, int qv, float gain)
{
    int a = qv < 0 ? -qv : qv;
    float m = a < 128 ? T.iq_head[a] : iq_table[a > 8190 ? 8190 : a];
    float x = m * gain;  // (q>0 ? IQ[q] : -IQ[-q]) * sf  ==  +-(IQ[|q|] * sf) exactly (q = 0 -> -0)
    return qv > 0 ? x : -x;
}

#ifndef JAAD_WAVES_PER_EU
#define JAAD_WAVES_PER_EU 2
#endif
template <bool kTnsSpec, int kOut>
__global__ __launch_bounds__(kWGThreads, JAAD_WAVES_PER_EU) void lc_decode_kernel(KernelArgs A)
{
    __shared__ LdsTables T;
    __shared__ LdsWave W[kWavesPerWG];

    // stage the constant tables (one coalesced copy per workgroup)
    {
        const uint4* src = reinterpret_cast<const uint4*>(A.tables);
        uint4* dst = reinterpret_cast<uint4*>(&T);
        for (int i = threadIdx.x; i < (int)(sizeof(LdsTables) / 16); i += kWGThreads) dst[i] = src[i];
    }
    __syncthreads();

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int u = lane_id();
    LdsWave& lw = W[wave];
    const int nch = A.nch;
    constexpr bool big_endian = !(kOut & JAAD_PCM_LITTLE_ENDIAN);
    constexpr bool out_f32 = (kOut & JAAD_PCM_FLOAT32) != 0;

    for (uint32_t ci = blockIdx.x * kWavesPerWG + wave; ci < A.n_chunks; ci += gridDim.x * kWavesPerWG) {
        const ChunkDesc cd = A.chunks[ci];
        const int nfr = cd.info & 0xffff;
        const bool prefix = (cd.info & kChunkPrefix) != 0;
        float ovL[16], ovR[16];
        if (cd.info & kChunkLoadState) {
            const float* st = A.state_in + (size_t)cd.slot * 2048;
#pragma unroll
            for (int o = 0; o < 16; o++) {
                int P = long_pos(u, o >> 1, o & 1);
                ovL[o] = st[P];
                ovR[o] = st[1024 + P];
            }
        } else {
#pragma unroll
            for (int o = 0; o < 16; o++) ovL[o] = ovR[o] = 0.0f;
        }
        const int f_first = (int)cd.frame0 - (prefix ? 1 : 0);
        const int f_end = (int)cd.frame0 + nfr;
        for (int f = f_first; f < f_end; f++) {
            const bool emit = f >= (int)cd.frame0;
            const size_t cf0 = (size_t)f * nch;
            const jaad_ics_info iL = A.ics[cf0];
            const jaad_ics_info iR = nch == 2 ? A.ics[cf0 + 1] : iL;

            // ---- per-band side info -> LDS (gain as ICStream.scaleFactors holds it, codebooks, ms bit)
#pragma unroll
            for (int hb = 0; hb < 2; hb++) {
                const int idx = u + 64 * hb;
                uint32_t code = 0;
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    if (c >= nch) break;
                    const jaad_ics_info& ic = c ? iR : iL;
                    const int ng = ic.window_sequence == JAAD_EIGHT_SHORT_SEQUENCE ? 8 - __builtin_popcount(ic.grouping & 0x7f) : 1;
                    if (idx < ng * ic.max_sfb) {
                        const size_t row = (cf0 + c) * 128 + idx;
                        uint32_t cbv = A.cb[row];
                        float g = T.sf_gain[A.sf[row]];
                        lw.gain[c][idx] = cbv == JAAD_NOISE_HCB ? -g : g;
                        code |= (cbv & 15u) << (4 * c);
                    }
                }
                if (nch == 2 && (iL.flags & JAAD_ICS_MS_PRESENT) && A.ms_used)
                    code |= (uint32_t)((A.ms_used[(size_t)f * 2 + (idx >> 6)] >> (idx & 63)) & 1u) << 8;
                lw.code[idx] = code;
            }
            wave_sync();

            // ---- inverse quantisation: lane owns bins 8u+512h+i (h = 0,1; i = 0..7), i.e. four band quads
            float x[2][16];
            int bidx[2][4];
#pragma unroll
            for (int c = 0; c < 2; c++) {
                if (c >= nch) break;
                const jaad_ics_info& ic = c ? iR : iL;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int4 qv4 = *reinterpret_cast<const int4*>(A.q + (cf0 + c) * 1024 + 512 * h + 8 * u);
                    const int16_t* qv = reinterpret_cast<const int16_t*>(&qv4);
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int bi = band_of(T, ic, 512 * h + 8 * u + 4 * j);
                        bidx[c][2 * h + j] = bi;
                        const uint32_t cbv = bi >= 0 ? (lw.code[bi] >> (4 * c)) & 15u : 0u;
                        const float g = bi >= 0 ? lw.gain[c][bi] : 0.0f;
                        const bool spectral = cbv != JAAD_ZERO_HCB && cbv != JAAD_NOISE_HCB &&
                                              cbv != JAAD_INTENSITY_HCB && cbv != JAAD_INTENSITY_HCB2;
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            x[c][8 * h + 4 * j + i] = spectral ? iq_value(T, A.iq_table, qv[4 * j + i], g) : 0.0f;
                    }
                }
            }
            // ---- PNS (rare): fill noise bands through LDS
#pragma unroll
            for (int c = 0; c < 2; c++) {
                if (c >= nch) break;
                const jaad_ics_info& ic = c ? iR : iL;
                if (ic.flags & JAAD_ICS_HAS_PNS) {
#pragma unroll
                    for (int i = 0; i < 16; i++) lw.buf[8 * u + 512 * (i >> 3) + (i & 7)] = x[c][i];
                    wave_sync();
                    pns_fill(lw, T, ic, c, A.cb + (cf0 + c) * 128);
#pragma unroll
                    for (int i = 0; i < 16; i++) x[c][i] = lw.buf[8 * u + 512 * (i >> 3) + (i & 7)];
                    wave_sync();
                }
            }
            if (nch == 2) {
                // ---- M/S (MS.java:17-41): common window, mask present, both codebooks < NOISE_HCB
                if ((iL.flags & JAAD_ICS_COMMON_WINDOW) && (iL.flags & JAAD_ICS_MS_PRESENT)) {
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        const int bi = bidx[0][h];
                        const uint32_t code = bi >= 0 ? lw.code[bi] : 0u;
                        if (bi >= 0 && (code & 0x100u) && (code & 15u) < JAAD_NOISE_HCB && ((code >> 4) & 15u) < JAAD_NOISE_HCB) {
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                float l = x[0][4 * h + i], r = x[1][4 * h + i];
                                float tt = l - r;
                                x[0][4 * h + i] = l + r;
                                x[1][4 * h + i] = tt;
                            }
                        }
                    }
                }
                // ---- I/S (IS.java:17-53), right channel's bands
                if (iR.flags & JAAD_ICS_HAS_IS) {
                    const bool msp = (iL.flags & JAAD_ICS_MS_PRESENT) != 0;
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        const int bi = bidx[1][h];
                        const uint32_t code = bi >= 0 ? lw.code[bi] : 0u;
                        const uint32_t cbr = (code >> 4) & 15u;
                        if (bi >= 0 && (cbr == JAAD_INTENSITY_HCB || cbr == JAAD_INTENSITY_HCB2)) {
                            int cs = cbr == JAAD_INTENSITY_HCB ? 1 : -1;
                            if (msp) cs *= (code & 0x100u) ? -1 : 1;
                            const float scale = (float)cs * lw.gain[1][bi];
#pragma unroll
                            for (int i = 0; i < 4; i++) x[1][4 * h + i] = x[0][4 * h + i] * scale;
                        }
                    }
                }
            }

            // ---- per channel: (TNS) -> IMDCT -> window/OLA -> PCM
            uint32_t pk[16];   // int16 modes: (L | R << 16) per slot
            float pf[2][16];   // f32 mode
#pragma unroll
            for (int c = 0; c < 2; c++) {
                if (c >= nch) break;
                const jaad_ics_info& ic = c ? iR : iL;
                float(&ov)[16] = c ? ovR : ovL;
#pragma unroll
                for (int i = 0; i < 16; i++) lw.buf[8 * u + 512 * (i >> 3) + (i & 7)] = x[c][i];
                wave_sync();
                const bool dump = A.dbg && ci == 0 && f == (int)cd.frame0;
                if (dump)
                    for (int i = 0; i < 16; i++) A.dbg[1024 * c + 8 * u + 512 * (i >> 3) + (i & 7)] = x[c][i];
                if (kTnsSpec && A.tns_mode == JAAD_TNS_SPEC && (ic.flags & JAAD_ICS_TNS) && A.tns)
                    tns_spec(lw, T, ic, A.tns + cf0 + c);
                FrameCtx fc{ic.window_sequence, ic.window_shape, ic.window_shape_prev};
                float re[8], im[8], out[16];
#ifndef JAAD_EXP_NO_SHORT
                if (fc.seq == JAAD_EIGHT_SHORT_SEQUENCE) {
                    imdct_short(lw, T, re, im);
                    ola_short(lw, T, fc, re, im, ov, out);
                } else
#endif
                {
                    imdct_long(lw, T, re, im);
                    if (dump)
                        for (int s2 = 0; s2 < 8; s2++) {
                            A.dbg[2048 + 1024 * c + 2 * (u + 64 * s2)] = re[s2];
                            A.dbg[2048 + 1024 * c + 2 * (u + 64 * s2) + 1] = im[s2];
                        }
                    ola_long(T, fc, re, im, ov, out);
                }
                wave_sync();
                if (dump)
                    for (int o = 0; o < 16; o++) A.dbg[4096 + 1024 * c + long_pos(u, o >> 1, o & 1)] = out[o];
                if (emit) {
#pragma unroll
                    for (int o = 0; o < 16; o++) {
                        if constexpr (out_f32) {
                            pf[c][o] = out[o];
                        } else {
                            uint32_t v = pack16(java_round16(out[o]), big_endian);
                            pk[o] = c ? (pk[o] | (v << 16)) : v;
                        }
                    }
                }
            }
            if (!emit) continue;
            if (nch == 1) {  // mono -> stereo duplication (SyntacticElements.java:243-245)
#pragma unroll
                for (int o = 0; o < 16; o++) {
                    if constexpr (out_f32) pf[1][o] = pf[0][o];
                    else pk[o] = pk[o] | (pk[o] << 16);
                }
            }
            // ---- PCM store: lane u writes samples 2u+128j and 2u+128j+1 (the latter computed by
            // lane 63-u as its odd slot 7-j), i.e. 512 contiguous bytes per wave instruction
            if constexpr (!out_f32) {
                uint2* dst = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(A.pcm) + (size_t)f * 4096);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    // even slot of column j and odd slot of column 7-j (see long_pos)
                    const int se = (j + 4) & 7;           // slot s whose even position is column j
                    const int oe = 2 * se + (se < 4 ? 1 : 0);
                    const int so = ((7 - j) + 4) & 7;     // slot s whose odd position is column 7-j
                    const int oo = 2 * so + (so < 4 ? 0 : 1);
                    uint32_t partner = (uint32_t)__shfl_xor((int)pk[oo], 63);
                    dst[u + 64 * j] = make_uint2(pk[oe], partner);
                }
            } else {
                float4* dst = reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(A.pcm) + (size_t)f * 8192);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int se = (j + 4) & 7;
                    const int oe = 2 * se + (se < 4 ? 1 : 0);
                    const int so = ((7 - j) + 4) & 7;
                    const int oo = 2 * so + (so < 4 ? 0 : 1);
                    float pl = __shfl_xor(pf[0][oo], 63);
                    float pr = __shfl_xor(pf[1][oo], 63);
                    dst[u + 64 * j] = make_float4(pf[0][oe], pf[1][oe], pl, pr);
                }
            }
        }
        if (cd.info & kChunkStoreState) {
            float* st = A.state_out + (size_t)cd.slot * 2048;
#pragma unroll
            for (int o = 0; o < 16; o++) {
                int P = long_pos(u, o >> 1, o & 1);
                st[P] = ovL[o];
                st[1024 + P] = nch == 2 ? ovR[o] : 0.0f;
            }
        }
    }
}


}  // namespace jaad

namespace jaad {
hipError_t launch_lc(const KernelArgs& a, int grid, hipStream_t stream, bool tns_spec)
{
#define JAAD_LAUNCH(T, O) hipLaunchKernelGGL((lc_decode_kernel<T, O>), dim3(grid), dim3(kWGThreads), 0, stream, a)
    const int o = (a.out_mode & JAAD_PCM_FLOAT32) ? 2 : (a.out_mode & JAAD_PCM_LITTLE_ENDIAN) ? 1 : 0;
    if (tns_spec) {
        if (o == 2) JAAD_LAUNCH(true, JAAD_PCM_FLOAT32);
        else if (o == 1) JAAD_LAUNCH(true, JAAD_PCM_LITTLE_ENDIAN);
        else JAAD_LAUNCH(true, JAAD_PCM_BIG_ENDIAN);
    } else {
        if (o == 2) JAAD_LAUNCH(false, JAAD_PCM_FLOAT32);
        else if (o == 1) JAAD_LAUNCH(false, JAAD_PCM_LITTLE_ENDIAN);
        else JAAD_LAUNCH(false, JAAD_PCM_BIG_ENDIAN);
    }
#undef JAAD_LAUNCH
    return hipGetLastError();
}
}  // namespace jaad
