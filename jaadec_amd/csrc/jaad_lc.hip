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
// Work decomposition.  A workgroup = 4 waves.  For a CPE stream the two waves of a "pair" each
// own one channel of a chunk of consecutive frames (mono: every wave its own stream); the pair
// meets in LDS (4 workgroup barriers per frame) for M/S and I/S and to interleave the PCM.  The
// 1024-sample IMDCT overlap of a channel stays in its wave's VGPRs between frames (lane u owns
// output positions {2u+128j} U {1023-2u-128j}); a chunk that does not start its stream
// re-decodes the previous frame to rebuild it.  All global inputs of frame f+1 are loaded while
// frame f is computed.  The 512-point complex IFFT of a frame is 8 complex values per lane in
// three register passes (bit-reversed radix-4 + one radix-2 stage, then 3 + 3 radix-2 stages)
// with two XOR-swizzled LDS transposes.  Butterflies, twiddles (the reference's float32
// recurrence tables) and evaluation order are those of the Java code, and the file is compiled
// with -ffp-contract=off, so the results are bit-exact.
#include <hip/hip_runtime.h>

#include "jaad_lc.h"

#ifndef JAAD_WAVES_PER_EU
#define JAAD_WAVES_PER_EU 4
#endif

namespace jaad {

// per pair (CPE) or per two mono streams: band side info, written by the owning wave
struct alignas(16) PairBands {
    float gain[2][128];     // +-SCALEFACTOR_TABLE[...] as ICStream.scaleFactors holds it
    uint8_t sf[2][128];     // raw scalefactor-table index - 100
    uint8_t cb[2][128];     // section codebook (sfbCB)
    uint8_t ms[128];        // ms_used bit per band (CPE, written by the left-channel wave)
};

// Lane id through a volatile asm: keeps the compiler from hoisting every lane-dependent LDS
// address out of the frame loop (which otherwise costs >100 VGPRs and all occupancy).
__device__ __forceinline__ int lane_id()
{
#ifndef JAAD_HOISTABLE_LANE
    int v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
#else
    int v = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#endif
    __builtin_assume(v >= 0 && v < 64);
    return v;
}

#ifdef JAAD_STAMPS
__device__ __forceinline__ uint32_t stamp()
{
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return (uint32_t)t;
}
#define STAMP(k)                                                                                     \
    do {                                                                                             \
        uint32_t t_ = stamp();                                                                       \
        if (A.dbg && lane_id() == 0 && (k) < 32)                                                     \
            reinterpret_cast<uint32_t*>(A.dbg)[(size_t)(blockIdx.x * kWavesPerWG + wave) * 32 + (k)] = t_; \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

__device__ __forceinline__ void wave_sync()
{
    // LDS traffic of one wave executes in order; this only stops the compiler from moving LDS
    // accesses across the point (lanes of one wave exchange data through LDS).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kWaveBuf = 1152;  // floats of LDS per wave

// spectrum layout in a wave's buffer: even bins at [0,576), odd bins at [576,1152), bin-pair
// index j padded by 8 every 64 so the lane-parallel pre-twiddle reads of long (k = u + 64s)
// and short (k = 64w + b + 8s) windows are conflict free with base + immediate addressing
__device__ __forceinline__ int eo_idx(int p)
{
    int j = p >> 1;
    return (p & 1) * 576 + j + 8 * (j >> 6);
}
// IFFT transpose layout (complex index): one pad slot every 16 (<= 2-way conflicts, affine)
__device__ __forceinline__ int xs(int i) { return i + (i >> 4); }

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
// radix-4 on r=0..3 and r=4..7, then the i=4 radix-2 stage with twiddles w[k*wstride], k=0..3.
__device__ __forceinline__ void fft_pass1(float (&re)[8], float (&im)[8], const float (*w)[2], int wstride)
{
    radix4_inv(re[BR3[0]], im[BR3[0]], re[BR3[1]], im[BR3[1]], re[BR3[2]], im[BR3[2]], re[BR3[3]], im[BR3[3]]);
    radix4_inv(re[BR3[4]], im[BR3[4]], re[BR3[5]], im[BR3[5]], re[BR3[6]], im[BR3[6]], re[BR3[7]], im[BR3[7]]);
#pragma unroll
    for (int k = 0; k < 4; k++)
        bfly(re[BR3[k]], im[BR3[k]], re[BR3[k + 4]], im[BR3[k + 4]], w[k * wstride][0], w[k * wstride][1]);
}

// Three radix-2 stages on elements (base + b + B*s), s = 0..7: pairs (s,s+1), (s,s+2), (s,s+4).
// tw(j) returns the twiddle of "slot" j: 0 for the first stage, 1+(s&1) for the second,
// 3+s for the third (the tables are pre-arranged that way, see build_lds_tables).
template <typename TW>
__device__ __forceinline__ void fft_3stages(float (&re)[8], float (&im)[8], TW tw)
{
    {
        float wr, wi;
        tw(0, wr, wi);
#pragma unroll
        for (int s = 0; s < 8; s += 2) bfly(re[s], im[s], re[s + 1], im[s + 1], wr, wi);
    }
#pragma unroll
    for (int e = 0; e < 2; e++) {
        float wr, wi;
        tw(1 + e, wr, wi);
        bfly(re[e], im[e], re[e + 2], im[e + 2], wr, wi);
        bfly(re[4 + e], im[4 + e], re[6 + e], im[6 + e], wr, wi);
    }
#pragma unroll
    for (int s = 0; s < 4; s++) {
        float wr, wi;
        tw(3 + s, wr, wi);
        bfly(re[s], im[s], re[s + 4], im[s + 4], wr, wi);
    }
}

// position of IMDCT output slot o = 2s+h for lane u (MDCT.java:56-80 reorder)
__device__ __forceinline__ int long_pos(int u, int o)
{
    int s = o >> 1, h = o & 1, k = u + 64 * s;
    if (s < 4) return h ? 512 + 2 * k : 511 - 2 * k;
    return h ? 1535 - 2 * k : 2 * k - 512;
}

// Math.round(float) (ties toward +inf, NaN -> 0) then the short clamp of SampleBuffer.accept
// (S/SampleBuffer.java:193-206).  floor/sub/compare are exact; v_cvt_i32_f32 maps NaN to 0
// and saturates out-of-range values.
__device__ __forceinline__ int java_round16(float x)
{
    float y = __builtin_floorf(x);
    float r = (x - y >= 0.5f) ? y + 1.0f : y;
    int v;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(v) : "v"(r));
    return v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
}

struct FrameCtx {
    int seq, shape, shape_prev;
};

// jaad_ics_info unpacked into wave-uniform scalars (kept in SGPRs; a struct of bytes selected
// at run time would be spilled to scratch)
struct Ics {
    int seq, shape, shape_prev, max_sfb, grouping, flags;
    uint32_t pns;
};
__device__ __forceinline__ Ics load_ics(const jaad_ics_info* p)
{
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
    const uint32_t a = __builtin_amdgcn_readfirstlane(w[0]);
    const uint32_t b = __builtin_amdgcn_readfirstlane(w[1]);
    Ics r;
    r.seq = a & 0xff;
    r.shape = (a >> 8) & 0xff;
    r.shape_prev = (a >> 16) & 0xff;
    r.max_sfb = a >> 24;
    r.grouping = b & 0xff;
    r.flags = (b >> 8) & 0xff;
    r.pns = __builtin_amdgcn_readfirstlane(w[2]);
    return r;
}
__device__ __forceinline__ Ics sel_ics(bool c, const Ics& x, const Ics& y)
{
    Ics r;
    r.seq = c ? x.seq : y.seq;
    r.shape = c ? x.shape : y.shape;
    r.shape_prev = c ? x.shape_prev : y.shape_prev;
    r.max_sfb = c ? x.max_sfb : y.max_sfb;
    r.grouping = c ? x.grouping : y.grouping;
    r.flags = c ? x.flags : y.flags;
    r.pns = c ? x.pns : y.pns;
    return r;
}

// ------------------------------------------------------------------------------------------
// IMDCT N = 2048 (MDCT.process): lane u holds k = u + 64 s.  Reads the spectrum from buf.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void imdct_long(float* buf, const LdsTables& T, int u, float (&re)[8], float (&im)[8])
{
#pragma unroll
    for (int s = 0; s < 8; s++) {
        int k = u + 64 * s;
        float in0 = buf[eo_idx(2 * k)];
        float in1 = buf[eo_idx(1023 - 2 * k)];
        float c = T.mdct_l[k][0], sn = T.mdct_l[k][1];
        im[s] = (in0 * c) + (in1 * sn);  // MDCT.java:39-42
        re[s] = (in1 * c) - (in0 * sn);
    }
    wave_sync();
    // pass 1: this lane is bit-reversed row t = bitrev6(u): rev[8t+r] = buf[u + 64*bitrev3(r)]
    fft_pass1(re, im, T.tw1, 1);
    float2* X = reinterpret_cast<float2*>(buf);
    const int t = (int)(__builtin_bitreverse32((uint32_t)u) >> 26);
#pragma unroll
    for (int r = 0; r < 8; r++) X[xs(8 * t + r)] = make_float2(re[BR3[r]], im[BR3[r]]);
    wave_sync();
    // pass 2: elements 64a + b + 8s, stages i = 8, 16, 32
    const int a = u >> 3, b = u & 7;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float2 v = X[xs(64 * a + b + 8 * s)];
        re[s] = v.x;
        im[s] = v.y;
    }
    fft_3stages(re, im, [&](int j, float& wr, float& wi) {
        wr = T.tw2[j][b][0];
        wi = T.tw2[j][b][1];
    });
#pragma unroll
    for (int s = 0; s < 8; s++) X[xs(64 * a + b + 8 * s)] = make_float2(re[s], im[s]);
    wave_sync();
    // pass 3: elements u + 64 s, stages i = 64, 128, 256
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float2 v = X[xs(u + 64 * s)];
        re[s] = v.x;
        im[s] = v.y;
    }
    wave_sync();
    // stages 64 (m = 4, k = u), 128 (m = 2, k = u + 64e), 256 (m = 1, k = u + 64s)
    fft_3stages(re, im, [&](int j, float& wr, float& wi) {
        const int idx = j == 0 ? 4 * u : (j < 3 ? 2 * (u + 64 * (j - 1)) : u + 64 * (j - 3));
        wr = T.roots_l[idx][0];
        wi = T.roots_l[idx][1];
    });
#pragma unroll
    for (int s = 0; s < 8; s++) {  // MDCT.java:48-53
        int k = u + 64 * s;
        float c = T.mdct_l[k][0], sn = T.mdct_l[k][1];
        float t0 = re[s], t1 = im[s];
        im[s] = (t1 * c) + (t0 * sn);
        re[s] = (t0 * c) - (t1 * sn);
    }
}

// FilterBank.process for ONLY_LONG / LONG_START / LONG_STOP (FilterBank.java:41-70, 102-119).
// Lane u's slot (s,h) holds output position P = long_pos(u, 2s+h); its mirror 1023-P is slot
// (s,1-h) of the same lane, so the falling window W[1023-P] is win_slot[shape][o^1][u].
// Specialised per sequence so the common ONLY_LONG path carries no joint-window logic.
template <int kSeq>
__device__ __forceinline__ void ola_long_t(const LdsTables& T, const FrameCtx& fc, const float (&re)[8],
                                           const float (&im)[8], float (&ov)[16], float (&out)[16])
{
    const int u = lane_id();
    const float* SWp = T.win_short[fc.shape_prev];
    const float* SWc = T.win_short[fc.shape];
    const float* Wp = &T.win_slot[fc.shape_prev][0][0];
    const float* Wc = &T.win_slot[fc.shape][0][0];
#pragma unroll
    for (int s = 0; s < 8; s++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int o = 2 * s + h;
            float f, g;  // IMDCT samples buf[P] and buf[1024+P]
            if (s < 4) {
                f = h ? re[s] : -re[s];
                g = -im[s];
            } else {
                f = h ? -im[s] : im[s];
                g = re[s];
            }
            float o_v, n_v;
            if constexpr (kSeq == JAAD_LONG_STOP_SEQUENCE) {
                const int P = long_pos(u, o);
                if (P < 448) o_v = ov[o];
                else if (P < 576) o_v = ov[o] + (f * SWp[P - 448]);
                else o_v = ov[o] + f;
            } else {
                o_v = ov[o] + (f * Wp[64 * o + u]);
            }
            if constexpr (kSeq == JAAD_LONG_START_SEQUENCE) {
                const int P = long_pos(u, o);
                if (P < 448) n_v = g;
                else if (P < 576) n_v = g * SWc[127 - (P - 448)];
                else n_v = 0.0f;
            } else {
                n_v = g * Wc[64 * (o ^ 1) + u];
            }
            out[o] = o_v;
            ov[o] = n_v;
        }
    }
}

__device__ __forceinline__ void ola_long(const LdsTables& T, int, const FrameCtx& fc, const float (&re)[8],
                                         const float (&im)[8], float (&ov)[16], float (&out)[16])
{
    if (fc.seq == JAAD_ONLY_LONG_SEQUENCE) ola_long_t<JAAD_ONLY_LONG_SEQUENCE>(T, fc, re, im, ov, out);
    else if (fc.seq == JAAD_LONG_START_SEQUENCE) ola_long_t<JAAD_LONG_START_SEQUENCE>(T, fc, re, im, ov, out);
    else ola_long_t<JAAD_LONG_STOP_SEQUENCE>(T, fc, re, im, ov, out);
}

// ------------------------------------------------------------------------------------------
// EIGHT_SHORT_SEQUENCE: 8 x MDCT(256) (64-point IFFTs), FilterBank.java:71-101.
// Lane (w = u>>3, b = u&7) holds window w's elements b + 8s.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void imdct_short(float* buf, const LdsTables& T, int u, float (&re)[8], float (&im)[8])
{
    const int w = u >> 3, b = u & 7;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        int k = b + 8 * s;
        float in0 = buf[eo_idx(128 * w + 2 * k)];
        float in1 = buf[eo_idx(128 * w + 127 - 2 * k)];
        float c = T.mdct_s[k][0], sn = T.mdct_s[k][1];
        im[s] = (in0 * c) + (in1 * sn);
        re[s] = (in1 * c) - (in0 * sn);
    }
    wave_sync();
    fft_pass1(re, im, T.roots_s, 8);
    float2* X = reinterpret_cast<float2*>(buf);
    const int t = (int)(__builtin_bitreverse32((uint32_t)b) >> 29);
#pragma unroll
    for (int r = 0; r < 8; r++) X[xs(64 * w + 8 * t + r)] = make_float2(re[BR3[r]], im[BR3[r]]);
    wave_sync();
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float2 v = X[xs(64 * w + b + 8 * s)];
        re[s] = v.x;
        im[s] = v.y;
    }
    wave_sync();
    // stages i = 8, 16, 32 of the 64-point IFFT: roots[k*m], m = 4, 2, 1
    fft_3stages(re, im, [&](int j, float& wr, float& wi) {
        int idx = j == 0 ? 4 * b : (j < 3 ? 2 * (b + 8 * (j - 1)) : b + 8 * (j - 3));
        wr = T.roots_s[idx][0];
        wi = T.roots_s[idx][1];
    });
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

// Overlap-add of the 8 short windows in Java's evaluation order (FilterBank.java:76-100):
// out = (ov + A) + B and new overlap = A + B, where A is window m-1's windowed falling half and
// B window m's windowed rising half at the same time index.  Two LDS phases: all falling halves
// (A terms) are written and gathered per owned position, then all rising halves (B terms).
__device__ __forceinline__ void ola_short(float* Tb, const LdsTables& T, int u, const FrameCtx& fc,
                                          const float (&re)[8], const float (&im)[8], float (&ov)[16],
                                          float (&out)[16])
{
    const int w = u >> 3, b = u & 7;
    const float* SWc = T.win_short[fc.shape];
    const float* SWr = T.win_short[w == 0 ? fc.shape_prev : fc.shape];
    float nv[16];
#pragma unroll
    for (int phase = 0; phase < 2; phase++) {  // 0: falling halves (A), 1: rising halves (B)
#pragma unroll
        for (int s = 0; s < 8; s++) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                int n;
                float v;
                short_slot(b, s, j, re, im, n, v);
                if ((n < 128) != (phase == 1)) continue;  // j = 0,1 rising; j = 2,3 falling (compile-time)
                if (phase == 0) Tb[128 * w + (n - 128)] = v * SWc[255 - n];
                else Tb[128 * w + n] = v * SWr[n];
            }
        }
        wave_sync();
        const int uu = lane_id();  // opaque: stop index math being hoisted/kept across phases
#pragma unroll
        for (int o = 0; o < 16; o++) {
            const int P = long_pos(uu, o);
            // output sample t = P: window m = (P-448)>>7, offset i; overlap sample t = 1024+P
            const int mo = (P - 448) >> 7, io = (P - 448) & 127;
            const int mq = (P + 576) >> 7, iq = (P + 576) & 127;
            if (phase == 0) {
                out[o] = (P >= 448 + 128) ? ov[o] + Tb[128 * (mo - 1) + io] : ov[o];
                nv[o] = (mq <= 8) ? Tb[128 * (mq - 1) + iq] : 0.0f;
            } else {
                if (P >= 448) out[o] = out[o] + Tb[128 * mo + io];
                if (mq <= 7) nv[o] = nv[o] + Tb[128 * mq + iq];
            }
        }
        wave_sync();
    }
#pragma unroll
    for (int o = 0; o < 16; o++) ov[o] = nv[o];
}

// ------------------------------------------------------------------------------------------
// TNS, spec mode (ISO/IEC 14496-3 4.6.9.3), in place on the spectrum; one lane per filter.
// The reference parses TNS (A/tools/TNS.java:35-61) but its process() is a no-op.
// ------------------------------------------------------------------------------------------
__device__ void tns_spec(float* buf, float* scratch, const LdsTables& T, const GlobalTables& G, int u,
                         const Ics& info, const jaad_tns* tp)
{
    const bool is_short = info.seq == JAAD_EIGHT_SHORT_SEQUENCE;
    const int nswb = is_short ? T.nswb_s : T.nswb_l;
    const int16_t* offs = is_short ? G.swb_s : G.swb_l;
    const int tns_max = is_short ? T.tns_max_s : T.tns_max_l;
    const int nf = tp->n_filters;
    if (u < nf && u < 8) {
        const jaad_tns_filter& F = tp->filt[u];
        int top = nswb, bottom = nswb;
        for (int f = 0; f <= u; f++) {  // walk this window's filters parsed before this one
            const jaad_tns_filter& G = tp->filt[f];
            if (G.window != F.window) continue;
            top = bottom;
            bottom = top - G.length;
            if (bottom < 0) bottom = 0;
        }
        const int order = F.order > 20 ? 20 : F.order;
        float* a = scratch + 24 * u;  // a[0..20]
        float bb[21];
        const float* tab = G.tns_coef[2 * ((F.flags >> 2) & 1) + ((F.flags >> 1) & 1)];
        a[0] = 1.0f;
        for (int m = 1; m <= order; m++) {
            float tm = -tab[F.coef[m - 1] & 15];
            for (int i = 1; i < m; i++) bb[i] = a[i] + tm * a[m - i];
            for (int i = 1; i < m; i++) a[i] = bb[i];
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
            const int base = (is_short ? 128 * F.window : 0) + start;
            for (int n = 0; n < size; n++) {
                float y = buf[eo_idx(base + n * inc)];
                for (int j = 0; j < order; j++) {
                    float st = (n - 1 - j >= 0) ? buf[eo_idx(base + (n - 1 - j) * inc)] : 0.0f;
                    y -= st * a[j + 1];
                }
                buf[eo_idx(base + n * inc)] = y;
            }
        }
    }
    wave_sync();
}

// ------------------------------------------------------------------------------------------
// PNS slow path (ICStream.java:241-257): lane 0 replays the static LCG in parse order.
// ------------------------------------------------------------------------------------------
__device__ void pns_fill(float* buf, const PairBands& pb, int bc, const GlobalTables& G, int u, const Ics& info)
{
    if (u == 0) {
        const bool is_short = info.seq == JAAD_EIGHT_SHORT_SEQUENCE;
        const int16_t* offs = is_short ? G.swb_s : G.swb_l;
        int glen[8], ng = 1;
        glen[0] = 1;
        if (is_short)
            for (int i = 0; i < 7; i++) {
                if (info.grouping & (1u << i)) glen[ng - 1]++;
                else glen[ng++] = 1;
            }
        uint32_t rs = info.pns;
        const int maxSFB = info.max_sfb;
        for (int g = 0, idx = 0, groupOff = 0; g < ng; g++) {
            for (int sfb = 0; sfb < maxSFB; sfb++, idx++) {
                if (pb.cb[bc][idx] != JAAD_NOISE_HCB) continue;
                int off = groupOff + offs[sfb];
                int width = offs[sfb + 1] - offs[sfb];
                float sfv = pb.gain[bc][idx];
                for (int w = 0; w < glen[g]; w++, off += 128) {
                    float energy = 0.0f;
                    for (int k = 0; k < width; k++) {
                        rs = 1664525u * rs + 1013904223u;
                        float v = (float)(int32_t)rs;
                        buf[eo_idx(off + k)] = v;
                        energy += v * v;
                    }
                    float scale = (float)((double)sfv / sqrt((double)energy));
                    for (int k = 0; k < width; k++) buf[eo_idx(off + k)] *= scale;
                }
            }
            groupOff += glen[g] << 7;
        }
    }
    wave_sync();
}

// band index (g*max_sfb + sfb) of the bin quad starting at position p (4-aligned), or -1
__device__ __forceinline__ int band_of(const LdsTables& T, const Ics& info, int p)
{
    int sfb, g = 0;
    if (info.seq == JAAD_EIGHT_SHORT_SEQUENCE) {
        int w = p >> 7;
        sfb = T.quad2band_s[(p & 127) >> 2];
        g = w - __builtin_popcount(info.grouping & ((1u << w) - 1u));
    } else {
        sfb = T.quad2band_l[p >> 2];
    }
    if (sfb >= info.max_sfb) return -1;
    return g * info.max_sfb + sfb;
}

// lane u's 16 spectral bins p = 8u + 512h + i (h = 0,1; i = 0..7) <-> buf (E/O layout), as
// four float4 accesses (bins 8u+512h+{0,2,4,6} and {1,3,5,7})
__device__ __forceinline__ void store_spec(float* buf, int u, const float (&x)[16])
{
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int p = 8 * u + 512 * h;
        *reinterpret_cast<float4*>(&buf[eo_idx(p)]) = make_float4(x[8 * h], x[8 * h + 2], x[8 * h + 4], x[8 * h + 6]);
        *reinterpret_cast<float4*>(&buf[eo_idx(p + 1)]) =
            make_float4(x[8 * h + 1], x[8 * h + 3], x[8 * h + 5], x[8 * h + 7]);
    }
}
__device__ __forceinline__ void load_spec(const float* buf, int u, float (&x)[16])
{
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int p = 8 * u + 512 * h;
        float4 e = *reinterpret_cast<const float4*>(&buf[eo_idx(p)]);
        float4 o = *reinterpret_cast<const float4*>(&buf[eo_idx(p + 1)]);
        x[8 * h + 0] = e.x; x[8 * h + 2] = e.y; x[8 * h + 4] = e.z; x[8 * h + 6] = e.w;
        x[8 * h + 1] = o.x; x[8 * h + 3] = o.y; x[8 * h + 5] = o.z; x[8 * h + 7] = o.w;
    }
}

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

struct Prefetch {
    v4i q[2];       // own channel bins 8u+512h .. +7
    uint32_t sfcb;  // lane u < 32: sf bytes 4u..4u+3; lane u >= 32: cb bytes 4(u-32)..
    uint32_t side;  // lane i < 4*nch: dword i of the frame's jaad_ics_info records;
                    // lanes 8..11: the frame's ms_used words (read back with readlane)
};

// Everything frame f needs from HBM, loaded one frame ahead with vector loads (vmcnt is in
// order; scalar loads would share lgkmcnt with the LDS traffic and could not be hidden).
__device__ __forceinline__ void prefetch(const KernelArgs& A, int f, int nch, int c, int u, Prefetch& pf)
{
    const size_t cf = (size_t)f * nch + c;
    const v4i* q = reinterpret_cast<const v4i*>(A.q + cf * 1024);
    pf.q[0] = __builtin_nontemporal_load(q + u);
    pf.q[1] = __builtin_nontemporal_load(q + 64 + u);
    const uint32_t* row = reinterpret_cast<const uint32_t*>(u < 32 ? A.sf + cf * 128 : A.cb + cf * 128);
    pf.sfcb = row[u & 31];
    const uint32_t* side = u < 8 ? reinterpret_cast<const uint32_t*>(A.ics + (size_t)f * nch) + (u < 4 * nch ? u : 0)
                                 : (A.ms_used ? reinterpret_cast<const uint32_t*>(A.ms_used + (size_t)f * 2) + (u & 3)
                                              : reinterpret_cast<const uint32_t*>(A.ics));
    pf.side = *side;
}

__device__ __forceinline__ Ics ics_from_lanes(uint32_t side, int base)
{
    const uint32_t a = __builtin_amdgcn_readlane(side, base);
    const uint32_t b = __builtin_amdgcn_readlane(side, base + 1);
    Ics r;
    r.seq = a & 0xff;
    r.shape = (a >> 8) & 0xff;
    r.shape_prev = (a >> 16) & 0xff;
    r.max_sfb = a >> 24;
    r.grouping = b & 0xff;
    r.flags = (b >> 8) & 0xff;
    r.pns = __builtin_amdgcn_readlane(side, base + 2);
    return r;
}

template <bool kTnsSpec, int kOut>
__global__ __launch_bounds__(kWGThreads, kTnsSpec ? 2 : JAAD_WAVES_PER_EU) void lc_decode_kernel(KernelArgs A)
{
    __shared__ LdsTables T;
    __shared__ float Wb[kWavesPerWG][kWaveBuf];
    __shared__ PairBands PB[kWavesPerWG / 2];

    {
        const uint4* src = reinterpret_cast<const uint4*>(A.tables);
        uint4* dst = reinterpret_cast<uint4*>(&T);
        for (int i = threadIdx.x; i < (int)(sizeof(LdsTables) / 16); i += kWGThreads) dst[i] = src[i];
    }
    __syncthreads();

    constexpr bool big_endian = !(kOut & JAAD_PCM_LITTLE_ENDIAN);
    constexpr bool planar = kOut == (int)kOutPlanarF32;
    constexpr bool out_f32 = (kOut & JAAD_PCM_FLOAT32) != 0 || planar;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    STAMP(0);
    const bool stereo = A.nch == 2;
    const int c = stereo ? (wave & 1) : 0;  // channel of this wave
    const int bc = wave & 1;                // channel slot in the PairBands record
    PairBands& pb = PB[wave >> 1];
    float* buf = Wb[wave];
    const int per_wg = stereo ? kWavesPerWG / 2 : kWavesPerWG;
    const int my_idx = stereo ? (wave >> 1) : wave;
    const int nch = stereo ? 2 : 1;

    for (uint32_t g = blockIdx.x; g * per_wg < A.n_chunks; g += gridDim.x) {
        STAMP(1);
        // iteration count shared by the whole workgroup (barriers must match)
        int n_iter = 0;
        for (int j = 0; j < per_wg; j++) {
            uint32_t cj = g * per_wg + j;
            if (cj < A.n_chunks) {
                uint32_t inf = A.chunks[cj].info;
                int n = (int)(inf & 0xffff) + ((inf & kChunkPrefix) ? 1 : 0);
                n_iter = n > n_iter ? n : n_iter;
            }
        }
        const uint32_t ci = g * per_wg + my_idx;
        ChunkDesc cd{0, 0, 0, 0};
        if (ci < A.n_chunks) cd = A.chunks[ci];
        const int nfr = cd.info & 0xffff;
        const bool prefix = (cd.info & kChunkPrefix) != 0;
        const int my_n = nfr + (prefix ? 1 : 0);
        const int f_first = (int)cd.frame0 - (prefix ? 1 : 0);

        float ov[16];
        {
            const int u = lane_id();
            if (cd.info & kChunkLoadState) {
                const float* st = A.state_in + (size_t)cd.slot * 2048 + 1024 * c;
#pragma unroll
                for (int o = 0; o < 16; o++) ov[o] = st[long_pos(u, o)];
            } else {
#pragma unroll
                for (int o = 0; o < 16; o++) ov[o] = 0.0f;
            }
        }
        // two frames in flight per wave (>= 64 KiB of loads in flight per CU)
        Prefetch pf, pf2;
        if (my_n > 0) prefetch(A, f_first, nch, c, lane_id(), pf);
        if (my_n > 1) prefetch(A, f_first + 1, nch, c, lane_id(), pf2);

        // frame body; pfx holds frame `it`'s inputs and is refilled with frame it+2 (two frames in
        // flight; the loop is unrolled by 2 so the prefetch registers never need copying, which
        // would force a vmcnt(0) drain of every outstanding load and store)
        auto frame = [&](const int it, Prefetch& pfx) {
            if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 0);
            const int u = lane_id();
            const bool active = it < my_n;
            const int f = f_first + it;
            const bool emit = active && f >= (int)cd.frame0;
            const size_t cf0 = (size_t)(active ? f : 0) * nch;
            Ics ic{}, iL{}, iR{};
            bool ms_on = false, is_on = false, xchg = false;
            float x[16];

            // ---------------- phase A: side info, inverse quantisation, PNS ----------------
            if (active) {
                iL = ics_from_lanes(pfx.side, 0);
                iR = stereo ? ics_from_lanes(pfx.side, 4) : iL;
                ic = sel_ics(c != 0, iR, iL);
                ms_on = stereo && (iL.flags & JAAD_ICS_COMMON_WINDOW) && (iL.flags & JAAD_ICS_MS_PRESENT);
                is_on = stereo && (iR.flags & JAAD_ICS_HAS_IS);
                xchg = ms_on || is_on;
#ifdef JAAD_ABL_NO_MS
                xchg = false;
#endif
                // raw sf/cb rows of this channel -> pair record
                reinterpret_cast<uint32_t*>(u < 32 ? pb.sf[bc] : pb.cb[bc])[u & 31] = pfx.sfcb;
                const Prefetch cur = pfx;
#ifdef JAAD_DEBUG_SIDE
                if (A.dbg && ci == 0 && u == 0 && f < 16) {
                    A.dbg[6144 + 32 * f + 8 * c + 0] = (float)ic.seq;
                    A.dbg[6144 + 32 * f + 8 * c + 1] = (float)ic.shape;
                    A.dbg[6144 + 32 * f + 8 * c + 2] = (float)ic.shape_prev;
                    A.dbg[6144 + 32 * f + 8 * c + 3] = (float)ic.max_sfb;
                    A.dbg[6144 + 32 * f + 8 * c + 4] = (float)ic.flags;
                    A.dbg[6144 + 32 * f + 8 * c + 5] = (float)(ic.pns & 0xffff);
                    A.dbg[6144 + 32 * f + 8 * c + 6] = (float)f;
                }
#endif
                if (it + 2 < my_n) prefetch(A, f + 2, nch, c, u, pfx);
                if (stereo && c == 0) {
                    uint64_t m0 = 0, m1 = 0;
                    if (ms_on && A.ms_used) {
                        // readlane returns int: widen through uint32_t (no sign extension)
                        m0 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 8) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 9) << 32);
                        m1 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 10) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 11) << 32);
                    }
                    pb.ms[u] = (uint8_t)((m0 >> u) & 1u);
                    pb.ms[u + 64] = (uint8_t)((m1 >> u) & 1u);
                }
                wave_sync();
                if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 1);
#pragma unroll
                for (int hb = 0; hb < 2; hb++) {
                    const int idx = u + 64 * hb;
                    const uint32_t cbv = pb.cb[bc][idx];
                    const float gv = T.sf_gain[pb.sf[bc][idx]];
                    pb.gain[bc][idx] = cbv == JAAD_NOISE_HCB ? -gv : gv;
                }
                wave_sync();
                // inverse quantisation (ICStream.java:258-271): lane owns bins 8u+512h+i
                if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 2);
                bool esc = false;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int16_t* qv = reinterpret_cast<const int16_t*>(&cur.q[h]);
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int bi = band_of(T, ic, 512 * h + 8 * u + 4 * j);
                        const uint32_t cbv = bi >= 0 ? pb.cb[bc][bi] : 0u;
                        const float gn = bi >= 0 ? pb.gain[bc][bi] : 0.0f;
                        const bool spectral = cbv != JAAD_ZERO_HCB && cbv < JAAD_NOISE_HCB;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const int qq = qv[4 * j + i];
                            const int qc = qq < -128 ? -128 : (qq > 127 ? 127 : qq);
                            esc |= qc != qq;
                            // (q>0 ? IQ[q] : -IQ[-q]) * sf, sign folded into the table
#ifdef JAAD_ABL_NO_IQ
                            const float m = (float)qc * gn;
#else
                            const float m = T.iq_signed[qc + 128] * gn;
#endif
                            x[8 * h + 4 * j + i] = spectral ? m : 0.0f;
                        }
                    }
                }
                if (__ballot(esc)) {  // escape values beyond the LDS head of IQ_TABLE
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int16_t* qv = reinterpret_cast<const int16_t*>(&cur.q[h]);
#pragma unroll
                        for (int j = 0; j < 2; j++) {
                            const int bi = band_of(T, ic, 512 * h + 8 * u + 4 * j);
                            const uint32_t cbv = bi >= 0 ? pb.cb[bc][bi] : 0u;
                            const float gn = bi >= 0 ? pb.gain[bc][bi] : 0.0f;
                            const bool spectral = cbv != JAAD_ZERO_HCB && cbv < JAAD_NOISE_HCB;
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const int qq = qv[4 * j + i];
                                const int aq = qq < 0 ? -qq : qq;
                                if ((qq > 127 || qq < -128) && spectral) {
                                    const float m = A.iq_table[aq > 8190 ? 8190 : aq] * gn;
                                    x[8 * h + 4 * j + i] = qq > 0 ? m : -m;
                                }
                            }
                        }
                    }
                }
                if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 3);
                store_spec(buf, u, x);
                if (ic.flags & JAAD_ICS_HAS_PNS) {
                    wave_sync();
                    pns_fill(buf, pb, bc, *A.gtab, u, ic);
                    load_spec(buf, u, x);
                }
            }
#ifndef JAAD_ABL_NO_BARRIER
            __syncthreads();  // B1
#endif  // both channels' spectra + band records visible to the pair

            if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 4);
            // ---------------- phase C: M/S (MS.java:17-41) and I/S (IS.java:17-53) ----------------
            if (active && xchg) {
                float xp[16];
                load_spec(Wb[wave ^ 1], u, xp);
#pragma unroll
                for (int h = 0; h < 2; h++) {
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int p = 512 * h + 8 * u + 4 * j;
                        if (ms_on) {
                            const int bi = band_of(T, iL, p);
                            if (bi >= 0 && pb.ms[bi] && pb.cb[0][bi] < JAAD_NOISE_HCB && pb.cb[1][bi] < JAAD_NOISE_HCB) {
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    const int e = 8 * h + 4 * j + i;
                                    // t = L - R; L += R; R = t
                                    x[e] = c == 0 ? x[e] + xp[e] : xp[e] - x[e];
                                }
                            }
                        }
                        if (is_on && c == 1) {
                            const int bi = band_of(T, iR, p);
                            const uint32_t cbr = bi >= 0 ? pb.cb[1][bi] : 0u;
                            if (cbr == JAAD_INTENSITY_HCB || cbr == JAAD_INTENSITY_HCB2) {
                                int cs = cbr == JAAD_INTENSITY_HCB ? 1 : -1;
                                if (iL.flags & JAAD_ICS_MS_PRESENT) cs *= pb.ms[bi] ? -1 : 1;
                                const float scale = (float)cs * pb.gain[1][bi];
#pragma unroll
                                for (int i = 0; i < 4; i++) x[8 * h + 4 * j + i] = xp[8 * h + 4 * j + i] * scale;
                            }
                        }
                    }
                }
            }
            if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 5);
#ifndef JAAD_ABL_NO_BARRIER
            __syncthreads();  // B2
#endif  // the partner has read this wave's spectrum

            if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 6);
            // ---------------- phase D: (TNS) -> IMDCT -> window/OLA -> PCM into LDS ----------------
            if (active) {
                if (xchg) store_spec(buf, u, x);
                wave_sync();
                const bool dump = A.dbg && ci == 0 && f == A.dbg_frame;
                if (dump)
                    for (int i = 0; i < 16; i++) {
                        const int p = 8 * u + 512 * (i >> 3) + (i & 7);
                        A.dbg[1024 * c + p] = buf[eo_idx(p)];
                    }
                if (kTnsSpec && A.tns_mode == JAAD_TNS_SPEC && (ic.flags & JAAD_ICS_TNS) && A.tns)
                    tns_spec(buf, &pb.gain[bc][0], T, *A.gtab, u, ic, A.tns + cf0 + c);
                FrameCtx fc{ic.seq, ic.shape, ic.shape_prev};
                float re[8], im[8], out[16];
#ifdef JAAD_ABL_NO_IMDCT
                if (true) {
#pragma unroll
                    for (int o = 0; o < 16; o++) { out[o] = buf[o * 64 + u] + ov[o]; ov[o] = out[o] * 0.5f; }
                } else
#endif
                if (fc.seq == JAAD_EIGHT_SHORT_SEQUENCE) {
                    imdct_short(buf, T, u, re, im);
                    ola_short(buf, T, u, fc, re, im, ov, out);
                } else {
                    imdct_long(buf, T, u, re, im);
                    if (dump)
                        for (int s2 = 0; s2 < 8; s2++) {
                            A.dbg[2048 + 1024 * c + 2 * (u + 64 * s2)] = re[s2];
                            A.dbg[2048 + 1024 * c + 2 * (u + 64 * s2) + 1] = im[s2];
                        }
                    ola_long(T, u, fc, re, im, ov, out);
                }
                wave_sync();
                if (dump)
                    for (int o = 0; o < 16; o++) A.dbg[4096 + 1024 * c + long_pos(u, o)] = out[o];
#ifdef JAAD_ABL_NO_PCMLDS
                if (emit && A.n_chunks == 0) {
#else
                if (emit) {
#endif
#pragma unroll
                    for (int o = 0; o < 16; o++) {
                        const int P = long_pos(u, o);
                        if constexpr (out_f32) buf[P] = out[o];
                        else reinterpret_cast<int16_t*>(buf)[P] = (int16_t)java_round16(out[o]);
                    }
                }
            }
#ifndef JAAD_ABL_NO_BARRIER
            __syncthreads();  // B3
#endif  // PCM of both channels in LDS

            if (it >= 4 && it < 7) STAMP(2 + 9 * (it - 4) + 7);
            // ---------------- phase E: interleave + store (stereo: wave c stores samples [512c, 512c+512)) ----
#ifndef JAAD_ABL_NO_STORE
            if (emit) {
#else
            if (emit && A.n_chunks == 0) {
#endif
                const float* bL = stereo ? Wb[wave & ~1] : buf;
                const float* bR = stereo ? Wb[wave | 1] : buf;
                const int nj = stereo ? 2 : 4;
                if constexpr (planar) {  // this wave's channel, time order, for the SBR kernel
                    float* dst = reinterpret_cast<float*>(A.pcm) + ((size_t)f * nch + c) * 1024;
#pragma unroll
                    for (int jj = 0; jj < 4; jj++) {
                        const int p = 4 * u + 256 * jj;
                        *reinterpret_cast<float4*>(dst + p) = *reinterpret_cast<const float4*>(buf + p);
                    }
                } else
                for (int jj = 0; jj < nj; jj++) {
                    const int j = stereo ? 2 * c + jj : jj;
                    const int p = 4 * u + 256 * j;  // samples p..p+3
                    if constexpr (out_f32) {
                        float4 l = *reinterpret_cast<const float4*>(bL + p);
                        float4 r = *reinterpret_cast<const float4*>(bR + p);
                        float4* dst = reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(A.pcm) + (size_t)f * 8192 + 8 * p);
                        dst[0] = make_float4(l.x, r.x, l.y, r.y);
                        dst[1] = make_float4(l.z, r.z, l.w, r.w);
                    } else {
                        uint2 l = *reinterpret_cast<const uint2*>(reinterpret_cast<const int16_t*>(bL) + p);
                        uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const int16_t*>(bR) + p);
                        // (L_i, R_i) int16 pairs; big endian swaps the two bytes of every sample.
                        // v_perm_b32(s0=r, s1=l): selector bytes 0-3 pick l, 4-7 pick r.
                        const uint32_t sel0 = big_endian ? 0x04050001u : 0x05040100u;
                        const uint32_t sel1 = big_endian ? 0x06070203u : 0x07060302u;
                        v4u o;
                        o.x = __builtin_amdgcn_perm(r.x, l.x, sel0);
                        o.y = __builtin_amdgcn_perm(r.x, l.x, sel1);
                        o.z = __builtin_amdgcn_perm(r.y, l.y, sel0);
                        o.w = __builtin_amdgcn_perm(r.y, l.y, sel1);
                        v4u* dst = reinterpret_cast<v4u*>(reinterpret_cast<uint8_t*>(A.pcm) + (size_t)f * 4096 + 4 * p);
                        __builtin_nontemporal_store(o, dst);
                    }
                }
            }
#ifndef JAAD_ABL_NO_BARRIER
            __syncthreads();  // B4
#endif  // PCM staging buffers may be reused
                };
        for (int it = 0; it < n_iter; it += 2) {
            frame(it, pf);
            if (it + 1 < n_iter) frame(it + 1, pf2);
        }
        STAMP(31);
        if (cd.info & kChunkStoreState) {
            const int u = lane_id();
            float* st = A.state_out + (size_t)cd.slot * 2048 + 1024 * c;
#pragma unroll
            for (int o = 0; o < 16; o++) st[long_pos(u, o)] = ov[o];
        }
    }
}

hipError_t launch_lc(const KernelArgs& a, int grid, hipStream_t stream, bool tns_spec)
{
#define JAAD_LAUNCH(T, O) hipLaunchKernelGGL((lc_decode_kernel<T, O>), dim3(grid), dim3(kWGThreads), 0, stream, a)
    const int o = (a.out_mode == kOutPlanarF32) ? 4 : (a.out_mode & JAAD_PCM_FLOAT32) ? 2 : (a.out_mode & JAAD_PCM_LITTLE_ENDIAN) ? 1 : 0;
    if (o == 4) {
        if (tns_spec) JAAD_LAUNCH(true, kOutPlanarF32);
        else JAAD_LAUNCH(false, kOutPlanarF32);
    } else if (tns_spec) {
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
