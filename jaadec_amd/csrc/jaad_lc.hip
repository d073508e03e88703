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
// Work decomposition.  One wave owns a chunk of consecutive frames of one stream and decodes
// BOTH channels of a CPE itself: lane u holds bins 8u+512h+i (h = 0,1; i = 0..7) of the left
// and the right spectrum in registers, so M/S and I/S are plain register arithmetic and the
// interleaved PCM is assembled in the wave's own LDS area.  Waves never wait for each other
// inside the frame loop (no workgroup barrier after the table prologue), so the VALU, LDS and
// memory phases of the 16 waves of a CU drift apart and overlap.  The 1024-sample IMDCT
// overlap of each channel stays in VGPRs between frames (lane u owns output positions
// {2u+128j} U {1023-2u-128j}); a chunk that does not start its stream re-decodes the previous
// frame to rebuild it.  Frame f+1's inputs are loaded while frame f's two IMDCTs run.
//
// The 512-point complex IFFT of a frame is 8 complex values per lane in three register passes
// (bit-reversed radix-4 + one radix-2 stage, then 3 + 3 radix-2 stages).  Between the passes
// the lanes trade register bits for lane bits with v_permlane32_swap / v_permlane16_swap and
// DPP moves (no LDS round trip).  Butterflies, twiddles (the reference's float32 recurrence tables) and evaluation
// order are those of the Java code and the file is compiled with -ffp-contract=off, so the
// results are bit-exact.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "jaad_lc.h"

namespace jaad {

__device__ __forceinline__ int lane_id()
{
    // opaque to the optimiser: index math derived from it is recomputed where used instead of
    // being hoisted into registers that live across the frame loop
    int v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    __builtin_assume(v >= 0 && v < 64);
    return v;
}

// IFFT output position (mod 64) held by lane u after the register transposes (lane_pos_host)
__device__ __forceinline__ int lane_pos(int u)
{
    return (u >> 3) | ((int)(__builtin_bitreverse32((uint32_t)u) >> 29) << 3);
}

__device__ __forceinline__ void wave_sync()
{
    // LDS traffic of one wave executes in order; this only stops the compiler from moving LDS
    // accesses across the point (lanes of one wave exchange data through LDS).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // and no forwarding of a lane's own LDS stores across the point either: values parked in
    // LDS (e.g. the right spectrum during the left IMDCT) must leave the registers
    asm volatile("" ::: "memory");
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
// long-window IFFT transpose layout: slot = sum of per-bit weights {1,2,4,8,16,33,72,138,276}
// (550 slots).  Additive per bit, so the compile-time index bits of every access fold into the
// instruction offset; the weights were searched (tools/lds_sim.py model of the gfx950 LDS
// lane groups) to leave 16 extra bank cycles over the 32 transpose accesses (i + i/16: 96).
__device__ __forceinline__ int xs_l(int i)
{
    return (i & 31) + ((i >> 5) & 1) * 33 + ((i >> 6) & 1) * 72 + ((i >> 7) & 1) * 138 + ((i >> 8) & 1) * 276;
}

__device__ constexpr int BR3[8] = {0, 4, 2, 6, 1, 5, 3, 7};

// position of IMDCT output slot o = 2s+h for lane u (MDCT.java:56-80 reorder)
__device__ __forceinline__ int long_pos(int u, int o)
{
    int s = o >> 1, h = o & 1, k = lane_pos(u) + 64 * s;
    if (s < 4) return h ? 512 + 2 * k : 511 - 2 * k;
    return h ? 1535 - 2 * k : 2 * k - 512;
}

struct FrameCtx {
    int seq, shape, shape_prev;
};

// jaad_ics_info unpacked into wave-uniform scalars
struct Ics {
    int seq, shape, shape_prev, max_sfb, grouping, flags;
    uint32_t pns;
    int nbands;  // number of (group, sfb) bands = groups * max_sfb
};
// The fields are clamped to what the kernel can index safely: jaad_decode_batch rejects out-of-
// range side info on the host, jaad_decode_batch_device does not look at it (jaad_gpu.h).
__device__ __forceinline__ Ics ics_from_lanes(uint32_t side, int base, int nswb_l, int nswb_s)
{
    const uint32_t a = __builtin_amdgcn_readlane(side, base);
    const uint32_t b = __builtin_amdgcn_readlane(side, base + 1);
    Ics r;
    r.seq = a & 3;
    r.shape = (a >> 8) & 1;
    r.shape_prev = (a >> 16) & 1;
    const int lim = r.seq == JAAD_EIGHT_SHORT_SEQUENCE ? nswb_s : nswb_l;
    r.max_sfb = min((int)(a >> 24), lim);
    r.grouping = b & 0xff;
    r.flags = (b >> 8) & 0xff;
    r.pns = __builtin_amdgcn_readlane(side, base + 2);
    const int groups = r.seq == JAAD_EIGHT_SHORT_SEQUENCE ? 8 - __builtin_popcount(r.grouping & 0x7f) : 1;
    r.nbands = groups * r.max_sfb;
    return r;
}

// ------------------------------------------------------------------------------------------
// Packed-FP32 form of the long IMDCT (CDNA v_pk_mul_f32 / v_pk_add_f32: two binary32 results
// per lane per instruction, each rounded exactly as the scalar operation).  A complex value is
// one register pair (re, im).  Every Java expression keeps its operands and rounding: a - b is
// evaluated as a + (-b) (identical in IEEE 754, signed zeros included), products keep their
// factors, sums their two operands (addition is commutative).  The half-swaps and negations
// the complex arithmetic needs are VOP3P op_sel / neg modifiers, written as inline asm because
// the compiler does not fold a partial negation.
// ------------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

// (x.y * -w.y, x.x * w.y)
__device__ __forceinline__ f2 pk_mul_swap_nlo(f2 x, f2 w)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1] neg_lo:[0,1]" : "=v"(r) : "v"(x), "v"(w));
    return r;
}
// z = x * w (complex): (x.x*w.x - x.y*w.y, x.x*w.y + x.y*w.x), each product rounded, then one sum
__device__ __forceinline__ f2 cmul(f2 x, f2 w) { return x * w.xx + pk_mul_swap_nlo(x, w); }
// (c.x - d.y, c.y + d.x)
__device__ __forceinline__ f2 pk_rot_p(f2 c, f2 d)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(c), "v"(d));
    return r;
}
// (c.x + d.y, c.y - d.x)
__device__ __forceinline__ f2 pk_rot_m(f2 c, f2 d)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(c), "v"(d));
    return r;
}
// FFT.java:113-130: z = (r1*wr - i1*wi, r1*wi + i1*wr); b = a - z; a = a + z
__device__ __forceinline__ void bfly_pk(f2& a, f2& b, f2 w)
{
    const f2 z = cmul(b, w);
    b = a - z;
    a = a + z;
}
// FFT.java:69-108 (inverse)
__device__ __forceinline__ void radix4_pk(f2& c0, f2& c1, f2& c2, f2& c3)
{
    const f2 a = c0 + c1, b = c2 + c3, c = c0 - c1, d = c2 - c3;
    c0 = a + b;
    c2 = a - b;
    c1 = pk_rot_p(c, d);
    c3 = pk_rot_m(c, d);
}
__device__ __forceinline__ f2 ld2(const float (&p)[2]) { return *reinterpret_cast<const f2*>(p); }

// ------------------------------------------------------------------------------------------
// +-1 LSB precision (jaad_stream_cfg.precision = JAAD_PRECISION_LSB1, kernel mode 4): the same
// transform, tables and evaluation structure with the complex products fused into v_pk_fma_f32
// (one rounding per multiply-add instead of one per product and one per sum).  A complex
// product is 2 packed operations instead of 3, a twiddled radix-2 butterfly 4 instead of 5 with a
// dependency depth of 2 instead of 3.  BASELINE.json's bar is PCM within +-1 LSB of the reference;
// the reordered roundings move a sample by ~1e-6 relative (tests/test_gpu_precision.py measures the
// off-by-one fraction and asserts max |delta| <= 1 on the full C2 / C3 batches).
// ------------------------------------------------------------------------------------------
// a + b.x * w
__device__ __forceinline__ f2 fma_bx(f2 b, f2 w, f2 a)
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(b), "v"(w), "v"(a));
    return r;
}
// a + b.y * (-w.y, w.x)
__device__ __forceinline__ f2 fma_by(f2 b, f2 w, f2 a)
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(b), "v"(w), "v"(a));
    return r;
}
// a - b.x * w
__device__ __forceinline__ f2 fma_nbx(f2 b, f2 w, f2 a)
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(r) : "v"(b), "v"(w), "v"(a));
    return r;
}
// a - b.y * (-w.y, w.x)
__device__ __forceinline__ f2 fma_nby(f2 b, f2 w, f2 a)
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,1,0] neg_hi:[1,0,0]"
        : "=v"(r) : "v"(b), "v"(w), "v"(a));
    return r;
}
// b.x * w
__device__ __forceinline__ f2 mul_bx(f2 b, f2 w)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(b), "v"(w));
    return r;
}
// x * w (complex): 2 packed operations
__device__ __forceinline__ f2 cmul_fma(f2 x, f2 w) { return fma_by(x, w, mul_bx(x, w)); }

template <bool F>
__device__ __forceinline__ f2 cmul_t(f2 x, f2 w)
{
    if constexpr (F) return cmul_fma(x, w);
    else return cmul(x, w);
}
template <bool F>
__device__ __forceinline__ void bfly_t(f2& a, f2& b, f2 w)
{
    if constexpr (F) {
        const f2 p = fma_bx(b, w, a), m = fma_nbx(b, w, a);
        a = fma_by(b, w, p);
        b = fma_nby(b, w, m);
    } else {
        bfly_pk(a, b, w);
    }
}
template <bool F = false>
__device__ __forceinline__ void fft_pass1_pk(f2 (&c)[8], const float (*w)[2])
{
    radix4_pk(c[BR3[0]], c[BR3[1]], c[BR3[2]], c[BR3[3]]);
    radix4_pk(c[BR3[4]], c[BR3[5]], c[BR3[6]], c[BR3[7]]);
#pragma unroll
    for (int k = 0; k < 4; k++) bfly_t<F>(c[BR3[k]], c[BR3[k + 4]], ld2(w[k]));
}
template <bool F = false, typename TW>
__device__ __forceinline__ void fft_3stages_pk(f2 (&c)[8], TW tw)
{
    {
        const f2 w = tw(0);
#pragma unroll
        for (int s = 0; s < 8; s += 2) bfly_t<F>(c[s], c[s + 1], w);
    }
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const f2 w = tw(1 + e);
        bfly_t<F>(c[e], c[e + 2], w);
        bfly_t<F>(c[4 + e], c[6 + e], w);
    }
#pragma unroll
    for (int s = 0; s < 4; s++) bfly_t<F>(c[s], c[s + 4], tw(3 + s));
}

// The same stages on two channels in lockstep, interleaved operation by operation: each packed
// operation's successor is the other channel's (independent) one, so the one wait state that a
// dependent pair of packed FP32 operations needs is filled with work instead of an s_nop.
__device__ __forceinline__ void bfly_pk2(f2& a0, f2& b0, f2& a1, f2& b1, f2 w)
{
    const f2 m0 = b0 * w.xx, m1 = b1 * w.xx;
    const f2 n0 = pk_mul_swap_nlo(b0, w), n1 = pk_mul_swap_nlo(b1, w);
    const f2 z0 = m0 + n0, z1 = m1 + n1;
    b0 = a0 - z0;
    b1 = a1 - z1;
    a0 = a0 + z0;
    a1 = a1 + z1;
}
// both channels of the lockstep IMDCT, operation by operation
template <bool F>
__device__ __forceinline__ void bfly_t2(f2& a0, f2& b0, f2& a1, f2& b1, f2 w)
{
    if constexpr (F) {
        const f2 p0 = fma_bx(b0, w, a0), p1 = fma_bx(b1, w, a1);
        const f2 m0 = fma_nbx(b0, w, a0), m1 = fma_nbx(b1, w, a1);
        a0 = fma_by(b0, w, p0);
        a1 = fma_by(b1, w, p1);
        b0 = fma_nby(b0, w, m0);
        b1 = fma_nby(b1, w, m1);
    } else {
        bfly_pk2(a0, b0, a1, b1, w);
    }
}
__device__ __forceinline__ void radix4_pk2(f2 (&c)[8], f2 (&d)[8], int i0, int i1, int i2, int i3)
{
    const f2 a0 = c[i0] + c[i1], a1 = d[i0] + d[i1];
    const f2 b0 = c[i2] + c[i3], b1 = d[i2] + d[i3];
    const f2 e0 = c[i0] - c[i1], e1 = d[i0] - d[i1];
    const f2 g0 = c[i2] - c[i3], g1 = d[i2] - d[i3];
    c[i0] = a0 + b0;
    d[i0] = a1 + b1;
    c[i2] = a0 - b0;
    d[i2] = a1 - b1;
    c[i1] = pk_rot_p(e0, g0);
    d[i1] = pk_rot_p(e1, g1);
    c[i3] = pk_rot_m(e0, g0);
    d[i3] = pk_rot_m(e1, g1);
}
template <bool F = false>
__device__ __forceinline__ void fft_pass1_pk2(f2 (&c)[8], f2 (&d)[8], const float (*w)[2])
{
    radix4_pk2(c, d, BR3[0], BR3[1], BR3[2], BR3[3]);
    radix4_pk2(c, d, BR3[4], BR3[5], BR3[6], BR3[7]);
#pragma unroll
    for (int k = 0; k < 4; k++) bfly_t2<F>(c[BR3[k]], c[BR3[k + 4]], d[BR3[k]], d[BR3[k + 4]], ld2(w[k]));
}
template <bool F = false, typename TW>
__device__ __forceinline__ void fft_3stages_pk2(f2 (&c)[8], f2 (&d)[8], TW tw)
{
    {
        const f2 w = tw(0);
#pragma unroll
        for (int s = 0; s < 8; s += 2) bfly_t2<F>(c[s], c[s + 1], d[s], d[s + 1], w);
    }
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const f2 w = tw(1 + e);
        bfly_t2<F>(c[e], c[e + 2], d[e], d[e + 2], w);
        bfly_t2<F>(c[4 + e], c[6 + e], d[4 + e], d[6 + e], w);
    }
#pragma unroll
    for (int s = 0; s < 4; s++) bfly_t2<F>(c[s], c[s + 4], d[s], d[s + 4], tw(3 + s));
}

// ---- +-1 LSB kernel: the IFFT's 8-point stages with their trivial twiddles exact ----
// The reference's stage twiddles are FFT_TABLE_512 entries throughout (FFT.java:113-130); the fused
// kernel multiplies by 1, i, W8 = sqrt(1/2) (1 + i) and W8^3 exactly (their table values differ
// from these by <= 2.4e-6), so a butterfly by 1 or i is two packed additions and one by W8 or W8^3
// three packed operations.  Passes 2 and 3 become radix-8 butterflies: register r first takes
// the twiddle of its sub-transform (LdsTables::tw2f / tw3f), then one 8-point DFT -- the same
// transform as the three radix-2 stages (checked against them in float64 when this was written),
// with 26 + 14 packed operations per pass instead of 48.
__device__ __forceinline__ f2 pkfma(f2 a, f2 b, f2 c)  // a * b + c
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ f2 pkfma_n(f2 a, f2 b, f2 c)  // -a * b + c
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ f2 pkfma_i(f2 a, f2 b, f2 c)  // (i a) * b + c = (-a.y, a.x) * b + c
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ f2 pkfma_ni(f2 a, f2 b, f2 c)  // -(i a) * b + c = (a.y, -a.x) * b + c
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ f2 sqrt_half2() { return f2{0.70710678118654752f, 0.70710678118654752f}; }
// a, b = a + b, a - b
__device__ __forceinline__ void bf1(f2& a, f2& b)
{
    const f2 t = a;
    a = t + b;
    b = t - b;
}
// a, b = a + i b, a - i b
__device__ __forceinline__ void bfi(f2& a, f2& b)
{
    const f2 t = a;
    a = pk_rot_p(t, b);
    b = pk_rot_m(t, b);
}
// a, b = a + W8 b, a - W8 b   (W8 b = sqrt(1/2) u, u = (1 + i) b)
__device__ __forceinline__ void bf8(f2& a, f2& b, f2 h)
{
    const f2 u = pk_rot_p(b, b), t = a;
    a = pkfma(u, h, t);
    b = pkfma_n(u, h, t);
}
// a, b = a + W8^3 b, a - W8^3 b   (W8^3 b = sqrt(1/2) i u)
__device__ __forceinline__ void bf83(f2& a, f2& b, f2 h)
{
    const f2 u = pk_rot_p(b, b), t = a;
    a = pkfma_i(u, h, t);
    b = pkfma_ni(u, h, t);
}
// Two independent complex products / W8 butterflies interleaved: the second one's first operation
// fills the wait state that a packed FP32 result needs before a dependent packed operation reads it
// (the compiler keeps the inline-asm order it is given and would put an s_nop between).
__device__ __forceinline__ void cmul_fma2(f2& a, f2 wa, f2& b, f2 wb)
{
    const f2 ma = mul_bx(a, wa), mb = mul_bx(b, wb);
    a = fma_by(a, wa, ma);
    b = fma_by(b, wb, mb);
}
__device__ __forceinline__ void bf8_2(f2& a0, f2& b0, f2& a1, f2& b1, f2 h)
{
    const f2 u0 = pk_rot_p(b0, b0), u1 = pk_rot_p(b1, b1), t0 = a0, t1 = a1;
    a0 = pkfma(u0, h, t0);
    a1 = pkfma(u1, h, t1);
    b0 = pkfma_n(u0, h, t0);
    b1 = pkfma_n(u1, h, t1);
}
__device__ __forceinline__ void bf83_2(f2& a0, f2& b0, f2& a1, f2& b1, f2 h)
{
    const f2 u0 = pk_rot_p(b0, b0), u1 = pk_rot_p(b1, b1), t0 = a0, t1 = a1;
    a0 = pkfma_i(u0, h, t0);
    a1 = pkfma_i(u1, h, t1);
    b0 = pkfma_ni(u0, h, t0);
    b1 = pkfma_ni(u1, h, t1);
}
// 8-point DFT of registers holding the sub-transforms in bit-reversed order (fft_3stages_pk's
// structure with twiddles 1 | 1, i | 1, W8, i, W8^3), N channels operation by operation
template <int N>
__device__ __forceinline__ void dft8_r8(f2 (&c)[N][8])
{
    const f2 h = sqrt_half2();
#pragma unroll
    for (int s = 0; s < 8; s += 2)
#pragma unroll
        for (int n = 0; n < N; n++) bf1(c[n][s], c[n][s + 1]);
#pragma unroll
    for (int n = 0; n < N; n++) {
        bf1(c[n][0], c[n][2]);
        bf1(c[n][4], c[n][6]);
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
        bfi(c[n][1], c[n][3]);
        bfi(c[n][5], c[n][7]);
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
        bf1(c[n][0], c[n][4]);
        bfi(c[n][2], c[n][6]);
    }
    if constexpr (N == 2) {
        bf8_2(c[0][1], c[0][5], c[1][1], c[1][5], h);
        bf83_2(c[0][3], c[0][7], c[1][3], c[1][7], h);
    } else {
        const f2 u1 = pk_rot_p(c[0][5], c[0][5]), u3 = pk_rot_p(c[0][7], c[0][7]), t1 = c[0][1], t3 = c[0][3];
        c[0][1] = pkfma(u1, h, t1);
        c[0][3] = pkfma_i(u3, h, t3);
        c[0][5] = pkfma_n(u1, h, t1);
        c[0][7] = pkfma_ni(u3, h, t3);
    }
}
// pass 1 (FFT.java:69-108 radix-4, then the 8-point stage with twiddles W8^k, k = 0..3)
template <int N>
__device__ __forceinline__ void fft_pass1_r8(f2 (&c)[N][8])
{
    const f2 h = sqrt_half2();
#pragma unroll
    for (int n = 0; n < N; n++) {
        radix4_pk(c[n][BR3[0]], c[n][BR3[1]], c[n][BR3[2]], c[n][BR3[3]]);
        radix4_pk(c[n][BR3[4]], c[n][BR3[5]], c[n][BR3[6]], c[n][BR3[7]]);
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
        bf1(c[n][BR3[0]], c[n][BR3[4]]);
        bfi(c[n][BR3[2]], c[n][BR3[6]]);
    }
    if constexpr (N == 2) {
        bf8_2(c[0][BR3[1]], c[0][BR3[5]], c[1][BR3[1]], c[1][BR3[5]], h);
        bf83_2(c[0][BR3[3]], c[0][BR3[7]], c[1][BR3[3]], c[1][BR3[7]], h);
    } else {
        const f2 u1 = pk_rot_p(c[0][BR3[5]], c[0][BR3[5]]), u3 = pk_rot_p(c[0][BR3[7]], c[0][BR3[7]]);
        const f2 t1 = c[0][BR3[1]], t3 = c[0][BR3[3]];
        c[0][BR3[1]] = pkfma(u1, h, t1);
        c[0][BR3[3]] = pkfma_i(u3, h, t3);
        c[0][BR3[5]] = pkfma_n(u1, h, t1);
        c[0][BR3[7]] = pkfma_ni(u3, h, t3);
    }
}
// passes 2 and 3: register r (1..7) times tw(r - 1), then the 8-point DFT
template <int N, typename TW>
__device__ __forceinline__ void fft_pass_r8(f2 (&c)[N][8], TW tw)
{
    if constexpr (N == 2) {
#pragma unroll
        for (int r = 1; r < 8; r++) {
            const f2 w = tw(r - 1);
            cmul_fma2(c[0][r], w, c[1][r], w);
        }
    } else {
#pragma unroll
        for (int r = 1; r < 7; r += 2) cmul_fma2(c[0][r], tw(r - 1), c[0][r + 1], tw(r));
        c[0][7] = cmul_fma(c[0][7], tw(6));
    }
    dft8_r8<N>(c);
}



// Register transposes between the IFFT passes.  A pair of registers (a: register bit i clear,
// b: set) trades register bit i for lane bit L: the element at (register bit, lane bit L) =
// (x, y) moves to (y, x), every other lane bit unchanged.
// Lane bits 5 / 4: one v_permlane32_swap / v_permlane16_swap swaps a's upper half-lanes with
// b's lower ones.
template <int L>
__device__ __forceinline__ void xch_hi(float& a, float& b)
{
    static_assert(L == 5 || L == 4, "lane bits 0..3 go through xch2");
    const int ia = __float_as_int(a), ib = __float_as_int(b);
    const auto r = L == 5 ? __builtin_amdgcn_permlane32_swap(ia, ib, false, false)
                          : __builtin_amdgcn_permlane16_swap(ia, ib, false, false);
    a = __int_as_float(r[0]);
    b = __int_as_float(r[1]);
}
// Lane bits 0..3 for two register pairs (a0, b0) and (a1, b1) at once:
//   a' = bit clear ? a : b(partner),  b' = bit set ? b : a(partner).
// Each output is one VOP2 v_cndmask_b32_dpp: src0 read through the swizzle (quad_perm for lane
// bits 0, 1; row_ror:4 / row_ror:12 for bit 2, row_ror:8 for bit 3), VCC = the lanes that keep
// their own value, set by two s_mov_b32 of a literal (which also give the 2 wait states a DPP
// read of a freshly written VGPR needs).  Round 4 measured the alternative without VCC (DPP
// moves under bank masks for bits 2, 3; DPP moves + v_cndmask_b32_e64 on an SGPR-pair mask for
// bits 0, 1; measured and removed): an instruction micro-benchmark prices the VOP2 select at ~13.9
// SIMD cycles against 3.3-3.6 for the other forms (tools/valu_rate.hip,
// profiles/round4_valu_rate.txt), yet inside this kernel the VCC form is 1-2 % faster per C2
// batch (same-call A/B over 30 launches, profiles/round4_xch_ab.txt) -- the exchanges are not
// issue-bound here, and the VCC form needs fewer instructions and temporaries.
template <int L>
__device__ __forceinline__ void xch2(f2& a0, f2& b0, f2& a1, f2& b1)
{
    // lanes with bit L set (the pattern repeats per 32 lanes: vcc_lo = vcc_hi, literal operands,
    // no SGPRs held across the exchanges)
    constexpr uint32_t kHi = L == 0 ? 0xAAAAAAAAu : L == 1 ? 0xCCCCCCCCu : L == 2 ? 0xF0F0F0F0u : 0xFF00FF00u;
    f2 na0, nb0, na1, nb1;
#define JAAD_XCH_BODY(QA, QB)                                                                    \
    asm("s_mov_b32 vcc_lo, %[lo]\n\t"                                                            \
        "s_mov_b32 vcc_hi, %[lo]\n\t"                                                            \
        "v_cndmask_b32_dpp %[na0x], %[b0x], %[a0x], vcc " QA " row_mask:0xf bank_mask:0xf\n\t"   \
        "v_cndmask_b32_dpp %[na0y], %[b0y], %[a0y], vcc " QA " row_mask:0xf bank_mask:0xf\n\t"   \
        "v_cndmask_b32_dpp %[na1x], %[b1x], %[a1x], vcc " QA " row_mask:0xf bank_mask:0xf\n\t"   \
        "v_cndmask_b32_dpp %[na1y], %[b1y], %[a1y], vcc " QA " row_mask:0xf bank_mask:0xf\n\t"   \
        "s_mov_b32 vcc_lo, %[hi]\n\t"                                                            \
        "s_mov_b32 vcc_hi, %[hi]\n\t"                                                            \
        "v_cndmask_b32_dpp %[nb0x], %[a0x], %[b0x], vcc " QB " row_mask:0xf bank_mask:0xf\n\t"   \
        "v_cndmask_b32_dpp %[nb0y], %[a0y], %[b0y], vcc " QB " row_mask:0xf bank_mask:0xf\n\t"   \
        "v_cndmask_b32_dpp %[nb1x], %[a1x], %[b1x], vcc " QB " row_mask:0xf bank_mask:0xf\n\t"   \
        "v_cndmask_b32_dpp %[nb1y], %[a1y], %[b1y], vcc " QB " row_mask:0xf bank_mask:0xf"       \
        : [na0x] "=&v"(na0.x), [na0y] "=&v"(na0.y), [na1x] "=&v"(na1.x), [na1y] "=&v"(na1.y),     \
          [nb0x] "=&v"(nb0.x), [nb0y] "=&v"(nb0.y), [nb1x] "=&v"(nb1.x), [nb1y] "=&v"(nb1.y)      \
        : [a0x] "v"(a0.x), [a0y] "v"(a0.y), [a1x] "v"(a1.x), [a1y] "v"(a1.y), [b0x] "v"(b0.x),    \
          [b0y] "v"(b0.y), [b1x] "v"(b1.x), [b1y] "v"(b1.y), [lo] "i"(~kHi), [hi] "i"(kHi)        \
        : "vcc")
    if constexpr (L == 0) JAAD_XCH_BODY("quad_perm:[1,0,3,2]", "quad_perm:[1,0,3,2]");
    else if constexpr (L == 1) JAAD_XCH_BODY("quad_perm:[2,3,0,1]", "quad_perm:[2,3,0,1]");
    else if constexpr (L == 2) JAAD_XCH_BODY("row_ror:4", "row_ror:12");
    else JAAD_XCH_BODY("row_ror:8", "row_ror:8");
#undef JAAD_XCH_BODY
    a0 = na0;
    b0 = nb0;
    a1 = na1;
    b1 = nb1;
}

// Lane bits 0..3 for 16 register pairs at once (both channels of the lockstep long IMDCT): the
// same selects as xch2, with VCC set twice per 32 selects instead of twice per 8.
//   a'[i] = bit clear ? a[i] : b[i](partner),  b'[i] = bit set ? b[i] : a[i](partner).
template <int L>
__device__ __forceinline__ void xch16(float (&a)[16], float (&b)[16])
{
    constexpr uint32_t kHi = L == 0 ? 0xAAAAAAAAu : L == 1 ? 0xCCCCCCCCu : L == 2 ? 0xF0F0F0F0u : 0xFF00FF00u;
    float na[16], nb[16];
#define JAAD_X16(QA, QB) \
    asm("s_mov_b32 vcc_lo, %[lo]\n\t" \
        "s_mov_b32 vcc_hi, %[lo]\n\t" \
        "v_cndmask_b32_dpp %[na0], %[b0], %[a0], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na1], %[b1], %[a1], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na2], %[b2], %[a2], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na3], %[b3], %[a3], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na4], %[b4], %[a4], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na5], %[b5], %[a5], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na6], %[b6], %[a6], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na7], %[b7], %[a7], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na8], %[b8], %[a8], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na9], %[b9], %[a9], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na10], %[b10], %[a10], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na11], %[b11], %[a11], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na12], %[b12], %[a12], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na13], %[b13], %[a13], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na14], %[b14], %[a14], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[na15], %[b15], %[a15], vcc " QA " row_mask:0xf bank_mask:0xf\n\t" \
        "s_mov_b32 vcc_lo, %[hi]\n\t" \
        "s_mov_b32 vcc_hi, %[hi]\n\t" \
        "v_cndmask_b32_dpp %[nb0], %[a0], %[b0], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb1], %[a1], %[b1], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb2], %[a2], %[b2], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb3], %[a3], %[b3], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb4], %[a4], %[b4], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb5], %[a5], %[b5], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb6], %[a6], %[b6], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb7], %[a7], %[b7], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb8], %[a8], %[b8], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb9], %[a9], %[b9], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb10], %[a10], %[b10], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb11], %[a11], %[b11], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb12], %[a12], %[b12], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb13], %[a13], %[b13], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb14], %[a14], %[b14], vcc " QB " row_mask:0xf bank_mask:0xf\n\t" \
        "v_cndmask_b32_dpp %[nb15], %[a15], %[b15], vcc " QB " row_mask:0xf bank_mask:0xf" \
        : [na0] "=&v"(na[0]), [na1] "=&v"(na[1]), [na2] "=&v"(na[2]), [na3] "=&v"(na[3]), [na4] "=&v"(na[4]), [na5] "=&v"(na[5]), [na6] "=&v"(na[6]), [na7] "=&v"(na[7]), [na8] "=&v"(na[8]), [na9] "=&v"(na[9]), [na10] "=&v"(na[10]), [na11] "=&v"(na[11]), [na12] "=&v"(na[12]), [na13] "=&v"(na[13]), [na14] "=&v"(na[14]), [na15] "=&v"(na[15]), [nb0] "=&v"(nb[0]), [nb1] "=&v"(nb[1]), [nb2] "=&v"(nb[2]), [nb3] "=&v"(nb[3]), [nb4] "=&v"(nb[4]), [nb5] "=&v"(nb[5]), [nb6] "=&v"(nb[6]), [nb7] "=&v"(nb[7]), [nb8] "=&v"(nb[8]), [nb9] "=&v"(nb[9]), [nb10] "=&v"(nb[10]), [nb11] "=&v"(nb[11]), [nb12] "=&v"(nb[12]), [nb13] "=&v"(nb[13]), [nb14] "=&v"(nb[14]), [nb15] "=&v"(nb[15]) \
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [a4] "v"(a[4]), [a5] "v"(a[5]), [a6] "v"(a[6]), [a7] "v"(a[7]), [a8] "v"(a[8]), [a9] "v"(a[9]), [a10] "v"(a[10]), [a11] "v"(a[11]), [a12] "v"(a[12]), [a13] "v"(a[13]), [a14] "v"(a[14]), [a15] "v"(a[15]), [b0] "v"(b[0]), [b1] "v"(b[1]), [b2] "v"(b[2]), [b3] "v"(b[3]), [b4] "v"(b[4]), [b5] "v"(b[5]), [b6] "v"(b[6]), [b7] "v"(b[7]), [b8] "v"(b[8]), [b9] "v"(b[9]), [b10] "v"(b[10]), [b11] "v"(b[11]), [b12] "v"(b[12]), [b13] "v"(b[13]), [b14] "v"(b[14]), [b15] "v"(b[15]), [lo] "i"(~kHi), [hi] "i"(kHi) \
        : "vcc")
    if constexpr (L == 0) JAAD_X16("quad_perm:[1,0,3,2]", "quad_perm:[1,0,3,2]");
    else if constexpr (L == 1) JAAD_X16("quad_perm:[2,3,0,1]", "quad_perm:[2,3,0,1]");
    else if constexpr (L == 2) JAAD_X16("row_ror:4", "row_ror:12");
    else JAAD_X16("row_ror:8", "row_ror:8");
#undef JAAD_X16
#pragma unroll
    for (int i = 0; i < 16; i++) {
        a[i] = na[i];
        b[i] = nb[i];
    }
}

// register bit I <-> lane bit L (<= 3) for both channels of the lockstep long IMDCT
template <int I, int L>
__device__ __forceinline__ void xch_bit_pair(f2 (&c0)[8], f2 (&c1)[8])
{
    static_assert(L <= 3, "lane bits 4, 5 go through xch_hi");
    constexpr int m = 1 << I;
    auto clr = [](int k) { return ((k >> I) << (I + 1)) | (k & (m - 1)); };
    float a[16], b[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        a[4 * k + 0] = c0[clr(k)].x;
        a[4 * k + 1] = c0[clr(k)].y;
        a[4 * k + 2] = c1[clr(k)].x;
        a[4 * k + 3] = c1[clr(k)].y;
        b[4 * k + 0] = c0[clr(k) | m].x;
        b[4 * k + 1] = c0[clr(k) | m].y;
        b[4 * k + 2] = c1[clr(k) | m].x;
        b[4 * k + 3] = c1[clr(k) | m].y;
    }
    xch16<L>(a, b);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        c0[clr(k)] = f2{a[4 * k + 0], a[4 * k + 1]};
        c1[clr(k)] = f2{a[4 * k + 2], a[4 * k + 3]};
        c0[clr(k) | m] = f2{b[4 * k + 0], b[4 * k + 1]};
        c1[clr(k) | m] = f2{b[4 * k + 2], b[4 * k + 3]};
    }
}

// register bit I <-> lane bit L for all four register pairs, both floats of each complex value
template <int I, int L>
__device__ __forceinline__ void xch_bit(f2 (&c)[8], int u)
{
    if constexpr (L <= 3) {
        constexpr int m = 1 << I;
        // k-th register index with bit I clear
        auto clr = [](int k) { return ((k >> I) << (I + 1)) | (k & (m - 1)); };
        xch2<L>(c[clr(0)], c[clr(0) | m], c[clr(1)], c[clr(1) | m]);
        xch2<L>(c[clr(2)], c[clr(2) | m], c[clr(3)], c[clr(3) | m]);
    } else {
#pragma unroll
        for (int s = 0; s < 8; s++) {
            if ((s >> I) & 1) continue;
            float ax = c[s].x, ay = c[s].y, bx = c[s | (1 << I)].x, by = c[s | (1 << I)].y;
            xch_hi<L>(ax, bx);
            xch_hi<L>(ay, by);
            c[s] = f2{ax, ay};
            c[s | (1 << I)] = f2{bx, by};
        }
    }
    (void)u;
}

// IMDCT N = 2048 (MDCT.process, A/filterbank/MDCT.java:36-81) of N channels in lockstep (N = 2:
// the two channels of a CPE share the table reads and give the scheduler two independent
// dependency chains).  Reads the spectrum (E/O layout) from bufs[n]; on return c[n][s] = (re, im)
// of IFFT position lane_pos(u) + 64 s after the post-twiddle.
//
// Element e (0..511) of the bit-reversed IFFT array: pass 1 works on e bits 0-2, pass 2 on bits
// 3-5, pass 3 on bits 6-8 (FFT.java:69-134), each as three in-register stages.  Lane u starts
// with k = u + 64 s (e = bitrev9(k): e bits 3-8 = bitrev6(u), register s holds e bits 2,1,0 in
// its bits 0,1,2).  The first exchange trades register bits 0,1,2 for lane bits 5,4,3 (e bits
// 3,4,5 into registers; lane bits 3-5 then hold e bits 0-2), the second register bits 0,1,2 for
// lane bits 2,1,0 (e bits 6,7,8 into registers), leaving lane u with positions lane_pos(u) + 64 s.
// +-1 LSB kernel: IMDCT output in PCM full-scale units (post-twiddles x 1/32767, LdsTables::
// mdct_post_f / mdct_s_f); the overlap state is converted where it enters and leaves the registers,
// the float outputs where they are stored (JAAD_NO_SCALED: A/B builds with the unscaled tables)
#if defined(JAAD_NO_SCALED)
constexpr bool kScaledOut = false;
#else
constexpr bool kScaledOut = true;
#endif
constexpr float kPcmScale = 32767.0f, kPcmUnit = 1.0f / 32767.0f;

template <int N, bool F = false>
__device__ __forceinline__ void imdct_long_pk(float* const (&bufs)[N], const LdsTables& T, int u, f2 (&c)[N][8])
{
    if constexpr (F && N == 2) {  // the two channels' products interleaved (cmul_fma2)
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const int k = u + 64 * s;
            const f2 w = ld2(T.mdct_l[k]);
            c[0][s] = f2{bufs[0][eo_idx(1023 - 2 * k)], bufs[0][eo_idx(2 * k)]};
            c[1][s] = f2{bufs[1][eo_idx(1023 - 2 * k)], bufs[1][eo_idx(2 * k)]};
            cmul_fma2(c[0][s], w, c[1][s], w);
        }
    } else {
#pragma unroll
    for (int n = 0; n < N; n++)
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const int k = u + 64 * s;
            // MDCT.java:39-42: re = in1*c - in0*sn, im = in0*c + in1*sn = cmul((in1, in0), (c, sn))
            const f2 x = {bufs[n][eo_idx(1023 - 2 * k)], bufs[n][eo_idx(2 * k)]};
            c[n][s] = cmul_t<F>(x, ld2(T.mdct_l[k]));
        }
    }
    // (JAAD_ABL_* macros: ablation builds of the fused lockstep path, design tool -- wrong output,
    // time only; scripts/build_exp.py)
#if defined(JAAD_ABL_NOFFT)
    constexpr bool kFft = !(F && N == 2);
#else
    constexpr bool kFft = true;
#endif
#if defined(JAAD_ABL_NODPP)
    constexpr bool kDpp = !(F && N == 2);
#else
    constexpr bool kDpp = kFft;
#endif
#if defined(JAAD_ABL_NOPERM)
    constexpr bool kPerm = !(F && N == 2);
#else
    constexpr bool kPerm = kFft;
#endif
#if defined(JAAD_NO_R8)  // (A/B builds: the fused kernel with the radix-2 stages)
    constexpr bool kR8 = false;
#else
    constexpr bool kR8 = F;
#endif
    // pass 1: register s holds e bits (s2, s1, s0) = e bits 0, 1, 2 (fft_pass1_pk's BR3 order)
    if constexpr (!kFft) {
    } else if constexpr (kR8) fft_pass1_r8<N>(c);
    else if constexpr (N == 2) fft_pass1_pk2<F>(c[0], c[1], T.tw1);
    else fft_pass1_pk<F>(c[0], T.tw1);
#pragma unroll
    for (int n = 0; n < N; n++) {
        if constexpr (kPerm) {
            xch_bit<0, 5>(c[n], u);  // e bit 3 (lane bit 5) <-> e bit 2
            xch_bit<1, 4>(c[n], u);  // e bit 4 (lane bit 4) <-> e bit 1
        }
        if constexpr (N == 1) xch_bit<2, 3>(c[n], u);  // e bit 5 (lane bit 3) <-> e bit 0
    }
    if constexpr (N == 2 && kDpp) xch_bit_pair<2, 3>(c[0], c[1]);
    // pass 2: register bits 0,1,2 = e bits 3,4,5; e mod 8 = u >> 3
    const int b = u >> 3;
    if constexpr (!kFft) {
    } else if constexpr (kR8) fft_pass_r8<N>(c, [&](int j) { return ld2(T.tw2f[j][b]); });
    else if constexpr (N == 2) fft_3stages_pk2<F>(c[0], c[1], [&](int j) { return ld2(T.tw2[j][b]); });
    else fft_3stages_pk<F>(c[0], [&](int j) { return ld2(T.tw2[j][b]); });
    if constexpr (N == 2) {
        if constexpr (kDpp) {
            xch_bit_pair<0, 2>(c[0], c[1]);  // e bit 6 (lane bit 2) <-> e bit 3
            xch_bit_pair<1, 1>(c[0], c[1]);  // e bit 7 (lane bit 1) <-> e bit 4
            xch_bit_pair<2, 0>(c[0], c[1]);  // e bit 8 (lane bit 0) <-> e bit 5
        }
    } else {
#pragma unroll
        for (int n = 0; n < N; n++) {
            xch_bit<0, 2>(c[n], u);  // e bit 6 (lane bit 2) <-> e bit 3
            xch_bit<1, 1>(c[n], u);  // e bit 7 (lane bit 1) <-> e bit 4
            xch_bit<2, 0>(c[n], u);  // e bit 8 (lane bit 0) <-> e bit 5
        }
    }
    // pass 3: register bits 0,1,2 = e bits 6,7,8, e mod 64 = lane_pos(u)
    if constexpr (!kFft) {
    } else if constexpr (kR8) fft_pass_r8<N>(c, [&](int j) { return ld2(T.tw3f[j][u]); });
    else if constexpr (N == 2) fft_3stages_pk2<F>(c[0], c[1], [&](int j) { return ld2(T.tw3[j][u]); });
    else fft_3stages_pk<F>(c[0], [&](int j) { return ld2(T.tw3[j][u]); });
    // MDCT.java:48-53: re = t0*c - t1*sn, im = t1*c + t0*sn = cmul((t0, t1), (c, sn))
    if constexpr (F && N == 2) {
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const f2 w = ld2(kScaledOut ? T.mdct_post_f[s][u] : T.mdct_post[s][u]);
            cmul_fma2(c[0][s], w, c[1][s], w);
        }
    } else {
#pragma unroll
    for (int s = 0; s < 8; s++)
#pragma unroll
        for (int n = 0; n < N; n++) c[n][s] = cmul_t<F>(c[n][s], ld2(F && kScaledOut ? T.mdct_post_f[s][u] : T.mdct_post[s][u]));
    }
}

// FilterBank.process for ONLY_LONG / LONG_START / LONG_STOP (FilterBank.java:41-70, 102-119).
// Lane u's slot (s,h) holds output position P = long_pos(u, 2s+h); its mirror 1023-P is slot
// (s,1-h) of the same lane, so the falling window W[1023-P] is the other half of the pair.
// Specialised per sequence so the common ONLY_LONG path carries no joint-window logic.
template <int kSeq>
__device__ __forceinline__ void ola_long_t(const LdsTables& T, const FrameCtx& fc, const float (&re)[8],
                                           const float (&im)[8], float (&ov)[16], float (&out)[16])
{
    const int u = lane_id();
    const float* SWp = T.win_short[fc.shape_prev];
    const float* SWc = T.win_short[fc.shape];
    // win_pair[shape][s][u] = {W[pos(u, 2s)], W[pos(u, 2s+1)]}: one 8-byte read per slot pair
    const float2* Wp = reinterpret_cast<const float2*>(&T.win_pair[fc.shape_prev][0][0][0]);
    const float2* Wc = reinterpret_cast<const float2*>(&T.win_pair[fc.shape][0][0][0]);
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float2 wp = make_float2(0.0f, 0.0f), wc = make_float2(0.0f, 0.0f);
        if constexpr (kSeq != JAAD_LONG_STOP_SEQUENCE) wp = Wp[64 * s + u];
        if constexpr (kSeq != JAAD_LONG_START_SEQUENCE) wc = Wc[64 * s + u];
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
                o_v = ov[o] + (f * (h ? wp.y : wp.x));  // rising window W[P]
            }
            if constexpr (kSeq == JAAD_LONG_START_SEQUENCE) {
                const int P = long_pos(u, o);
                if (P < 448) n_v = g;
                else if (P < 576) n_v = g * SWc[127 - (P - 448)];
                else n_v = 0.0f;
            } else {
                n_v = g * (h ? wc.x : wc.y);  // falling window W[1023-P] = slot o^1
            }
            out[o] = o_v;
            ov[o] = n_v;
        }
    }
}

// ONLY_LONG window + overlap-add in packed form (slot pair (2s, 2s+1) of ola_long_t):
//   out[o] = ov[o] + f_o * W[P_o],  new ov[o] = g * W[1023 - P_o]
// with (f_0, f_1, g) = (-re, re, -im) for s < 4 and (im, -im, re) for s >= 4
// (Wp / Wc: the rising and falling windows in win_pair's layout; the +-1 LSB kernel passes
// LdsTables::win_ss for LONG_STOP's rising and LONG_START's falling half)
template <bool F = false>
__device__ __forceinline__ void ola_only_long_pk(const LdsTables& T, const FrameCtx& fc, const f2 (&c)[8],
                                                 float (&ov)[16], float (&out)[16], const f2* Wp = nullptr,
                                                 const f2* Wc = nullptr)
{
    const int u = lane_id();
    if (!Wp) Wp = reinterpret_cast<const f2*>(&T.win_pair[fc.shape_prev][0][0][0]);
    if (!Wc) Wc = reinterpret_cast<const f2*>(&T.win_pair[fc.shape][0][0][0]);
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const f2 wp = Wp[64 * s + u], wc = Wc[64 * s + u];
        f2 fw, nv, o;
        const f2 ovp = f2{ov[2 * s], ov[2 * s + 1]};
        if (s < 4) {
            if constexpr (F)  // o = ov + (-re, re) * wp in one fused operation
                asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
                    : "=v"(o) : "v"(c[s]), "v"(wp), "v"(ovp));
            else
                asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1] neg_lo:[1,0]" : "=v"(fw) : "v"(c[s]), "v"(wp));
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0] neg_hi:[1,0]"
                : "=v"(nv) : "v"(c[s]), "v"(wc));
        } else {
            if constexpr (F)  // o = ov + (im, -im) * wp
                asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1] neg_hi:[1,0,0]"
                    : "=v"(o) : "v"(c[s]), "v"(wp), "v"(ovp));
            else
                asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_hi:[1,0]" : "=v"(fw) : "v"(c[s]), "v"(wp));
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,0]" : "=v"(nv) : "v"(c[s]), "v"(wc));
        }
        if constexpr (!F) o = ovp + fw;
        out[2 * s] = o.x;
        out[2 * s + 1] = o.y;
        ov[2 * s] = nv.x;
        ov[2 * s + 1] = nv.y;
    }
}

template <bool F = false>
__device__ __forceinline__ void ola_long_pk(const LdsTables& T, const FrameCtx& fc, const f2 (&c)[8], float (&ov)[16],
                                            float (&out)[16])
{
    if (fc.seq == JAAD_ONLY_LONG_SEQUENCE) {
        ola_only_long_pk<F>(T, fc, c, ov, out);
        return;
    }
#if !defined(JAAD_NO_WIN_SS)  // (A/B builds: the +-1 LSB kernel with ola_long_t for START / STOP)
    if constexpr (F) {  // one half through win_ss (w * 1 and w * 0 instead of copies and zeros)
        const f2* Wss = reinterpret_cast<const f2*>(
            &T.win_ss[fc.seq == JAAD_LONG_START_SEQUENCE ? fc.shape : fc.shape_prev][0][0][0]);
        if (fc.seq == JAAD_LONG_START_SEQUENCE) ola_only_long_pk<F>(T, fc, c, ov, out, nullptr, Wss);
        else ola_only_long_pk<F>(T, fc, c, ov, out, Wss, nullptr);
        return;
    }
#endif
    float re[8], im[8];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        re[s] = c[s].x;
        im[s] = c[s].y;
    }
    if (fc.seq == JAAD_LONG_START_SEQUENCE) ola_long_t<JAAD_LONG_START_SEQUENCE>(T, fc, re, im, ov, out);
    else ola_long_t<JAAD_LONG_STOP_SEQUENCE>(T, fc, re, im, ov, out);
}


// ------------------------------------------------------------------------------------------
// EIGHT_SHORT_SEQUENCE: 8 x MDCT(256) (64-point IFFTs), FilterBank.java:71-101.
// Lane (w = u>>3, b = u&7) holds window w's elements b + 8s.
// ------------------------------------------------------------------------------------------
// 8 x 64-point IFFTs in packed FP32 (one register pair per complex value, the long path's
// primitives; a - b as a + (-b))
template <bool F = false>
__device__ __forceinline__ void imdct_short_pk(float* buf, const LdsTables& T, int u, float (&re)[8], float (&im)[8])
{
    const int w = u >> 3, b = u & 7;
    f2 c[8];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const int k = b + 8 * s;
        // MDCT.java:39-42: re = in1*c - in0*sn, im = in0*c + in1*sn = cmul((in1, in0), (c, sn))
        const f2 x = {buf[eo_idx(128 * w + 127 - 2 * k)], buf[eo_idx(128 * w + 2 * k)]};
        c[s] = cmul_t<F>(x, ld2(T.mdct_s[k]));
    }
    wave_sync();
    radix4_pk(c[BR3[0]], c[BR3[1]], c[BR3[2]], c[BR3[3]]);
    radix4_pk(c[BR3[4]], c[BR3[5]], c[BR3[6]], c[BR3[7]]);
#pragma unroll
    for (int k = 0; k < 4; k++) bfly_t<F>(c[BR3[k]], c[BR3[k + 4]], ld2(T.roots_s[8 * k]));
    f2* X = reinterpret_cast<f2*>(buf);
    const int t = (int)(__builtin_bitreverse32((uint32_t)b) >> 29);
#pragma unroll
    for (int r = 0; r < 8; r++) X[xs(64 * w + 8 * t + r)] = c[BR3[r]];
    wave_sync();
#pragma unroll
    for (int s = 0; s < 8; s++) c[s] = X[xs(64 * w + b + 8 * s)];
    wave_sync();
    // stages i = 8, 16, 32 of the 64-point IFFT: roots[k*m], m = 4, 2, 1
    fft_3stages_pk<F>(c, [&](int j) {
        const int idx = j == 0 ? 4 * b : (j < 3 ? 2 * (b + 8 * (j - 1)) : b + 8 * (j - 3));
        return ld2(T.roots_s[idx]);
    });
#pragma unroll
    for (int s = 0; s < 8; s++) {
        // MDCT.java:48-53: re = t0*c - t1*sn, im = t1*c + t0*sn = cmul((t0, t1), (c, sn))
        const f2 z = cmul_t<F>(c[s], ld2(F && kScaledOut ? T.mdct_s_f[b + 8 * s] : T.mdct_s[b + 8 * s]));
        re[s] = z.x;
        im[s] = z.y;
    }
}

// imdct_short_pk on both channels of a CPE whose windows are both EIGHT_SHORT, in lockstep as the
// long path runs its two IMDCTs: every LDS phase serves both spectra (one wave_sync each instead of
// one per channel) and the two FFT chains interleave operation by operation, each channel's
// operations those of imdct_short_pk.  Only the mixed-window instantiations (kernel modes 5, 6,
// chosen per launch when the batch holds EIGHT_SHORT frames) carry it: in one kernel body with
// the long path it cost C2's long frames 1-3 % (round 5, profiles/round5_short_pair/).
#if defined(JAAD_SHORT_R2)  // (A/B builds: the +-1 LSB short pair with the radix-2 stages)
constexpr bool kShortR2 = true;
#else
constexpr bool kShortR2 = false;
#endif
template <bool F = false>
__device__ __forceinline__ void imdct_short_pk2(float* bufL, float* bufR, const LdsTables& T, int u, float (&reL)[8],
                                                float (&imL)[8], float (&reR)[8], float (&imR)[8])
{
    const int w = u >> 3, b = u & 7;
    f2 c[2][8];
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const int k = b + 8 * s;
        const f2 tw = ld2(T.mdct_s[k]);
        const f2 x = {bufL[eo_idx(128 * w + 127 - 2 * k)], bufL[eo_idx(128 * w + 2 * k)]};
        const f2 y = {bufR[eo_idx(128 * w + 127 - 2 * k)], bufR[eo_idx(128 * w + 2 * k)]};
        c[0][s] = cmul_t<F>(x, tw);
        c[1][s] = cmul_t<F>(y, tw);
    }
    wave_sync();
    if constexpr (F) {
        fft_pass1_r8<2>(c);
    } else {
        radix4_pk2(c[0], c[1], BR3[0], BR3[1], BR3[2], BR3[3]);
        radix4_pk2(c[0], c[1], BR3[4], BR3[5], BR3[6], BR3[7]);
#pragma unroll
        for (int k = 0; k < 4; k++) bfly_pk2(c[0][BR3[k]], c[0][BR3[k + 4]], c[1][BR3[k]], c[1][BR3[k + 4]], ld2(T.roots_s[8 * k]));
    }
    // transpose within each window's 8 lanes: register p holds element e bits 0-2 = bitrev3(p), lane
    // bits 0-2 hold e bits 5,4,3; afterwards register s holds e = b + 8 s.  Three register-bit /
    // lane-bit exchanges (the long transform's second exchange: register bits 0,1,2 <-> lane bits
    // 2,1,0) do it in registers, without the LDS round trip (JAAD_SHORT_LDS: A/B builds with it)
#if !defined(JAAD_SHORT_LDS)
    xch_bit_pair<0, 2>(c[0], c[1]);
    xch_bit_pair<1, 1>(c[0], c[1]);
    xch_bit_pair<2, 0>(c[0], c[1]);
    (void)bufL;
    (void)bufR;
#else
    f2* XL = reinterpret_cast<f2*>(bufL);
    f2* XR = reinterpret_cast<f2*>(bufR);
    const int t = (int)(__builtin_bitreverse32((uint32_t)b) >> 29);
#pragma unroll
    for (int r = 0; r < 8; r++) {
        XL[xs(64 * w + 8 * t + r)] = c[0][BR3[r]];
        XR[xs(64 * w + 8 * t + r)] = c[1][BR3[r]];
    }
    wave_sync();
#pragma unroll
    for (int s = 0; s < 8; s++) {
        c[0][s] = XL[xs(64 * w + b + 8 * s)];
        c[1][s] = XR[xs(64 * w + b + 8 * s)];
    }
    wave_sync();
#endif
    // stages i = 8, 16, 32 of the 64-point IFFT: roots[k*m], m = 4, 2, 1.  The +-1 LSB kernel runs
    // them as the long transform's pass 2 (the same 64-point sub-transform structure, element
    // b + 8 s in register s): radix-8 with the W64 twiddles of LdsTables::tw2f (FFT_TABLE_512
    // entries, equal to FFT_TABLE_64's within the tables' rounding)
    if constexpr (F && !kShortR2) {
        fft_pass_r8<2>(c, [&](int j) { return ld2(T.tw2f[j][b]); });
    } else {
        fft_3stages_pk2<F>(c[0], c[1], [&](int j) {
            const int idx = j == 0 ? 4 * b : (j < 3 ? 2 * (b + 8 * (j - 1)) : b + 8 * (j - 3));
            return ld2(T.roots_s[idx]);
        });
    }
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const f2 tw = ld2(F && kScaledOut ? T.mdct_s_f[b + 8 * s] : T.mdct_s[b + 8 * s]);
        const f2 z = cmul_t<F>(c[0][s], tw), y = cmul_t<F>(c[1][s], tw);
        reL[s] = z.x;
        imL[s] = z.y;
        reR[s] = y.x;
        imR[s] = y.y;
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

// ola_short on both channels of a CPE (imdct_short_pk2's outputs): each channel's own windows and
// overlap, every LDS phase shared (two wave_syncs per phase instead of four per channel pair)
__device__ __forceinline__ void ola_short2(float* TL, float* TR, const LdsTables& T, int u, const FrameCtx& fL,
                                           const FrameCtx& fR, const float (&reL)[8], const float (&imL)[8],
                                           const float (&reR)[8], const float (&imR)[8], float (&ovL)[16],
                                           float (&ovR)[16], float (&outL)[16], float (&outR)[16])
{
    const int w = u >> 3, b = u & 7;
    const float* SWcL = T.win_short[fL.shape];
    const float* SWrL = T.win_short[w == 0 ? fL.shape_prev : fL.shape];
    const float* SWcR = T.win_short[fR.shape];
    const float* SWrR = T.win_short[w == 0 ? fR.shape_prev : fR.shape];
    float nvL[16], nvR[16];
#pragma unroll
    for (int phase = 0; phase < 2; phase++) {  // 0: falling halves (A), 1: rising halves (B)
#pragma unroll
        for (int s = 0; s < 8; s++) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                int n;
                float vl, vr;
                short_slot(b, s, j, reL, imL, n, vl);
                short_slot(b, s, j, reR, imR, n, vr);
                if ((n < 128) != (phase == 1)) continue;  // j = 0,1 rising; j = 2,3 falling (compile-time)
                if (phase == 0) {
                    TL[128 * w + (n - 128)] = vl * SWcL[255 - n];
                    TR[128 * w + (n - 128)] = vr * SWcR[255 - n];
                } else {
                    TL[128 * w + n] = vl * SWrL[n];
                    TR[128 * w + n] = vr * SWrR[n];
                }
            }
        }
        wave_sync();
        const int uu = lane_id();  // opaque: stop index math being hoisted/kept across phases
#pragma unroll
        for (int o = 0; o < 16; o++) {
            const int P = long_pos(uu, o);
            const int mo = (P - 448) >> 7, io = (P - 448) & 127;
            const int mq = (P + 576) >> 7, iq = (P + 576) & 127;
            if (phase == 0) {
                outL[o] = (P >= 448 + 128) ? ovL[o] + TL[128 * (mo - 1) + io] : ovL[o];
                outR[o] = (P >= 448 + 128) ? ovR[o] + TR[128 * (mo - 1) + io] : ovR[o];
                nvL[o] = (mq <= 8) ? TL[128 * (mq - 1) + iq] : 0.0f;
                nvR[o] = (mq <= 8) ? TR[128 * (mq - 1) + iq] : 0.0f;
            } else {
                if (P >= 448) {
                    outL[o] = outL[o] + TL[128 * mo + io];
                    outR[o] = outR[o] + TR[128 * mo + io];
                }
                if (mq <= 7) {
                    nvL[o] = nvL[o] + TL[128 * mq + iq];
                    nvR[o] = nvR[o] + TR[128 * mq + iq];
                }
            }
        }
        wave_sync();
    }
#pragma unroll
    for (int o = 0; o < 16; o++) {
        ovL[o] = nvL[o];
        ovR[o] = nvR[o];
    }
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
            const int base = (is_short ? 128 * (F.window & 7) : 0) + start;
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

// Math.round(float) followed by SampleBuffer's short clamp (S/SampleBuffer.java:193-206), two
// samples at a time.  v_cvt_rpi_i32_f32 = (int)floor(x + 0.5) evaluated exactly, which equals
// Math.round for every float except NaN (checked exhaustively over all 2^32 bit patterns on
// MI355X, tools/probe_round.hip); v_cvt_pk_i16_i32 saturates to int16.  A NaN cannot reach
// this point: |spectral value| <= IQ[8191] * 2^(155/4) < 2^57, so no IMDCT/OLA sum overflows,
// PNS energy is a sum of squares of consecutive (distinct) LCG states and never 0, and
// jaad_state_import rejects non-finite overlap values.
__device__ __forceinline__ uint32_t round_pk16(float a, float b)
{
    int ia, ib;
    uint32_t w;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(ia) : "v"(a));
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(ib) : "v"(b));
    asm("v_cvt_pk_i16_i32 %0, %1, %2" : "=v"(w) : "v"(ia), "v"(ib));
    return w;
}

// +-1 LSB kernel: two samples to int16 in one conversion -- v_cvt_pknorm_i16_f32 rounds x * 32767 to
// nearest and saturates to [-32767, 32767], and the kernel's samples are already in those units
// (kScaledOut: the post-twiddles carry the 1/32767; JAAD_NO_SCALED builds multiply here).  The
// integer can differ from Math.round's by one at a tie, and -32768 comes out as -32767; both within
// the mode's bar.  1 instruction per sample pair instead of 3.
__device__ __forceinline__ uint32_t round_pk16_lsb1(float a, float b)
{
    f2 x = f2{a, b};
    if constexpr (!kScaledOut) x = x * f2{kPcmUnit, kPcmUnit};
    uint32_t w;
    asm("v_cvt_pknorm_i16_f32 %0, %1, %2" : "=v"(w) : "v"(x.x), "v"(x.y));
    return w;
}

// s_waitcnt vmcnt(0) that the compiler's wait insertion sees (an asm statement it would not).
// vmcnt counts loads and stores together, and the compiler cannot rely on a load completing
// before a younger store (it then waits for vmcnt(0)); so the prefetched loads of frame f+1 are
// drained explicitly BEFORE frame f's PCM stores are issued.  Otherwise the first use of frame
// f+1's inputs at the top of the loop waits for frame f's stores to reach memory.
__device__ __forceinline__ void vmem_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0) expcnt(7) lgkmcnt(15)

// PCM stores of one frame through a buffer resource covering exactly that frame: a prefix frame
// (re-decoded only to rebuild the overlap) stores to offset >= num_records, which the hardware
// drops.  So every frame issues the same stores: the compiler then knows that the next frame's
// prefetched loads have exactly those stores younger than them and waits with vmcnt(N) at the
// top of the frame loop instead of vmcnt(0) -- which would wait for the previous frame's stores
// to reach memory (a wave would stall once per frame for the whole store round trip).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(void* base, int bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);  // gfx9 raw buffer
}
__device__ __forceinline__ void store16(v4u v, __amdgpu_buffer_rsrc_t r, int off, bool nt)
{
    if (nt) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 2);  // aux 2: nt
    else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

// per-wave LDS area: 8.5 KiB (16 waves + the 20 KiB table image fill a CU's 160 KiB)
//   buf  band records [0,512) -> spectrum (E/O) -> IFFT transposes ->
//        OLA scratch -> PCM staging
//   rsp  the right channel's spectrum while the left one is transformed (PNS: raw row copy)
constexpr int kRspFloats = kWaveBuf;  // second channel buffer (spectrum + PCM staging)
template <bool kTns>
struct alignas(16) WaveLds {
    float buf[kWaveBuf];
    float rsp[kRspFloats];
};
template <>
struct alignas(16) WaveLds<true> {
    float buf[kWaveBuf];
    float rsp[kRspFloats];
    float tns[192];  // spec-TNS LPC scratch (8 filters x 24)
};
#ifndef JAAD_LC_WAVES
#define JAAD_LC_WAVES 12
#endif
template <bool kTns>
constexpr int waves_per_wg()
{
    return kTns ? 8 : JAAD_LC_WAVES;
}

// One scalefactor band (index g*max_sfb+sfb) of one frame, both channels:
//   gl / gr   gain applied to IQ values, 0 for bands that are not spectral (ZERO/NOISE/IS)
//   ms        1.0 where M/S applies (ms_used bit and both codebooks < NOISE_HCB, MS.java:25-27)
//   is        +-gain_R where the right band is intensity coded (IS.java:26-40), else 0
struct alignas(16) BandRec {
    float gl, ms, gr, is;
};
constexpr int kNoBand = 127;  // a record index that is always all-zero (bands < 8*15 = 120)
constexpr float kZeroBandGain = -0.0f;  // gain of bands that are not spectral (see iq_channel)

// record index of the bin quad starting at position p (4-aligned); long windows use the
// lane's precomputed band byte
__device__ __forceinline__ int band_short(const LdsTables& T, const Ics& ic, int p)
{
    const int w = p >> 7;
    const int sfb = T.quad2band_s[(p & 127) >> 2];
    const int g = w - __builtin_popcount(ic.grouping & ((1u << w) - 1u));
    return sfb < ic.max_sfb ? g * ic.max_sfb + sfb : kNoBand;
}

// PNS (ICStream.java:241-257): lane 0 replays the static LCG in parse order over the channel's
// noise bands; gain = -SCALEFACTOR_TABLE[...] (ICStream.java:205-206).
__device__ void pns_fill(float* buf, const uint32_t* raw, const LdsTables& T, const GlobalTables& G, int u,
                         const Ics& info)
{
    if (u == 0) {
        const uint8_t* sfr = reinterpret_cast<const uint8_t*>(raw);
        const uint8_t* cbr = sfr + 128;
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
                if (cbr[idx] != JAAD_NOISE_HCB) continue;
                int off = groupOff + offs[sfb];
                const int width = offs[sfb + 1] - offs[sfb];
                const float sfv = -T.sf_gain[sfr[idx]];
                for (int w = 0; w < glen[g]; w++, off += 128) {
                    float energy = 0.0f;
                    for (int k = 0; k < width; k++) {
                        rs = 1664525u * rs + 1013904223u;
                        const float v = (float)(int32_t)rs;
                        buf[eo_idx(off + k)] = v;
                        energy += v * v;
                    }
                    const float scale = (float)((double)sfv / sqrt((double)energy));
                    for (int k = 0; k < width; k++) buf[eo_idx(off + k)] *= scale;
                }
            }
            groupOff += glen[g] << 7;
        }
    }
    wave_sync();
}

struct Prefetch {
    v4i q[2][2];       // [channel][h]: bins 8u+512h .. +7
    uint32_t sf2[2], cb2[2];  // [channel] sf / cb bytes of bands 2u, 2u+1 (zero-extended 16 bits)
    uint32_t side;     // lane i < 4*nch: dword i of the frame's jaad_ics_info records;
                       // lanes 8..11: the frame's ms_used words (read back with readlane)
};

// Everything frame f needs from HBM, as vector loads (vmcnt is in order; scalar loads would
// share lgkmcnt with the LDS traffic and could not be left in flight).
__device__ __forceinline__ void prefetch(const KernelArgs& A, int f, bool stereo, int u, Prefetch& pf, int skip = 0)
{
    const int nch = stereo ? 2 : 1;
#pragma unroll
    for (int c = 0; c < 2; c++) {
        if (c == 1 && !stereo) break;
        const size_t cf = (size_t)f * A.cf_stride + c;
        const v4i* q = reinterpret_cast<const v4i*>(A.q + cf * 1024);
        pf.q[c][0] = __builtin_nontemporal_load(q + u);
        pf.q[c][1] = __builtin_nontemporal_load(q + 64 + u);
        // lane u's two bands straight from the rows (no LDS round trip to regroup row dwords)
        pf.sf2[c] = reinterpret_cast<const uint16_t*>(A.sf + cf * 128)[u];
        pf.cb2[c] = reinterpret_cast<const uint16_t*>(A.cb + cf * 128)[u];
    }
    const uint32_t* side = u < 8 ? reinterpret_cast<const uint32_t*>(A.ics + (size_t)f * A.cf_stride) + (u < 4 * nch ? u : 0)
                                 : (A.ms_used ? reinterpret_cast<const uint32_t*>(A.ms_used + (size_t)f * 2 * A.ms_stride) + (u & 3)
                                              : reinterpret_cast<const uint32_t*>(A.ics));
    // batches with dropped frames: lanes 63 / 62 carry skip entry `skip` (first frame, count of
    // the next run of dropped frames), which the loop reads to step to the frame after this one
    if (A.skips && u >= 62) side = A.skips + 2 * skip + (u == 62);
    pf.side = *side;
}

// inverse quantisation of one channel's 16 bins (ICStream.java:258-271):
// x = gain != 0 ? (q>0 ? IQ[q] : -IQ[-q]) * gain : 0
__device__ __forceinline__ void iq_channel(const LdsTables& T, const float* iq_global, const v4i (&q)[2],
                                           const float (&g)[4], float (&x)[16])
{
    // all 16 table reads are issued before the first is consumed (one LDS round trip, not 16)
    float v[16];
    // two bins per dword: one packed 16-bit add biases both to table indices q + kIqHead, which
    // lie in [0, 2 kIqHead) exactly when no escape is needed (bits 11..15 of each half clear);
    // the halves become byte offsets by SDWA word selects.  Escaped bins read some LDS word (an
    // LDS read never faults) that the escape pass below replaces.
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    static_assert(kIqHead == 1024, "escape mask assumes a 2048-entry head");
    uint32_t t[8];
#pragma unroll
    for (int d = 0; d < 8; d++) {
        const uint32_t w = reinterpret_cast<const uint32_t*>(&q[d >> 2])[d & 3];
        t[d] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, w) + (us2){kIqHead, kIqHead});
    }
    const bool esc = ((t[0] | t[1] | t[2] | t[3] | t[4] | t[5] | t[6] | t[7]) & 0xF800F800u) != 0u;
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const uint32_t idx = (e & 1) ? (t[e >> 1] >> 16) : (t[e >> 1] & 0xFFFFu);
        v[e] = T.iq_signed[idx];
    }
    // the 8 packed adds, then each table read right after its address (no SDWA-after-VALU nops)
    __builtin_amdgcn_sched_group_barrier(0x0002, 8, 0);
#pragma unroll
    for (int e = 0; e < 16; e++) {
        __builtin_amdgcn_sched_group_barrier(0x0002, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x0002, 64, 0);  // then the VALU
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const float gn = g[e >> 2];
        x[e] = v[e] * gn;  // gn = -0.0 for a non-spectral band (kZeroBandGain): -0.0 * -0.0 = +0.0
    }
    // escape values beyond the LDS head of IQ_TABLE (|q| >= 1024: rare in real streams and absent
    // from the synthetic ones); global loads, which also wait for the previous frame's PCM stores
    if (__builtin_expect(__ballot(esc) != 0, 0)) {
        // uniform branch; every lane recomputes its 16 bins: the head entry of the clamped index
        // (an escaped bin of a non-spectral band gives +-0 as in the reference, not whatever the
        // fast path read), the global table where the gain is nonzero
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const int qq = reinterpret_cast<const int16_t*>(&q[e >> 3])[e & 7];
            const int qc = qq < -kIqHead ? -kIqHead : (qq > kIqHead - 1 ? kIqHead - 1 : qq);
            const int aq = qq < 0 ? -qq : qq;
            const float gn = g[e >> 2];
            const float m = iq_global[aq > 8190 ? 8190 : aq] * gn;
            const bool big = (qq > kIqHead - 1 || qq < -kIqHead) && gn != 0.0f;
            x[e] = big ? (qq > 0 ? m : -m) : T.iq_signed[qc + kIqHead] * gn;
        }
    }
}

// iq_channel in two halves (the +-1 LSB kernel): the 16 table reads are issued at the top of the
// frame, from the prefetched q alone, so that their LDS round trip overlaps the band-record phase's
// two; iq_finish applies the gains once the records are read.  Same arithmetic as iq_channel.
struct IqPending {
    float v[16];
    bool esc;
};
__device__ __forceinline__ void iq_issue(const LdsTables& T, const v4i (&q)[2], IqPending& P)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    uint32_t t[8];
#pragma unroll
    for (int d = 0; d < 8; d++) {
        const uint32_t w = reinterpret_cast<const uint32_t*>(&q[d >> 2])[d & 3];
        t[d] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, w) + (us2){kIqHead, kIqHead});
    }
    P.esc = ((t[0] | t[1] | t[2] | t[3] | t[4] | t[5] | t[6] | t[7]) & 0xF800F800u) != 0u;
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const uint32_t idx = (e & 1) ? (t[e >> 1] >> 16) : (t[e >> 1] & 0xFFFFu);
        P.v[e] = T.iq_signed[idx];
    }
}
__device__ __forceinline__ void iq_finish(const LdsTables& T, const float* iq_global, const v4i (&q)[2],
                                          const IqPending& P, const float (&g)[4], float (&x)[16])
{
#pragma unroll
    for (int e = 0; e < 16; e++) x[e] = P.v[e] * g[e >> 2];
    if (__builtin_expect(__ballot(P.esc) != 0, 0)) {  // (iq_channel's escape pass)
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const int qq = reinterpret_cast<const int16_t*>(&q[e >> 3])[e & 7];
            const int qc = qq < -kIqHead ? -kIqHead : (qq > kIqHead - 1 ? kIqHead - 1 : qq);
            const int aq = qq < 0 ? -qq : qq;
            const float gn = g[e >> 2];
            const float m = iq_global[aq > 8190 ? 8190 : aq] * gn;
            const bool big = (qq > kIqHead - 1 || qq < -kIqHead) && gn != 0.0f;
            x[e] = big ? (qq > 0 ? m : -m) : T.iq_signed[qc + kIqHead] * gn;
        }
    }
}

// (TNS) -> IMDCT -> window/OLA of one channel whose spectrum is in buf (E/O layout); result
// in out (slot o = position long_pos(u, o)), new overlap in ov
// Dependent coupling with spec TNS (kernel mode 3): frame f's AFTER_TNS terms for channel ch of
// this launch, added to the channel's spectrum in LDS once its TNS filters have run (CPE.java:
// 172-179, SCE.java:100-108; the terms' addends from cce_term_kernel, -0.0 adds nothing)
__device__ __forceinline__ void couple_after_tns(const KernelArgs& A, float* buf, int f, int ch, int u)
{
    const uint32_t t0 = A.cce_off[f], t1 = A.cce_off[f + 1];
    bool any = false;
    float x[16];
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t meta = A.cce_meta[t];
        if (!(meta >> 24) || (int)((meta >> 16) & 0xFF) - (int)A.ch0 != ch) continue;
        if (!any) load_spec(buf, u, x);  // (the TNS filters ended with a wave_sync)
        any = true;
        const float4* sp = reinterpret_cast<const float4*>(A.cce_spec + (size_t)t * 1024);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const float4 a = sp[(512 * h + 8 * u) / 4], c = sp[(512 * h + 8 * u) / 4 + 1];
            const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 8; i++) x[8 * h + i] += v[i];
        }
    }
    if (any) {
        store_spec(buf, u, x);
        wave_sync();
    }
}

template <bool kTnsSpec, bool kCoupleAfter = false, bool F = false>
__device__ __forceinline__ void synth_channel(const KernelArgs& A, const LdsTables& T, WaveLds<kTnsSpec>& W, float* buf,
                                              const Ics& ic, size_t cf, float (&ov)[16], float (&out)[16], int f = 0,
                                              int ch = 0)
{
    const int u = lane_id();
    if constexpr (kTnsSpec)
        if (A.tns_mode == JAAD_TNS_SPEC && (ic.flags & JAAD_ICS_TNS) && A.tns) tns_spec(buf, W.tns, T, *A.gtab, u, ic, A.tns + cf);
    if constexpr (kCoupleAfter) couple_after_tns(A, buf, f, ch, u);
    const FrameCtx fc{ic.seq, ic.shape, ic.shape_prev};
    if (fc.seq == JAAD_EIGHT_SHORT_SEQUENCE) {
        float re[8], im[8];
        imdct_short_pk<F>(buf, T, u, re, im);
        ola_short(buf, T, u, fc, re, im, ov, out);
    } else {
        float* const bufs[1] = {buf};
        f2 cx[1][8];
        imdct_long_pk<1, F>(bufs, T, u, cx);
        ola_long_pk<F>(T, fc, cx[0], ov, out);
    }
    wave_sync();
}

#ifdef JAAD_STAMPS
// per-phase wave-time accounting (ablation/profiling builds only): phase k gets the s_memtime
// ticks since the previous stamp; lane 0 writes the 16 totals of each wave to A.dbg
#define STAMP(k)                                                  \
    do {                                                          \
        uint64_t t_;                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        st_acc[k] += (uint32_t)(t_ - st_prev);                    \
        st_prev = t_;                                             \
    } while (0)
#elif defined(JAAD_MARKS)  // design tool: phase markers in the device assembly (tools/isa_mix.py)
#define STAMP(k) asm volatile(";PHASE " #k)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

// JAAD_BOUNDS builds (diagnostics): every global access of lc_decode_kernel is checked
// against the launch's bounds (KernelArgs::frame_lo/hi, n_slots, n_skip_pairs, n_cce_terms) before
// it is issued; a failing check prints the chunk, the frame, what was accessed and the two values
// compared, and the wave leaves the kernel (the conditions are wave-uniform).  Product builds
// compile the checks away (the chunk-level guard below stays).
#ifdef JAAD_BOUNDS
#define JAAD_BOUND(ci, f, cond, what, a, b)                                                                 \
    do {                                                                                                   \
        if (!(cond)) {                                                                                     \
            if (lane_id() == 0)                                                                            \
                printf("JAAD_BOUNDS lc_decode_kernel: chunk %u frame %d: %s %u vs %u\n", (unsigned)(ci), (int)(f), \
                       what, (unsigned)(a), (unsigned)(b));                                                \
            return;                                                                                        \
        }                                                                                                  \
    } while (0)
#else
#define JAAD_BOUND(ci, f, cond, what, a, b) \
    do {                                    \
    } while (0)
#endif

// kMode: 0 = TNS compat (the reference), 1 = spec TNS, 2 = TNS compat with dependent coupling,
// 3 = spec TNS with dependent coupling (BEFORE_TNS terms, the TNS filters, AFTER_TNS terms),
// 4 = mode 0 at +-1 LSB precision (JAAD_PRECISION_LSB1: fused multiply-adds in the transforms),
// 5 / 6 = mode 0 / 4 built for batches with EIGHT_SHORT frames (both channels' short IMDCTs and
// overlap-adds in lockstep; chosen per launch by the host, KernelArgs::short_pair)
template <int kMode, int kOut, bool kStereo>
__global__ __launch_bounds__(64 * waves_per_wg<kMode == 1 || kMode == 3>()) void lc_decode_kernel(KernelArgs A)
{
    constexpr bool kTnsSpec = kMode == 1 || kMode == 3;
    [[maybe_unused]] constexpr bool kCouple = kMode == 2 || kMode == 3;
    constexpr bool kFast = kMode == 4 || kMode == 6;
    [[maybe_unused]] constexpr bool kShortPair = kMode == 5 || kMode == 6;
    constexpr int kW = waves_per_wg<kTnsSpec>();
    constexpr int kThreads = 64 * kW;
    // one LDS object with the tables first: every table access is a 16-bit immediate offset
    struct Lds {
        LdsTables T;
        WaveLds<kTnsSpec> W[kW];
        uint32_t rem[kW];  // frames each wave has left in its chunk (issue priority, below)
    };
    __shared__ Lds S;
    LdsTables& T = S.T;

    {
        const uint4* src = reinterpret_cast<const uint4*>(A.tables);
        uint4* dst = reinterpret_cast<uint4*>(&T);
        for (int i = threadIdx.x; i < (int)(sizeof(LdsTables) / 16); i += kThreads) dst[i] = src[i];
        if (threadIdx.x < kW) S.rem[threadIdx.x] = 0u;
    }
    __syncthreads();  // the only workgroup barrier: waves are independent from here on
#ifdef JAAD_WAVETIME
    const uint64_t wt0 = __builtin_amdgcn_s_memrealtime();
    uint32_t wt_frames = 0;
#endif

    constexpr bool big_endian = !(kOut & JAAD_PCM_LITTLE_ENDIAN);
    constexpr bool planar = kOut == (int)kOutPlanarF32;
    constexpr bool out_f32 = (kOut & JAAD_PCM_FLOAT32) != 0 && !planar;
    [[maybe_unused]] constexpr bool out_i16 = !planar && !out_f32;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // channel count is a template parameter: a run-time flag would leave the register allocator
    // with paths where the right channel's values live across frames
    constexpr bool stereo = kStereo;
    constexpr int nch = stereo ? 2 : 1;
    WaveLds<kTnsSpec>& W = S.W[wave];
    BandRec* rec = reinterpret_cast<BandRec*>(W.buf);

    // scalefactor band counts (frame invariant: read once, not from LDS in every frame)
    const int nswb_l = __builtin_amdgcn_readfirstlane(T.nswb_l), nswb_s = __builtin_amdgcn_readfirstlane(T.nswb_s);
    // long-window band of each of the lane's 4 bin quads (frame invariant)
    uint32_t q2b_long = 0;
    {
        const int u = lane_id();
#pragma unroll
        for (int qd = 0; qd < 4; qd++) {
            const uint32_t b = T.quad2band_l[(512 * (qd >> 1) + 8 * u + 4 * (qd & 1)) >> 2];
            q2b_long |= (b > kNoBand ? kNoBand : b) << (8 * qd);
        }
    }

#ifdef JAAD_STAMPS
    uint32_t st_acc[16] = {};
    uint64_t st_prev;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
#endif
    for (uint32_t ci = blockIdx.x * kW + wave; ci < A.n_chunks; ci += gridDim.x * kW) {
        const ChunkDesc cd = A.chunks[ci];
        const int nfr = cd.info & 0xffff;
        const bool prefix = (cd.info & kChunkPrefix) != 0;
        const int my_n = nfr + (prefix ? 1 : 0);
        const int f_first = (int)cd.frame0;  // batch frame of the first iteration
        // a descriptor outside this launch's bounds is never walked (plan() validates the table on
        // the host; this guards the device copy the kernel actually reads): one scalar test per chunk
        JAAD_BOUND(ci, -1, cd.slot < A.n_slots, "chunk slot", cd.slot, A.n_slots);
        JAAD_BOUND(ci, f_first, my_n == 0 || (cd.frame0 >= A.frame_lo && cd.frame0 + (uint32_t)my_n <= A.frame_hi),
                   "chunk frames", cd.frame0 + (uint32_t)my_n, A.frame_hi);
        JAAD_BOUND(ci, f_first, !A.skips || cd.skip < A.n_skip_pairs, "chunk skip entry", cd.skip, A.n_skip_pairs);
        if (cd.slot >= A.n_slots || (my_n && (cd.frame0 < A.frame_lo || cd.frame0 >= A.frame_hi))) continue;

        float ovL[16], ovR[16];
        {
            const int u = lane_id();
            if (cd.info & kChunkLoadState) {
                const float* st = A.state_in + (size_t)cd.slot * 2048;
#pragma unroll
                for (int o = 0; o < 16; o++) {
                    ovL[o] = st[long_pos(u, o)];
                    ovR[o] = st[1024 + long_pos(u, o)];
                    if constexpr (kFast && kScaledOut) {  // (the state is in reference units)
                        ovL[o] *= kPcmUnit;
                        ovR[o] *= kPcmUnit;
                    }
                }
            } else {
#pragma unroll
                for (int o = 0; o < 16; o++) ovL[o] = ovR[o] = 0.0f;
            }
        }
        // The chunk's frames are batch frames f_first, then f + 1 after each frame f, except
        // where a run of dropped frames starts (KernelArgs::skips: entry `skip` is the next such
        // run, loaded with each frame's side info).
        int skip = (int)cd.skip;
        int fr_next = f_first;  // batch frame of the iteration's frame
        Prefetch pf;
        if (my_n > 0) prefetch(A, fr_next, stereo, lane_id(), pf, skip);
        vmem_drain();  // (see vmem_drain) the loop head then finds no load pending on any path

        for (int it = 0; it < my_n; it++) {
            // Issue arbitration between the waves of a SIMD favours the oldest wave: left alone,
            // the three waves of a SIMD end ~12 us apart and the last ones run with their latency
            // exposed.  The waves sharing this wave's SIMD are w +- 4 (a workgroup's waves go to the
            // SIMDs in a fixed cyclic order); the one with the most frames left gets the highest
            // priority, so that they end together (C2 wave ends 132-171 -> 147-160 us, busy 88 ->
            // 95 % of span x waves; batch -1 %, profiles/round5_balance/).
#if defined(JAAD_PRIO_LATE)  // (A/B builds: the mates' counts read here, the priority set after the IQ)
            const uint32_t rem_late = (uint32_t)(my_n - it);
            uint32_t mates_late[kW / 4 - 1];
            {
                volatile uint32_t* R = S.rem;
                R[wave] = rem_late;
#pragma unroll
                for (int m = 1; m < kW / 4; m++) mates_late[m - 1] = R[(wave + 4 * m) % kW];
            }
#elif !defined(JAAD_ABL_NOPRIO)
#ifndef JAAD_PRIO_EVERY  // (A/B builds: the priority recomputed every N frames)
#define JAAD_PRIO_EVERY 1
#endif
            if ((it % JAAD_PRIO_EVERY) == 0) {
                const uint32_t rem = (uint32_t)(my_n - it);
                volatile uint32_t* R = S.rem;
                R[wave] = rem;
                int p = 0;
#pragma unroll
                for (int m = 1; m < kW / 4; m++) {
                    const int mate = (wave + 4 * m) % kW;
                    const uint32_t r = __builtin_amdgcn_readfirstlane(R[mate]);
                    p += (rem > r || (rem == r && wave > mate)) ? 1 : 0;
                }
                if (p >= 2) __builtin_amdgcn_s_setprio(3);
                else if (p == 1) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(1);
            }
#endif
            STAMP(5);
#ifdef JAAD_WAVETIME
            wt_frames++;
#endif
            const int u = lane_id();
            const bool emit = it >= (prefix ? 1 : 0);
            const int f = fr_next;                   // batch frame
            const size_t cf0 = (size_t)f * A.cf_stride;
            const Prefetch cur = pf;
            fr_next = f + 1;
            if (A.skips && fr_next == __builtin_amdgcn_readlane(cur.side, 63)) {  // step over dropped frames
                fr_next += __builtin_amdgcn_readlane(cur.side, 62);
                skip++;
            }
            // (JAAD_BOUNDS: the frame this iteration decodes was prefetched in the previous one; the
            // frame the next prefetch reads and its skip entry are checked here, before it is issued)
            JAAD_BOUND(ci, f, (uint32_t)f >= A.frame_lo && (uint32_t)f < A.frame_hi, "frame rows / pcm", f, A.frame_hi);
            JAAD_BOUND(ci, f, it + 1 >= my_n || ((uint32_t)fr_next >= A.frame_lo && (uint32_t)fr_next < A.frame_hi),
                       "prefetched frame", fr_next, A.frame_hi);
            JAAD_BOUND(ci, f, !A.skips || (uint32_t)skip < A.n_skip_pairs, "skip entry", skip, A.n_skip_pairs);
            if constexpr (kCouple) {
                JAAD_BOUND(ci, f, A.cce_off[f] <= A.cce_off[f + 1] && A.cce_off[f + 1] <= A.n_cce_terms, "coupling terms",
                           A.cce_off[f + 1], A.n_cce_terms);
            }

#if defined(JAAD_NO_IQ_EARLY)  // (A/B builds)
            constexpr bool kIqEarly = false;
#else
            constexpr bool kIqEarly = kFast;
#endif
            [[maybe_unused]] IqPending iqL, iqR;
            if constexpr (kIqEarly) {  // the IQ table reads first (iq_issue)
                iq_issue(T, cur.q[0], iqL);
                if (stereo) iq_issue(T, cur.q[1], iqR);
            }
            // ---------------- side info ----------------
            const Ics iL = ics_from_lanes(cur.side, 0, nswb_l, nswb_s);
            STAMP(6);
            const Ics iR = stereo ? ics_from_lanes(cur.side, 4, nswb_l, nswb_s) : iL;
            const bool ms_on = stereo && (iL.flags & JAAD_ICS_COMMON_WINDOW) && (iL.flags & JAAD_ICS_MS_PRESENT);
            const bool is_on = stereo && (iR.flags & JAAD_ICS_HAS_IS);
            const bool same_bands = !stereo || (iL.seq == iR.seq && iL.max_sfb == iR.max_sfb && iL.grouping == iR.grouping);
            uint64_t m0 = 0, m1 = 0;
            if (ms_on && A.ms_used) {
                // readlane returns int: widen through uint32_t (no sign extension)
                m0 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 8) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 9) << 32);
                m1 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 10) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur.side, 11) << 32);
            }

            STAMP(0);
            // ---------------- band records (lane u: bands 2u, 2u+1) ----------------
            {
                const uint32_t sfL2 = cur.sf2[0], cbL2 = cur.cb2[0];
                const uint32_t sfR2 = stereo ? cur.sf2[1] : 0u, cbR2 = stereo ? cur.cb2[1] : 0u;
                const uint64_t mw = u < 32 ? m0 : m1;
                const uint32_t msb = (uint32_t)(mw >> ((2 * u) & 63)) & 3u;
                BandRec br[2];
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const int b = 2 * u + e;
                    const uint32_t sfL = (sfL2 >> (8 * e)) & 255u, cbL = (cbL2 >> (8 * e)) & 255u;
                    const uint32_t sfR = (sfR2 >> (8 * e)) & 255u, cbR = (cbR2 >> (8 * e)) & 255u;
                    const bool inL = b < iL.nbands, inR = b < iR.nbands;
                    const bool msbit = (msb >> e) & 1u;
                    const float gvL = T.sf_gain[sfL];
                    // non-spectral bands get -0.0: q is 0 there and iq_signed[0] = -0.0, so the
                    // product is the reference's +0.0 (ICStream.java:236-239) without a select
                    br[e].gl = (inL && cbL != JAAD_ZERO_HCB && cbL < JAAD_NOISE_HCB) ? gvL : kZeroBandGain;
                    br[e].ms = (ms_on && inL && msbit && cbL < JAAD_NOISE_HCB && cbR < JAAD_NOISE_HCB) ? 1.0f : 0.0f;
                    float gr = 0.0f, is = 0.0f;
                    if (stereo) {
                        const float gvR = T.sf_gain[sfR];
                        gr = (inR && cbR != JAAD_ZERO_HCB && cbR < JAAD_NOISE_HCB) ? gvR : kZeroBandGain;
                        if (is_on && inR && (cbR == JAAD_INTENSITY_HCB || cbR == JAAD_INTENSITY_HCB2)) {
                            float cs = cbR == JAAD_INTENSITY_HCB ? 1.0f : -1.0f;
                            if ((iL.flags & JAAD_ICS_MS_PRESENT) && msbit) cs = -cs;
                            is = cs * gvR;
                        }
                    }
                    br[e].gr = gr;
                    br[e].is = is;
                }
                wave_sync();
                reinterpret_cast<float4*>(rec)[2 * u] = make_float4(br[0].gl, br[0].ms, br[0].gr, br[0].is);
                reinterpret_cast<float4*>(rec)[2 * u + 1] = make_float4(br[1].gl, br[1].ms, br[1].gr, br[1].is);
            }
            wave_sync();

            // ---------------- inverse quantisation, PNS, M/S, I/S ----------------
            STAMP(1);
            float gL[4], gR[4], msq[4], isq[4];
            uint32_t q2b = q2b_long;
            asm volatile("" : "+v"(q2b));  // one packed register across frames, unpacked here
            if (iL.seq != JAAD_EIGHT_SHORT_SEQUENCE && same_bands) {
                // the common frame (long windows, one band layout): one record read per quad
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    const float4 r = reinterpret_cast<const float4*>(rec)[(q2b >> (8 * qd)) & 255u];
                    gL[qd] = r.x;
                    msq[qd] = r.y;
                    gR[qd] = r.z;
                    isq[qd] = r.w;
                }
            } else {
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    const int p = 512 * (qd >> 1) + 8 * u + 4 * (qd & 1);
                    const int bl = iL.seq == JAAD_EIGHT_SHORT_SEQUENCE ? band_short(T, iL, p) : (int)((q2b >> (8 * qd)) & 255u);
                    const float4 r = reinterpret_cast<const float4*>(rec)[bl];
                    gL[qd] = r.x;
                    msq[qd] = r.y;
                    if (same_bands) {
                        gR[qd] = r.z;
                        isq[qd] = r.w;
                    } else {
                        const int br = iR.seq == JAAD_EIGHT_SHORT_SEQUENCE ? band_short(T, iR, p) : (int)((q2b >> (8 * qd)) & 255u);
                        const float2 rr = reinterpret_cast<const float2*>(rec)[2 * br + 1];
                        gR[qd] = rr.x;
                        isq[qd] = rr.y;
                    }
                }
            }
            float xL[16], xR[16];
            STAMP(14);
            if constexpr (kIqEarly) {
                iq_finish(T, A.iq_table, cur.q[0], iqL, gL, xL);
                STAMP(13);
                if (stereo) iq_finish(T, A.iq_table, cur.q[1], iqR, gR, xR);
            } else {
                iq_channel(T, A.iq_table, cur.q[0], gL, xL);
                STAMP(13);
                if (stereo) iq_channel(T, A.iq_table, cur.q[1], gR, xR);
            }
#if defined(JAAD_PRIO_LATE)
            {
                int p = 0;
#pragma unroll
                for (int m = 1; m < kW / 4; m++) {
                    const int mate = (wave + 4 * m) % kW;
                    const uint32_t r = __builtin_amdgcn_readfirstlane(mates_late[m - 1]);
                    p += (rem_late > r || (rem_late == r && wave > mate)) ? 1 : 0;
                }
                if (p >= 2) __builtin_amdgcn_s_setprio(3);
                else if (p == 1) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(1);
            }
#endif
            // the inputs are consumed: frame f+1's loads fly while this frame's IMDCTs run
            STAMP(12);
            // issued on every iteration (the last one reloads its own frame) so that the VMEM
            // pattern of the loop body is the same on every path: see the PCM stores below
#ifdef JAAD_ABL_NOPREF
            if (it == 0)
#endif
            prefetch(A, it + 1 < my_n ? fr_next : f, stereo, u, pf, skip);

            if ((iL.flags | (stereo ? iR.flags : 0)) & JAAD_ICS_HAS_PNS) {  // rare: lane 0 replays the LCG
                // pns_fill reads the channel's raw sf/cb rows from rsp
                uint32_t* rcopy = reinterpret_cast<uint32_t*>(W.rsp);
                wave_sync();
                {  // the raw rows as the prefetch left them: sf bytes [0,128), cb bytes [128,256) per channel
                    uint16_t* r16 = reinterpret_cast<uint16_t*>(rcopy);
                    r16[u] = (uint16_t)cur.sf2[0];
                    r16[64 + u] = (uint16_t)cur.cb2[0];
                    if (stereo) {
                        r16[128 + u] = (uint16_t)cur.sf2[1];
                        r16[192 + u] = (uint16_t)cur.cb2[1];
                    }
                }
                if (iL.flags & JAAD_ICS_HAS_PNS) {
                    wave_sync();
                    store_spec(W.buf, u, xL);
                    wave_sync();
                    pns_fill(W.buf, rcopy, T, *A.gtab, u, iL);
                    load_spec(W.buf, u, xL);
                }
                if (stereo && (iR.flags & JAAD_ICS_HAS_PNS)) {
                    wave_sync();
                    store_spec(W.buf, u, xR);
                    wave_sync();
                    pns_fill(W.buf, rcopy + 64, T, *A.gtab, u, iR);
                    load_spec(W.buf, u, xR);
                }
            }
            STAMP(2);
            if (ms_on) {  // MS.java:28-33: L' = L + R, R' = L - R (no scaling)
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    if (msq[qd] != 0.0f) {
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const int e = 8 * (qd >> 1) + 4 * (qd & 1) + i;
                            const float l = xL[e], r = xR[e];
                            xL[e] = l + r;
                            xR[e] = l - r;
                        }
                    }
                }
            }
            if (is_on) {  // IS.java:41-46: R = L * (+-gain); never on an M/S band (cb_R >= 14)
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    if (isq[qd] != 0.0f) {
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const int e = 8 * (qd >> 1) + 4 * (qd & 1) + i;
                            xR[e] = xL[e] * isq[qd];
                        }
                    }
                }
            }

            if constexpr (kCouple) {
                // dependent coupling after M/S and I/S (CPE.java:172-179, SCE.java:100-108): the
                // frame's terms in order, each adding its addend (CCE.applyDependentCoupling,
                // A/syntax/CCE.java:188-215, precomputed by cce_term_kernel; -0.0 adds nothing)
                // (with spec TNS, mode 3, the AFTER_TNS terms -- the frame's last ones -- wait for
                // the filters: couple_after_tns)
                const uint32_t t0 = A.cce_off[f], t1 = A.cce_off[f + 1];
                for (uint32_t t = t0; t < t1; t++) {
                    if (kMode == 3 && (A.cce_meta[t] >> 24)) break;
                    const int ch = (int)((A.cce_meta[t] >> 16) & 0xFF) - (int)A.ch0;
                    if (ch < 0 || ch >= nch) continue;
                    const float4* sp = reinterpret_cast<const float4*>(A.cce_spec + (size_t)t * 1024);
                    float v[16];
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const float4 a = sp[(512 * h + 8 * u) / 4], c = sp[(512 * h + 8 * u) / 4 + 1];
                        v[8 * h + 0] = a.x;
                        v[8 * h + 1] = a.y;
                        v[8 * h + 2] = a.z;
                        v[8 * h + 3] = a.w;
                        v[8 * h + 4] = c.x;
                        v[8 * h + 5] = c.y;
                        v[8 * h + 6] = c.z;
                        v[8 * h + 7] = c.w;
                    }
                    if (ch == 0) {
#pragma unroll
                        for (int e = 0; e < 16; e++) xL[e] += v[e];
                    } else {
                        if constexpr (stereo) {
#pragma unroll
                            for (int e = 0; e < 16; e++) xR[e] += v[e];
                        }
                    }
                }
            }

            STAMP(3);
            // both spectra to LDS (E/O layout): left in buf, right in rsp
            wave_sync();
            store_spec(W.buf, u, xL);
            if (stereo) store_spec(W.rsp, u, xR);
            wave_sync();
            STAMP(4);
            float outL[16], outR[16];
            if (stereo && iL.seq != JAAD_EIGHT_SHORT_SEQUENCE && iR.seq != JAAD_EIGHT_SHORT_SEQUENCE) {
                // the two long-window IMDCTs in lockstep: one set of LDS round trips, two chains
                if constexpr (kTnsSpec) {
                    if (A.tns_mode == JAAD_TNS_SPEC && A.tns) {
                        if (iL.flags & JAAD_ICS_TNS) tns_spec(W.buf, W.tns, T, *A.gtab, u, iL, A.tns + cf0);
                        if (iR.flags & JAAD_ICS_TNS) tns_spec(W.rsp, W.tns, T, *A.gtab, u, iR, A.tns + cf0 + 1);
                    }
                }
                if constexpr (kMode == 3) {
                    couple_after_tns(A, W.buf, f, 0, u);
                    couple_after_tns(A, W.rsp, f, 1, u);
                }
                float* const bufs[2] = {W.buf, W.rsp};
                f2 cx[2][8];
                imdct_long_pk<2, kFast>(bufs, T, lane_id(), cx);
                ola_long_pk<kFast>(T, FrameCtx{iL.seq, iL.shape, iL.shape_prev}, cx[0], ovL, outL);
                ola_long_pk<kFast>(T, FrameCtx{iR.seq, iR.shape, iR.shape_prev}, cx[1], ovR, outR);
                wave_sync();
            } else if (kShortPair && stereo && iL.seq == JAAD_EIGHT_SHORT_SEQUENCE && iR.seq == JAAD_EIGHT_SHORT_SEQUENCE) {
                // both channels' 8 short IMDCTs and overlap-adds in lockstep (mixed-window batches)
                float reL[8], imL[8], reR[8], imR[8];
                imdct_short_pk2<kFast>(W.buf, W.rsp, T, lane_id(), reL, imL, reR, imR);
                ola_short2(W.buf, W.rsp, T, lane_id(), FrameCtx{iL.seq, iL.shape, iL.shape_prev},
                           FrameCtx{iR.seq, iR.shape, iR.shape_prev}, reL, imL, reR, imR, ovL, ovR, outL, outR);
                wave_sync();
            } else {
                synth_channel<kTnsSpec, kMode == 3, kFast>(A, T, W, W.buf, iL, cf0, ovL, outL, f, 0);
                if (stereo) synth_channel<kTnsSpec, kMode == 3, kFast>(A, T, W, W.rsp, iR, cf0 + 1, ovR, outR, f, 1);
            }
            STAMP(8);
            // frame f+1's inputs (loaded since the IQ, a whole IMDCT ago) are in registers before
            // this frame's PCM stores are issued
            vmem_drain();
            STAMP(9);
            {
                const int u2 = lane_id();
                // a prefix frame's stores land past the frame's 4096-byte range (dropped by the
                // buffer resource); the offset is added as a wave-uniform value, not selected per
                // lane (a VOP2 v_cndmask costs ~4 VALU issue slots on gfx950)
                const int drop = emit ? 0 : 4096;
                if constexpr (planar) {
#pragma unroll
                    for (int o = 0; o < 16; o++) {
                        W.buf[long_pos(u2, o)] = kFast && kScaledOut ? outL[o] * kPcmScale : outL[o];
                        if (stereo) W.rsp[long_pos(u2, o)] = kFast && kScaledOut ? outR[o] * kPcmScale : outR[o];
                    }
                    wave_sync();
#pragma unroll
                    for (int c = 0; c < nch; c++) {
                        const __amdgpu_buffer_rsrc_t dst = frame_rsrc(reinterpret_cast<float*>(A.pcm) + (cf0 + c) * 1024, 4096);
                        const float* srcb = c ? W.rsp : W.buf;
#pragma unroll
                        for (int jj = 0; jj < 4; jj++)
                            store16(*reinterpret_cast<const v4u*>(srcb + 4 * u2 + 256 * jj), dst, 16 * u2 + 1024 * jj + drop, false);
                    }
                    wave_sync();
                } else if constexpr (out_f32) {  // tolerance/debug format: strided stores
                    // through a buffer resource over exactly the frame's 8192 bytes, as the int16
                    // form: a prefix frame's stores land past it and are dropped by the hardware,
                    // and no store of this form can leave its frame (round 6: it was the one LC
                    // output form whose addresses no resource bounded)
                    typedef unsigned v2u __attribute__((ext_vector_type(2)));
                    const __amdgpu_buffer_rsrc_t dst = frame_rsrc(reinterpret_cast<uint8_t*>(A.pcm) + (size_t)f * 8192, 8192);
                    const int drop8 = emit ? 0 : 8192;
#pragma unroll
                    for (int o = 0; o < 16; o++) {
                        const float sl = kFast && kScaledOut ? outL[o] * kPcmScale : outL[o];
                        const float sr = stereo ? (kFast && kScaledOut ? outR[o] * kPcmScale : outR[o]) : sl;
                        const v2u w = {__float_as_uint(sl), __float_as_uint(sr)};
                        __builtin_amdgcn_raw_buffer_store_b64(w, dst, 8 * long_pos(u2, o) + drop8, 0, 0);
                    }
                } else {
                    // word P = (L_P, R_P), staged in buf; big endian swaps the bytes of each sample.
                    // v_perm_b32(s0 = R pair, s1 = L pair): selector bytes 0-3 pick L, 4-7 pick R.
                    const uint32_t sel0 = big_endian ? 0x04050001u : 0x05040100u;
                    const uint32_t sel1 = big_endian ? 0x06070203u : 0x07060302u;
                    uint32_t* stage = reinterpret_cast<uint32_t*>(W.buf);
#ifdef JAAD_ABL_NOPCM
                    if (f < 0)  // never: the PCM stage's work and stores are left out (time only)
#endif
#pragma unroll
                    for (int m = 0; m < 8; m++) {
                        uint32_t pl, pr;
#if defined(JAAD_NO_PKNORM)  // (A/B builds: the exact rounding in the fused kernel too)
                        constexpr bool kPkNorm = false;
#else
                        constexpr bool kPkNorm = kFast;
#endif
                        if constexpr (kPkNorm) {
                            pl = round_pk16_lsb1(outL[2 * m], outL[2 * m + 1]);
                            pr = stereo ? round_pk16_lsb1(outR[2 * m], outR[2 * m + 1]) : pl;
                        } else if constexpr (kFast && kScaledOut) {
                            pl = round_pk16(outL[2 * m] * kPcmScale, outL[2 * m + 1] * kPcmScale);
                            pr = stereo ? round_pk16(outR[2 * m] * kPcmScale, outR[2 * m + 1] * kPcmScale) : pl;
                        } else {
                            pl = round_pk16(outL[2 * m], outL[2 * m + 1]);
                            pr = stereo ? round_pk16(outR[2 * m], outR[2 * m + 1]) : pl;
                        }
                        stage[long_pos(u2, 2 * m)] = __builtin_amdgcn_perm(pr, pl, sel0);
                        stage[long_pos(u2, 2 * m + 1)] = __builtin_amdgcn_perm(pr, pl, sel1);
                    }
                    wave_sync();
                    const __amdgpu_buffer_rsrc_t dst = frame_rsrc(reinterpret_cast<uint8_t*>(A.pcm) + (size_t)f * 4096, 4096);
#pragma unroll
                    for (int jj = 0; jj < 4; jj++)
                        store16(*reinterpret_cast<const v4u*>(stage + 4 * u2 + 256 * jj), dst, 16 * u2 + 1024 * jj + drop, true);
                    wave_sync();
                }
            }
            STAMP(10);
        }
        STAMP(11);
        reinterpret_cast<volatile uint32_t*>(S.rem)[wave] = 0u;  // (done: no longer ahead of its mates)
        if (cd.info & kChunkStoreState) {
            const int u = lane_id();
            float* st = A.state_out + (size_t)cd.slot * 2048;
            constexpr float sc = kFast && kScaledOut ? kPcmScale : 1.0f;
#pragma unroll
            for (int o = 0; o < 16; o++) {
                st[long_pos(u, o)] = kFast && kScaledOut ? ovL[o] * sc : ovL[o];
                if (stereo) st[1024 + long_pos(u, o)] = kFast && kScaledOut ? ovR[o] * sc : ovR[o];
            }
        }
    }
#ifdef JAAD_WAVETIME
    {   // profiling builds only: first/last s_memrealtime of each wave (scripts/wavetime.py)
        const uint64_t wt1 = __builtin_amdgcn_s_memrealtime();
        if (A.dbg && lane_id() == 0) {
            uint64_t* o = reinterpret_cast<uint64_t*>(A.dbg) + (size_t)(blockIdx.x * kW + wave) * 4;
            o[0] = wt0;
            o[1] = wt1;
            o[2] = (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID[3:0]
            o[3] = (uint64_t)wt_frames;
        }
    }
#endif
#ifdef JAAD_STAMPS
    if (A.dbg && lane_id() == 0) {
        uint32_t* o = reinterpret_cast<uint32_t*>(A.dbg) + (size_t)(blockIdx.x * kW + wave) * 16;
        for (int k = 0; k < 16; k++) o[k] = st_acc[k];
    }
#endif
}

template <int kMode, bool kStereo>
static void launch_lc_mode(const KernelArgs& a, hipStream_t stream)
{
    constexpr int W = waves_per_wg<kMode == 1 || kMode == 3>();
#define JAAD_LAUNCH(O) \
    hipLaunchKernelGGL((lc_decode_kernel<kMode, O, kStereo>), dim3((a.n_chunks + W - 1) / W), dim3(64 * W), 0, stream, a)
    const int o = (a.out_mode == kOutPlanarF32) ? 4 : (a.out_mode & JAAD_PCM_FLOAT32) ? 2 : (a.out_mode & JAAD_PCM_LITTLE_ENDIAN) ? 1 : 0;
    if (o == 4) JAAD_LAUNCH(kOutPlanarF32);
    else if (o == 2) JAAD_LAUNCH(JAAD_PCM_FLOAT32);
    else if (o == 1) JAAD_LAUNCH(JAAD_PCM_LITTLE_ENDIAN);
    else JAAD_LAUNCH(JAAD_PCM_BIG_ENDIAN);
#undef JAAD_LAUNCH
}

// The +-1 LSB instantiations (modes 4, 6) live in their own translation unit, jaad_lc_fast.hip (this
// file with JAAD_LC_FAST_TU), compiled with LLVM's iterative-ILP machine scheduler: -2.2 % on C2,
// -1.5 % on C3 (profiles/round6_ab/sched_itilp_c*.txt), while on the exact modes it spills
// (mode 0: 4 VGPRs, modes 1/3: 40+), so they keep the default scheduler.
hipError_t launch_lc_fast(const KernelArgs& a, hipStream_t stream);

#ifndef JAAD_LC_FAST_TU
template <bool kStereo>
static hipError_t launch_lc_ch(const KernelArgs& a, hipStream_t stream, bool tns_spec)
{
    if (a.cce_off && tns_spec) launch_lc_mode<3, kStereo>(a, stream);  // coupling around the spec TNS filters
    else if (a.cce_off) launch_lc_mode<2, kStereo>(a, stream);
    else if (tns_spec) launch_lc_mode<1, kStereo>(a, stream);
    else if (a.precision == JAAD_PRECISION_LSB1) return launch_lc_fast(a, stream);
    else {
        if constexpr (kStereo)
            if (a.short_pair) {
                launch_lc_mode<5, kStereo>(a, stream);
                return hipGetLastError();
            }
        launch_lc_mode<0, kStereo>(a, stream);
    }
    return hipGetLastError();
}

namespace {
// is batch frame f in one of the n dropped-frame runs of `skips` (KernelArgs::skips)?
__device__ __forceinline__ bool frame_skipped(const uint32_t* __restrict__ skips, uint32_t n, uint32_t f)
{
    uint32_t lo = 0, hi = n;  // first run starting after f
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (skips[2 * m] <= f) lo = m + 1;
        else hi = m;
    }
    return lo > 0 && f - skips[2 * (lo - 1)] < skips[2 * (lo - 1) + 1];
}

// one thread per (frame, sample instant): its n_ch planar samples -> n_ch interleaved outputs
// (dropped frames' PCM is left as it is)
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ planar, void* __restrict__ pcm,
                                                   uint32_t n_frames, int n_ch, uint32_t flags,
                                                   const uint32_t* __restrict__ skips, uint32_t n_skips)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // frame * 1024 + sample
    if (i >= (size_t)n_frames * 1024) return;
    const size_t f = i >> 10, n = i & 1023;
    if (n_skips && frame_skipped(skips, n_skips, (uint32_t)f)) return;
    const float* src = planar + f * (size_t)n_ch * 1024 + n;
    if (flags & JAAD_PCM_FLOAT32) {
        float* o = reinterpret_cast<float*>(pcm) + i * n_ch;
        for (int c = 0; c < n_ch; c++) o[c] = src[(size_t)c * 1024];
        return;
    }
    uint16_t* o = reinterpret_cast<uint16_t*>(pcm) + i * n_ch;
    for (int c = 0; c < n_ch; c++) {
        uint32_t s16 = round_pk16(src[(size_t)c * 1024], 0.0f) & 0xFFFFu;  // Math.round + clamp (as the LC PCM stage)
        if (!(flags & JAAD_PCM_LITTLE_ENDIAN)) s16 = ((s16 & 0xFF) << 8) | (s16 >> 8);
        o[c] = (uint16_t)s16;
    }
}
}  // namespace

namespace {
// 16 bytes (8 values) per thread and step, grid-stride over the range
__global__ __launch_bounds__(256) void check_q_kernel(const v4i* __restrict__ q, size_t n16, int* __restrict__ flag)
{
    int bad = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const v4i w = __builtin_nontemporal_load(q + i);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int lo = (int)(int16_t)(w[k] & 0xFFFF), hi = w[k] >> 16;
            bad |= (lo > 8190) | (lo < -8190) | (hi > 8190) | (hi < -8190);
        }
    }
    if (bad) *flag = 1;
}
}  // namespace

namespace {
// The addend of one coupling term: the CCE's ICStream spectrum as decodeSpectralData leaves it
// (A/syntax/ICStream.java:222-272: IQ x scalefactor gain, noise bands from the static LCG at the
// record's pns_state, ZERO / intensity bands 0) times the term's gain of the band, over the bins of
// the CCE's bands whose sfbCB != ZERO_HCB (CCE.applyDependentCoupling, A/syntax/CCE.java:188-215:
// data[k] += x * iqData[k]); every other bin -0.0, which leaves the target as it is.
__global__ __launch_bounds__(64) void cce_term_kernel(CceArgs A)
{
    __shared__ float buf[kWaveBuf];
    __shared__ uint32_t raw[64];
    const uint32_t t = blockIdx.x;
    if (t >= A.n_terms) return;
    const int u = lane_id();
    const LdsTables& T = *A.tables;
    const uint32_t rec = A.meta[t] & 0xFFFFu;
    const jaad_ics_info ic = A.ics[rec];
    Ics info;
    info.seq = ic.window_sequence & 3;
    info.shape = ic.window_shape & 1;
    info.shape_prev = ic.window_shape_prev & 1;
    const int lim = info.seq == JAAD_EIGHT_SHORT_SEQUENCE ? T.nswb_s : T.nswb_l;
    info.max_sfb = min((int)ic.max_sfb, lim);
    info.grouping = ic.grouping;
    info.flags = ic.flags;
    info.pns = ic.pns_state;
    const int groups = info.seq == JAAD_EIGHT_SHORT_SEQUENCE ? 8 - __builtin_popcount(info.grouping & 0x7f) : 1;
    info.nbands = groups * info.max_sfb;
    raw[u] = reinterpret_cast<const uint32_t*>(u < 32 ? A.sf + (size_t)rec * 128 : A.cb + (size_t)rec * 128)[u & 31];
    wave_sync();
    const uint8_t* sfr = reinterpret_cast<const uint8_t*>(raw);
    const uint8_t* cbr = sfr + 128;
    const int16_t* q = A.q + (size_t)rec * 1024;
    const float* gain = A.gain + (size_t)t * 120;
    float x[16], g[16];
    bool touched[16];
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const int p = 512 * (e >> 3) + 8 * u + (e & 7);
        int band = kNoBand;
        if (info.seq == JAAD_EIGHT_SHORT_SEQUENCE) {
            band = band_short(T, info, p & ~3);
        } else {
            const int b = T.quad2band_l[p >> 2];
            band = b < info.max_sfb ? b : kNoBand;
        }
        x[e] = 0.0f;
        g[e] = 0.0f;
        touched[e] = false;
        if (band == kNoBand) continue;
        const int c = cbr[band];
        touched[e] = c != JAAD_ZERO_HCB;
        g[e] = gain[band];
        if (c != JAAD_ZERO_HCB && c < JAAD_NOISE_HCB) {
            const int v = q[p];
            const int a = min(v < 0 ? -v : v, 8190);
            const float iq = v > 0 ? A.iq_table[a] : -A.iq_table[a];
            x[e] = iq * T.sf_gain[sfr[band]];
        }
    }
    if (info.flags & JAAD_ICS_HAS_PNS) {
        wave_sync();
        store_spec(buf, u, x);
        wave_sync();
        pns_fill(buf, raw, T, *A.gtab, u, info);
        load_spec(buf, u, x);
    }
    float* out = A.spec + (size_t)t * 1024;
#pragma unroll
    for (int e = 0; e < 16; e++) out[512 * (e >> 3) + 8 * u + (e & 7)] = touched[e] ? g[e] * x[e] : -0.0f;
}
}  // namespace

hipError_t launch_cce_terms(const CceArgs& a, hipStream_t stream)
{
    if (!a.n_terms) return hipSuccess;
    hipLaunchKernelGGL(cce_term_kernel, dim3(a.n_terms), dim3(64), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_check_q(const int16_t* q, size_t n, int* flag, hipStream_t stream)
{
    const size_t n16 = n / 8;  // q rows are 1024 values: whole 16-byte words
    if (!n16) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<size_t>((n16 + 255) / 256, 2048);
    hipLaunchKernelGGL(check_q_kernel, dim3(blocks), dim3(256), 0, stream, reinterpret_cast<const v4i*>(q), n16, flag);
    return hipGetLastError();
}

namespace {
// one thread per (frame, sample instant): the output channels' words from the elements' PCM
template <typename W>
__global__ __launch_bounds__(256) void mc_interleave_kernel(McInterleave m, W* __restrict__ out, size_t n,
                                                            uint32_t samples, const uint32_t* __restrict__ skips,
                                                            uint32_t n_skips)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // frame * samples + sample
    if (i >= n) return;
    if (n_skips && frame_skipped(skips, n_skips, (uint32_t)(i / samples))) return;  // dropped frame
    W* o = out + i * m.n_out;
    for (int c = 0; c < m.n_out; c++) o[c] = static_cast<const W*>(m.src[c])[2 * i + m.chan[c]];
}
}  // namespace

hipError_t launch_mc_interleave(const McInterleave& m, void* pcm, uint32_t n_frames, uint32_t samples, int bps,
                                hipStream_t stream, const uint32_t* skips, uint32_t n_skips)
{
    const size_t n = (size_t)n_frames * samples;
    if (!n) return hipSuccess;
    if (m.n_out < 1 || m.n_out > 16) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (bps == 4)
        hipLaunchKernelGGL(mc_interleave_kernel<uint32_t>, grid, dim3(256), 0, stream, m, static_cast<uint32_t*>(pcm), n,
                           samples, skips, n_skips);
    else
        hipLaunchKernelGGL(mc_interleave_kernel<uint16_t>, grid, dim3(256), 0, stream, m, static_cast<uint16_t*>(pcm), n,
                           samples, skips, n_skips);
    return hipGetLastError();
}

hipError_t launch_pack(const float* planar, void* pcm, uint32_t n_frames, int n_ch, uint32_t flags, hipStream_t stream,
                       const uint32_t* skips, uint32_t n_skips)
{
    const size_t n = (size_t)n_frames * 1024;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, planar, pcm, n_frames, n_ch,
                       flags, skips, n_skips);
    return hipGetLastError();
}

hipError_t launch_lc(const KernelArgs& a, hipStream_t stream, bool tns_spec)
{
    return a.nch == 2 ? launch_lc_ch<true>(a, stream, tns_spec) : launch_lc_ch<false>(a, stream, tns_spec);
}

int lc_resident_waves_per_cu(bool tns_spec)
{
    int blocks = 0;
    hipError_t e = tns_spec ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, lc_decode_kernel<1, JAAD_PCM_BIG_ENDIAN, true>,
                                                                            64 * waves_per_wg<true>(), 0)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, lc_decode_kernel<0, JAAD_PCM_BIG_ENDIAN, true>,
                                                                            64 * waves_per_wg<false>(), 0);
    if (e != hipSuccess) return 0;
    return blocks * (tns_spec ? waves_per_wg<true>() : waves_per_wg<false>());
}
#else  // JAAD_LC_FAST_TU
hipError_t launch_lc_fast(const KernelArgs& a, hipStream_t stream)
{
    // (the lockstep short path pairs a CPE's channels: stereo only)
    if (a.nch == 2) {
        if (a.short_pair) launch_lc_mode<6, true>(a, stream);
        else launch_lc_mode<4, true>(a, stream);
    } else {
        launch_lc_mode<4, false>(a, stream);
    }
    return hipGetLastError();
}
#endif

}  // namespace jaad
