// SBR (HE-AAC v1) signal path for gfx950, A/ = aac/src/main/java/net/sourceforge/jaad/aac/ of the
// reference.  Every binary32 expression keeps the Java evaluation order (the library is built with
// -ffp-contract=off; divisions and square roots are correctly rounded), so the output is
// bit-identical to the oracle's restatement.
//
// The per-channel state the Java carries from frame to frame (analysis ring, Xsbr rows 0..7,
// synthesis v ring, G/Q ring) only reaches back one frame, so every stage is frame-parallel: it
// reads what it needs of frame f-1 from the previous stage's output in HBM (or, for the first
// frame of a run, from the slot state) instead of waiting for it:
//   sbr_analysis_kernel   one wave per ch-frame: QMF analysis, 2 slots per pass
//   sbr_hf_kernel         one wave per ch-frame, lane = QMF band: HF generation, envelope
//                         estimation, gains, assembly
//   sbr_synthesis_kernel  one wave per chunk of kSbrSynFrames frames (9 history slots recomputed)
//   sbr_state_kernel      last frame of each run -> slot state
// A 32-point DCT-IV (A/sbr/DCT.java) is spread over 32 lanes, one complex point per lane; the
// radix-2 DIF stages exchange partners with v_permlane16_swap (xor 16) and DPP (xor 8..1).
#include <hip/hip_runtime.h>

#include <utility>

#include "jaad_sbr.h"
#define JAAD_DCT32_TABLE static constexpr
#include "tables/jaad_sbr_dct32.inc"
#include "jaad_wave.h"

namespace jaad {
namespace {

struct HfLds {
    float ecurr[5][64];
    float gl[5][64], ql[5][64], sl[5][64];
    float gq_eo[64];                        // per-envelope E_orig of band m
    float den_s[64], den_e[64], den_q[64];  // per-band terms of the limiter band's den sum
    float lim_gmax[64], lim_acc1[64], lim_boost[64];  // per limiter band
    SbrRec rec;                             // the channel-frame's record and its band tables,
    SbrTab tab;                             // copied once (see sbr_hf_kernel)
};
static_assert(sizeof(SbrRec) % 4 == 0 && sizeof(SbrTab) % 4 == 0, "record copies are dword-wise");
// the fused analysis (sbr_hf_kernel<5>) stages its 1568-sample window in the gain-stage scratch and
// reads SbrRec::first / ::slot from the record's dwords 2 (byte 3) and 16
static_assert(offsetof(HfLds, rec) - offsetof(HfLds, ecurr) >= 1568 * sizeof(float), "analysis window in the gain scratch");
static_assert(offsetof(SbrRec, first) == 11 && offsetof(SbrRec, slot) == 64, "SbrRec dwords read by readlane");

// Math.round + short clamp (S/SampleBuffer.java:190-205)
__device__ __forceinline__ int java_round16(float s)
{
    if (s != s) return 0;
    const float fl = floorf(s);
    int r = (s - fl) >= 0.5f ? (int)fl + 1 : (int)fl;
    if (s >= 2147483648.0f) r = 2147483647;
    if (s <= -2147483648.0f) r = (int)0x80000000;
    return r > 32767 ? 32767 : (r < -32768 ? -32768 : r);
}

// The same as a 16-bit word pair (s16, s16), byte-swapped within each half when swap: NaN -> 0,
// then v_cvt_rpi_i32_f32 = (int)floor(x + 0.5) evaluated exactly, which is Math.round for every
// non-NaN float (saturating like Java's int conversion; exhaustive check on MI355X,
// tools/probe_round.hip), and v_cvt_pk_i16_i32's int16 saturation is SampleBuffer's clamp.
__device__ __forceinline__ uint32_t java_round16_pair(float s, bool swap)
{
    const float v = s != s ? 0.0f : s;
    int i;
    uint32_t w;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(i) : "v"(v));
    asm("v_cvt_pk_i16_i32 %0, %1, %1" : "=v"(w) : "v"(i));
    return swap ? __builtin_amdgcn_perm(w, w, 0x02030001u) : w;
}

__device__ __forceinline__ float java_minf(float a, float b)
{
    if (a != a) return a;
    if (a == 0.0f && b == 0.0f) return __float_as_uint(a) >> 31 ? a : b;
    return a <= b ? a : b;
}

// per-lane constants of a 32-point DCT-IV (A/sbr/DCT.java:347-391): lane e's butterfly twiddles
// and the post-modulation constants of the output element E the lane returns
struct DctConst {
    float t0, t32, t64;        // pre-modulation (element e)
    float t96, t128, t160;     // post-modulation (element E)
    float w1r, w1i, w2r, w2i;  // stage 1/2 twiddles of the bottom lanes
    float w3;                  // stage 3 constant (w[4] or w[12])
};

__device__ __forceinline__ DctConst load_dct_const(const float* dct, int e, int E)
{
    DctConst K;
    const float* wr = dct + 192;
    const float* wi = dct + 208;
    K.t0 = dct[e];
    K.t32 = dct[e + 32];
    K.t64 = dct[e + 64];
    K.t96 = dct[E + 96];
    K.t128 = dct[E + 128];
    K.t160 = dct[E + 160];
    K.w1r = wr[e & 15];
    K.w1i = wi[e & 15];
    K.w2r = wr[2 * (e & 7)];
    K.w2i = wi[2 * (e & 7)];
    K.w3 = (e & 3) == 1 ? wr[4] : wr[12];
    return K;
}

// DCT.dct4_kernel distributed over the 32 lanes of a half-wave: (xr, xi) = input element e.  Each
// stage performs, per element, exactly the operation the sequential Java loop performs on it; the
// butterfly partners come through DPP (lane ^ 1, 2, 4, 8) and v_permlane16_swap (lane ^ 16), not
// LDS.  The Java post-modulation reads the stage outputs in bit-reversed order (:368-389); here
// they stay where the stages leave them, so lane e returns output element E = bitrev5(e)
// (K = load_dct_const(dct, e, E)).  N independent transforms run in lockstep.
template <int N>
__device__ __forceinline__ void dct4_n(const DctConst& K, int e, int E, const float (&xr)[N], const float (&xi)[N],
                                       float (&orr)[N], float (&oi)[N])
{
    float r[N], i[N];
#pragma unroll
    for (int n = 0; n < N; n++) {
        const float tmp = (xr[n] + xi[n]) * K.t0;
        r[n] = (xi[n] * K.t64) + tmp;
        i[n] = (xr[n] * K.t32) + tmp;
    }
    // stage 1 (DCT.java:143-164): pairs (i, i+16)
    {
        float pr[N], pi[N];
#pragma unroll
        for (int n = 0; n < N; n++) {
            pr[n] = xor16(r[n], e);
            pi[n] = xor16(i[n], e);
        }
#pragma unroll
        for (int n = 0; n < N; n++) {
            if (e < 16) {
                r[n] = r[n] + pr[n];
                i[n] = i[n] + pi[n];
            } else {
                const float tr = pr[n] - r[n], ti = pi[n] - i[n];
                r[n] = (tr * K.w1r) - (ti * K.w1i);
                i[n] = (tr * K.w1i) + (ti * K.w1r);
            }
        }
    }
    // stage 2 (:166-207): pairs (i, i+8) in each 16-group, twiddle w[2j]
    {
        float pr[N], pi[N];
#pragma unroll
        for (int n = 0; n < N; n++) {
            pr[n] = swz<8>(r[n]);
            pi[n] = swz<8>(i[n]);
        }
#pragma unroll
        for (int n = 0; n < N; n++) {
            if (!(e & 8)) {
                r[n] = r[n] + pr[n];
                i[n] = i[n] + pi[n];
            } else {
                const float tr = pr[n] - r[n], ti = pi[n] - i[n];
                r[n] = (tr * K.w2r) - (ti * K.w2i);
                i[n] = (tr * K.w2i) + (ti * K.w2r);
            }
        }
    }
    // stage 3 (:212-287): pairs (i, i+4) in each 8-group; four bottom variants
    {
        float pr[N], pi[N];
#pragma unroll
        for (int n = 0; n < N; n++) {
            pr[n] = swz<4>(r[n]);
            pi[n] = swz<4>(i[n]);
        }
#pragma unroll
        for (int n = 0; n < N; n++) {
            if (!(e & 4)) {
                r[n] = r[n] + pr[n];
                i[n] = i[n] + pi[n];
            } else {
                const int v = e & 3;
                const float tr = pr[n] - r[n], ti = pi[n] - i[n];
                if (v == 0) {
                    r[n] = tr;
                    i[n] = ti;
                } else if (v == 1) {
                    const float a = tr + ti, b = ti - tr;
                    r[n] = a * K.w3;
                    i[n] = b * K.w3;
                } else if (v == 2) {
                    const float nr = ti, ni = r[n] - pr[n];
                    r[n] = nr;
                    i[n] = ni;
                } else {
                    const float a = tr - ti, b = tr + ti;
                    r[n] = a * K.w3;
                    i[n] = b * K.w3;
                }
            }
        }
    }
    // stage 4 (:291-322): pairs (i, i+2) in each 4-group
    {
        float pr[N], pi[N];
#pragma unroll
        for (int n = 0; n < N; n++) {
            pr[n] = swz<2>(r[n]);
            pi[n] = swz<2>(i[n]);
        }
#pragma unroll
        for (int n = 0; n < N; n++) {
            if (!(e & 2)) {
                r[n] = r[n] + pr[n];
                i[n] = i[n] + pi[n];
            } else if (!(e & 1)) {
                r[n] = pr[n] - r[n];
                i[n] = pi[n] - i[n];
            } else {
                const float nr = pi[n] - i[n], ni = r[n] - pr[n];
                r[n] = nr;
                i[n] = ni;
            }
        }
    }
    // stage 5 (:326-341): pairs (i, i+1)
    {
        float pr[N], pi[N];
#pragma unroll
        for (int n = 0; n < N; n++) {
            pr[n] = swz<1>(r[n]);
            pi[n] = swz<1>(i[n]);
        }
#pragma unroll
        for (int n = 0; n < N; n++) {
            if (!(e & 1)) {
                r[n] = r[n] + pr[n];
                i[n] = i[n] + pi[n];
            } else {
                r[n] = pr[n] - r[n];
                i[n] = pi[n] - i[n];
            }
        }
    }
    // post-modulation of output element E, whose bit-reversed input the stages left in this lane
#pragma unroll
    for (int n = 0; n < N; n++) {
        if (E == 16) {
            orr[n] = (r[n] + i[n]) * K.t96;
            oi[n] = (i[n] - r[n]) * K.t96;
        } else {
            const float t = (r[n] + i[n]) * K.t96;
            orr[n] = (i[n] * K.t160) + t;
            oi[n] = (r[n] * K.t128) + t;
        }
    }
}

__device__ __forceinline__ void dct4(const DctConst& K, int e, int E, float xr, float xi, float& orr, float& oi)
{
    const float a[1] = {xr}, b[1] = {xi};
    float o1[1], o2[1];
    dct4_n<1>(K, e, E, a, b, o1, o2);
    orr = o1[0];
    oi = o2[0];
}

// Two 32-point DCT-IVs per half-wave, packed: the same transform of two slots (slot 0, slot 1)
// whose element e sits in lane e as a float2 (xr, xi) -- v_pk_* arithmetic does both slots at
// once.  Stage 1's xor-16 exchange is a single v_permlane16_swap of the two slots' registers: it
// leaves lanes 0..15 holding both partners (j, j+16) of slot 0 and lanes 16..31 both partners of
// slot 1, so from stage 1 on lane j (+16) computes positions j (S) and j + 16 (D) of one slot, with
// the same twiddles as before (they depend on j only), and no exchange crosses 16 lanes again.
// Outputs: (orr, oi).x = output element E_S = bitrev5(j), .y = element E_S + 1, of slot e >> 4.
// Every element sees exactly the binary32 operations of dct4_n.
typedef float f2 __attribute__((ext_vector_type(2)));
struct DctPairConst {
    float t0, t32, t64;     // pre-modulation (element e, both slots)
    float w1r, w1i, w2r, w2i, w3;
    f2 t96, t128, t160;     // post-modulation of elements E_S (x) and E_S + 1 (y)
};
__device__ __forceinline__ DctPairConst load_dct_pair_const(const float* dct, int e)
{
    const DctConst K = load_dct_const(dct, e, 0);
    const int es = bitrev5(e & 15);
    DctPairConst P;
    P.t0 = K.t0;
    P.t32 = K.t32;
    P.t64 = K.t64;
    P.w1r = K.w1r;
    P.w1i = K.w1i;
    P.w2r = K.w2r;
    P.w2i = K.w2i;
    P.w3 = K.w3;
    P.t96 = f2{dct[es + 96], dct[es + 97]};
    P.t128 = f2{dct[es + 128], dct[es + 129]};
    P.t160 = f2{dct[es + 160], dct[es + 161]};
    return P;
}
// (xor 4 through the LDS crossbar, ds_swizzle bit mode: one instruction instead of two DPP moves)
template <int kXor>
__device__ __forceinline__ float swz_x(float v)
{
    if constexpr (kXor == 4) return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (4 << 10)));
    else return swz<kXor>(v);
}
template <int kXor>
__device__ __forceinline__ f2 swz2(f2 v) { return f2{swz_x<kXor>(v.x), swz_x<kXor>(v.y)}; }

__device__ __forceinline__ void dct4_pair(const DctPairConst& K, int e, f2 xr, f2 xi, f2& orr, f2& oi)
{
    const f2 tmp = (xr + xi) * K.t0;
    const f2 r0 = (xi * K.t64) + tmp;
    const f2 i0 = (xr * K.t32) + tmp;
    // stage 1 (DCT.java:143-164), transposed: A = position j, B = position j + 16 of this lane's slot
    const auto sr = __builtin_amdgcn_permlane16_swap(__float_as_int(r0.x), __float_as_int(r0.y), false, false);
    const auto si = __builtin_amdgcn_permlane16_swap(__float_as_int(i0.x), __float_as_int(i0.y), false, false);
    const f2 A = f2{__int_as_float(sr[0]), __int_as_float(si[0])}, B = f2{__int_as_float(sr[1]), __int_as_float(si[1])};
    const f2 sum = A + B, dif = A - B;
    // (r, i).x = position j, .y = position j + 16
    f2 r = f2{sum.x, (dif.x * K.w1r) - (dif.y * K.w1i)};
    f2 i = f2{sum.y, (dif.x * K.w1i) + (dif.y * K.w1r)};
    // stage 2 (:166-207): pairs (i, i+8) in each 16-group, twiddle w[2j]
    {
        const f2 pr = swz2<8>(r), pi = swz2<8>(i);
        if (!(e & 8)) {
            r = r + pr;
            i = i + pi;
        } else {
            const f2 tr = pr - r, ti = pi - i;
            r = (tr * K.w2r) - (ti * K.w2i);
            i = (tr * K.w2i) + (ti * K.w2r);
        }
    }
    // stage 3 (:212-287): pairs (i, i+4) in each 8-group; four bottom variants
    {
        const f2 pr = swz2<4>(r), pi = swz2<4>(i);
        if (!(e & 4)) {
            r = r + pr;
            i = i + pi;
        } else {
            const int v = e & 3;
            const f2 tr = pr - r, ti = pi - i;
            if (v == 0) {
                r = tr;
                i = ti;
            } else if (v == 1) {
                r = (tr + ti) * K.w3;
                i = (ti - tr) * K.w3;
            } else if (v == 2) {
                const f2 ni = r - pr;
                r = ti;
                i = ni;
            } else {
                r = (tr - ti) * K.w3;
                i = (tr + ti) * K.w3;
            }
        }
    }
    // stage 4 (:291-322): pairs (i, i+2) in each 4-group
    {
        const f2 pr = swz2<2>(r), pi = swz2<2>(i);
        if (!(e & 2)) {
            r = r + pr;
            i = i + pi;
        } else if (!(e & 1)) {
            r = pr - r;
            i = pi - i;
        } else {
            const f2 nr = pi - i, ni = r - pr;
            r = nr;
            i = ni;
        }
    }
    // stage 5 (:326-341): pairs (i, i+1): x + p on even lanes, p - x on odd ones, as p + (x * +-1)
    // (a sign flip is exact and + commutes: the same binary32 results, no select)
    {
        const f2 pr = swz2<1>(r), pi = swz2<1>(i);
        const float sg = (e & 1) ? -1.0f : 1.0f;
        r = pr + (r * sg);
        i = pi + (i * sg);
    }
    // post-modulation; element 16 (E_S of j == 1) has its own form
    const f2 t = (r + i) * K.t96;
    orr = (i * K.t160) + t;
    oi = (r * K.t128) + t;
    if ((e & 15) == 1) oi.x = (i.x - r.x) * K.t96.x, orr.x = t.x;
}

constexpr int kWavesPerBlock = 4;

using gfloat = const __attribute__((address_space(1))) float;  // global memory (never flat)

// s_waitcnt vmcnt(0) the compiler's wait insertion sees (see the synthesis kernel)
__device__ __forceinline__ void vmem_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0) expcnt(7) lgkmcnt(15)

// batch frame / batch ch-frame of a record (frame) / record ch-frame (SbrArgs::fmap)
__device__ __forceinline__ size_t batch_frame(const SbrArgs& A, size_t rf) { return A.fmap ? (size_t)A.fmap[rf] : rf; }
__device__ __forceinline__ size_t batch_cf(const SbrArgs& A, size_t rcf)
{
    return A.fmap ? (size_t)A.fmap[rcf / (uint32_t)A.nch] * A.nch + rcf % (uint32_t)A.nch : rcf;
}

// ---------------------------------------------------------------------------------------------
// AnalysisFilterbank.sbr_qmf_analysis_32 (A/sbr/AnalysisFilterbank.java:9-73)
// ---------------------------------------------------------------------------------------------
static_assert(sizeof(SbrChState) % 16 == 0 && offsetof(SbrChState, tail) % 16 == 0, "analysis reads tail as float4");

// One pass of the analysis: slot 32-sample block l = 2p + half of the frame whose sample g is
// smp(g) (g may be negative: the samples before the frame), band e of it in lane (half, e) as
// (re, im), zero from band kx up.  Shared by sbr_analysis_kernel and the fused HF kernel.
struct QmfCoefs {
    float ca[5], cb[5];
};
__device__ __forceinline__ QmfCoefs load_qmf_coefs(const float* qmf_c, int e)
{
    QmfCoefs Q;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        Q.ca[j] = qmf_c[2 * (e + 64 * j)];
        Q.cb[j] = qmf_c[2 * (e + 32 + 64 * j)];
    }
    return Q;
}
template <class Smp>
__device__ __forceinline__ float2 qmf_analysis_pass(Smp smp, int l, int e, int hb, int E, const DctConst& K,
                                                    const QmfCoefs& Q, int kx)
{
    // v[v_index + x] = sample (32 l + 31 - x); u[n] = sum_j v[n + 64 j] * c[2 (n + 64 j)]  (:19-30)
    const int base = 32 * l + 31;
    float ulo, uhi;
    {
        const float a0 = smp(base - e) * Q.ca[0], a1 = smp(base - e - 64) * Q.ca[1];
        const float a2 = smp(base - e - 128) * Q.ca[2], a3 = smp(base - e - 192) * Q.ca[3];
        const float a4 = smp(base - e - 256) * Q.ca[4];
        ulo = (((a0 + a1) + a2) + a3) + a4;
        const int n = e + 32;
        const float b0 = smp(base - n) * Q.cb[0], b1 = smp(base - n - 64) * Q.cb[1];
        const float b2 = smp(base - n - 128) * Q.cb[2], b3 = smp(base - n - 192) * Q.cb[3];
        const float b4 = smp(base - n - 256) * Q.cb[4];
        uhi = (((b0 + b1) + b2) + b3) + b4;
    }
    // in_real[0] = u[0], in_real[n] = -u[64-n]; in_imag[m] = u[32-m]  (:39-46)
    const int src = hb + ((32 - e) & 31);
    const float slo = shfl(ulo, src), shi = shfl(uhi, src);
    const float in_r = e == 0 ? ulo : -shi;
    const float in_i = e == 0 ? uhi : slo;
    float orr, oi;
    dct4(K, e, E, in_r, in_i, orr, oi);
    // X[2n] = 2 out[n], X[2n+1] = -2 swap(out[31-n]) (:52-71): lane (half, k) holds band k of slot
    // 2p + half (the DCT left output element m in lane bitrev5(m))
    const int k = e;
    const int srcl = hb + bitrev5((k & 1) ? 31 - (k >> 1) : (k >> 1));
    const float vr = shfl(orr, srcl), vi = shfl(oi, srcl);
    float re = 0.0f, im = 0.0f;
    if (k < kx) {
        if (k & 1) {
            re = -2.0f * vi;
            im = -2.0f * vr;
        } else {
            re = 2.0f * vr;
            im = 2.0f * vi;
        }
    }
    return make_float2(re, im);
}

__global__ __launch_bounds__(256) void sbr_analysis_kernel(SbrArgs A)
{
    __shared__ __attribute__((aligned(16))) float win_s[kWavesPerBlock][288 + 1024];  // the 288 samples before the frame + the frame
    const uint32_t cf = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (cf >= A.n_cf) return;
    float* win = win_s[threadIdx.x >> 6];
    const int u = lane_id();
    const int e = u & 31, half = u >> 5, hb = half << 5;
    const int c = (int)(cf % (uint32_t)A.nch);
    const SbrRec& R = A.recs[cf];
    const int kx = (R.flags & kSbrProcess) ? A.tabs[R.table].kx : 32;
    const float* cur = A.time + batch_cf(A, cf) * 1024;
    // samples before the frame: previous record of the run, or the slot state (first record)
    const float* prev = R.first ? A.state[(size_t)R.slot * 2 + c].tail : A.time + batch_cf(A, cf - A.nch) * 1024 + 736;
    const int E = bitrev5(e);
    const DctConst K = load_dct_const(A.dct, e, E);
    const QmfCoefs Q = load_qmf_coefs(A.qmf_c, e);
    // the window's 1312 samples are staged in LDS with coalesced loads; the 160 taps per lane are
    // LDS reads (consecutive lanes, consecutive addresses)
    // (16-byte loads: tail and frame offsets are multiples of 4 floats, sizeof(SbrChState) of 16 B)
    {
        const float4* p4 = reinterpret_cast<const float4*>(prev);
        const float4* c4 = reinterpret_cast<const float4*>(cur);
        float4* w4 = reinterpret_cast<float4*>(win);
        for (int i = u; i < (288 + 1024) / 4; i += 64) w4[i] = i < 72 ? p4[i] : c4[i - 72];
    }
    wave_sync();
    auto smp = [&](int g) { return win[288 + g]; };
    float* out = A.xlow + (size_t)cf * 32 * 32 * 2;
    for (int p = 0; p < 16; p++)
        reinterpret_cast<float2*>(out)[(2 * p + half) * 32 + e] = qmf_analysis_pass(smp, 2 * p + half, e, hb, E, K, Q, kx);
}

// ---------------------------------------------------------------------------------------------
// Packed complex arithmetic of the HF kernel: a complex value is an f2 (re, im) in a VGPR pair and
// one VOP3P instruction makes both halves, each one correctly rounded binary32 operation (no
// contraction), so the results are the scalar expressions' bits.  op_sel / op_sel_hi pick the half
// of each source that feeds the lo / hi result, neg_lo / neg_hi negate it (a - b == a + (-b)).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ f2 pk_mul_xa(f2 a, f2 b)  // (a.x * b.x, a.y * b.x)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 pk_mul_ya(f2 a, f2 b)  // (a.y * b.y, a.x * b.y)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 pk_mul_bx(f2 g, f2 v)  // (g.x * v.x, g.x * v.y)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(g), "v"(v));
    return r;
}
__device__ __forceinline__ f2 pk_mul_by(f2 g, f2 v)  // (g.y * v.x, g.y * v.y)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(g), "v"(v));
    return r;
}
__device__ __forceinline__ f2 pk_add_nhi(f2 a, f2 b)  // (a.x + b.x, a.y - b.y)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 pk_add_nlo(f2 a, f2 b)  // (a.x - b.x, a.y + b.y)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 pk_add(f2 a, f2 b)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 pk_mul(f2 a, f2 b)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (t.re * c.re + t.im * c.im, t.im * c.re - t.re * c.im): one autocorrelation term of
// HFGeneration.calculate_lpc (t * conj(c), the Java's operand order)
__device__ __forceinline__ f2 pk_mul_conj(f2 t, f2 c) { return pk_add_nhi(pk_mul_xa(t, c), pk_mul_ya(t, c)); }
// two row loads of the HF kernel through a buffer resource: a lane whose offset is past the
// resource reads (0, 0), which is the reference's zero above the analysed bands
__device__ __forceinline__ f2 load_row_pair(__amdgpu_buffer_rsrc_t r, int off)
{
    return __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// ---------------------------------------------------------------------------------------------
// Channel.process_channel HF part: HFGeneration + HFAdjustment (A/sbr/Channel.java:596-604)
// phase 0: full; phase 1: gains and G/Q ring only; phase 2: full, ring from frame f-1
// ---------------------------------------------------------------------------------------------
// JAAD_HF_STAMPS builds (scripts/hf_stamps.py): s_memtime at the phase boundaries of each
// phase-0 channel-frame, lane 0 stores them to dbg[cf][16] (u64); the debug buffer is attached by
// jaad__sbr_debug_attach.  Product builds compile them out.
#if defined(JAAD_HF_STAMPS)
#define HF_STAMP(k)                                        \
    do {                                                   \
        __builtin_amdgcn_sched_barrier(0);                 \
        hf_t[k] = __builtin_amdgcn_s_memtime();            \
        __builtin_amdgcn_sched_barrier(0);                 \
    } while (0)
#else
#define HF_STAMP(k) \
    do {            \
    } while (0)
#endif
// phase 3: fix pass over the listed channel-frames; phase 4: chain walker, one wave per chain
// stepping its frames in order (each one a phase-3 frame reading the frame before it)
template <int kPhase>
__global__ __launch_bounds__(256, 3) void sbr_hf_kernel(SbrArgs A)
{
    // phase 5: phase 0 with the QMF analysis fused in (launches without smoothing and without fix
    // passes, launch_sbr): the rows come from the core time samples in registers, not from X_low
    // in HBM (no sbr_analysis_kernel, no X_low round trip)
    constexpr bool kFused = kPhase == 5;
    constexpr int P = kPhase == 4 ? 3 : kFused ? 0 : kPhase;  // the body's phase
#if defined(JAAD_HF_STAMPS)
    uint64_t hf_t[16] = {};
#endif
    HF_STAMP(0);
    __shared__ HfLds Ls[kWavesPerBlock];
    __shared__ float2 noise_s[512];  // NoiseTable.NOISE_TABLE (A/sbr/NoiseTable.java:6), read per slot
    static_assert(kWavesPerBlock * 64 * 2 == 512, "two noise entries per thread");
    const int wave = threadIdx.x >> 6;
    const int u = lane_id();
    uint32_t cf = blockIdx.x * kWavesPerBlock + wave;
    uint32_t n_iter = 1, o = 0;
    bool live = true;  // (every wave reaches the barrier below)
    if constexpr (kPhase == 4) {
        live = cf < A.n_chains;
        if (live) {
            o = A.chains[2 * cf];
            n_iter = A.chains[2 * cf + 1];
        }
    } else if constexpr (kPhase == 3) {  // fix pass: the listed channel-frames only
        live = cf < A.n_fix;
        if (live) cf = A.fix[cf];
    } else {
        live = cf < A.n_cf;
    }
    HfLds& L = Ls[wave];
    // Xsbr of this lane's band (sbr_save_matrix, A/sbr/SBR.java:286-300, then the analysis at
    // offset tHFGen = 8).  Rows 0..7 are rows 32..39 of frame f-1 AFTER its HF adjustment: below
    // kx_prev its analysis slots 24..31, from kx_prev up the high band it adjusted (rows 32, 33
    // always, 34.. when its last envelope ends past slot 32).  That high band is frame f-1's own
    // output of this launch, so this pass takes rows 0..7 from the analysis alone (bands < kx_prev,
    // zero above) -- exact unless the frame reads the high band (source band >= kx_prev, kx above
    // kx_prev or a band without patch with rows 2..7 carried: kSbrDep, jaad_sbr_host.cpp); those
    // frames run again in fix passes (kPhase 3) that read frame f-1's finished carry rows.  The
    // first frame of a run reads the slot state's carry rows (exact).  Rows 8..39 = this frame's
    // analysis slots 0..31 (zero from kx up).
    // The loads need nothing from the record: they are issued first, beside the record and table
    // copies (rows 0..7 from the previous channel-frame; a run's first record replaces them with the
    // slot state's rows once it has arrived) -- one global round trip before the record instead of
    // one after it.  (x[r] = (re, im) of row r: the packed complex arithmetic below works on pairs.)
    f2 x[40];
    // lanes past a resource's bands read (0, 0) without a select (bands >= 32, or >= kp)
    auto load_rows = [&](float* base, int r0, int nrows, int kp, int row_bytes) {
        // (the address is wave-uniform; readfirstlane says so, else every load became a waterfall loop)
        const uint64_t a = reinterpret_cast<uint64_t>(base);
        float* ub = reinterpret_cast<float*>((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                                             ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ub, (short)0, __builtin_amdgcn_readfirstlane(nrows * row_bytes), 0x00020000);
        const int off = u < kp ? 8 * u : 1 << 30;
#pragma unroll
        for (int r = 0; r < 8; r++) x[r0 + r] = load_row_pair(rs, off + r * row_bytes);
    };
    // Branch-free (a resource of 0 rows reads zeros): the loads of every path then sit in one block
    // and the waits after them count them exactly (a join made the compiler wait for vmcnt(0)).
    auto issue_rows = [&](const uint32_t cf, const bool live) {
        float* cur = A.xlow + (size_t)(live ? cf : 0) * 2048;
#pragma unroll
        for (int r = 8; r < 40; r += 8) load_rows(cur + (r - 8) * 64, r, live ? 8 : 0, 32, 256);
        // (a batch's first frame is necessarily its run's first record: zeros until the state rows)
        const bool prev = live && cf >= (uint32_t)A.nch;
        const uint32_t pcf = prev ? cf - A.nch : 0;
        if (P == 3) load_rows(A.xcarry + (size_t)pcf * kSbrCarryFloats, 0, prev ? 8 : 0, 64, 512);
        else load_rows(A.xlow + (size_t)pcf * 2048 + 24 * 64, 0, prev ? 8 : 0, 32, 256);
    };
    // The record's table index and the record itself: loaded beside the noise table (their round
    // trip overlaps the barrier's), so that the band-table copy can start right after it.
    constexpr int NR = sizeof(SbrRec) / 4;
    auto fetch_rec = [&](const uint32_t cf, int& table, uint32_t& rv) {
        table = A.recs[cf].table;
        rv = reinterpret_cast<const uint32_t*>(A.recs + cf)[u < NR ? u : NR - 1];
    };
    int table0 = 0;
    uint32_t rv0 = 0;
    // (fused) the analysis constants of lane (half, e) and the previous record's flags and table
    // (its kx masks rows 0..7, as sbr_analysis_kernel masked that frame's X_low)
    [[maybe_unused]] const int ea = u & 31, hba = u & 32, Ea = bitrev5(ea);
    [[maybe_unused]] DctConst Ka;
    [[maybe_unused]] QmfCoefs Qa;
    [[maybe_unused]] uint32_t pflags = 0, ptable = 0;
    {
        const float2 n0 = reinterpret_cast<const float2*>(A.noise)[threadIdx.x];
        const float2 n1 = reinterpret_cast<const float2*>(A.noise)[threadIdx.x + 256];
        if (kPhase != 4) fetch_rec(live ? cf : 0, table0, rv0);
        if constexpr (kFused) {
            Ka = load_dct_const(A.dct, ea, Ea);
            Qa = load_qmf_coefs(A.qmf_c, ea);
            const uint32_t pcf = live && cf >= (uint32_t)A.nch ? cf - A.nch : 0;
            pflags = A.recs[pcf].flags;
            ptable = A.recs[pcf].table;
        }
        noise_s[threadIdx.x] = n0;
        noise_s[threadIdx.x + 256] = n1;
    }
    // an LDS-only barrier (__syncthreads' release fence would wait for the record loads too)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (!live) return;
    HF_STAMP(1);
    auto frame = [&](const uint32_t cf) {
    const int c = (int)(cf % (uint32_t)A.nch);
    // The record and its band tables are read field by field all through the kernel: byte loads
    // at wave-uniform addresses, many inside the envelope and limiter-band loops, each a global
    // round trip the wave waits on.  One coalesced copy into the wave's LDS first; every field
    // read after it is an LDS round trip.
    {
        int table = table0;
        uint32_t rv = rv0;
        if constexpr (kPhase == 4) fetch_rec(cf, table, rv);
        // every lane loads (clamped indices, no lane-masked branch): all loads of the copy are in
        // flight together and wait once (a masked loop waited per iteration)
        constexpr int NT = sizeof(SbrTab) / 4, KT = (NT + 63) / 64;
        uint32_t* rd = reinterpret_cast<uint32_t*>(&L.rec);
        const uint32_t* ts = reinterpret_cast<const uint32_t*>(A.tabs + table);
        uint32_t* td = reinterpret_cast<uint32_t*>(&L.tab);
        uint32_t tv[KT];
#pragma unroll
        for (int j = 0; j < KT; j++) tv[j] = ts[u + 64 * j < NT ? u + 64 * j : NT - 1];
        if constexpr (kFused) {
            // the analysis window into the wave's gain scratch (free until the gain stage):
            // win[0..543] = samples 480..1023 of the previous record's frame (a run's first record:
            // win[256..543] = the slot state's 288-sample tail), win[544..1567] = this frame
            const bool firstr = (__builtin_amdgcn_readlane(rv, 2) >> 24) != 0;  // SbrRec::first (byte 11)
            const uint32_t slot = __builtin_amdgcn_readlane(rv, 16);             // SbrRec::slot
            const float4* cur4 = reinterpret_cast<const float4*>(A.time + batch_cf(A, cf) * 1024);
            const float4* prv4 = firstr ? reinterpret_cast<const float4*>(A.state[(size_t)slot * 2 + c].tail) - 64
                                        : reinterpret_cast<const float4*>(A.time + batch_cf(A, cf - A.nch) * 1024 + 480);
            float4* w4 = reinterpret_cast<float4*>(&L.ecurr[0][0]);
            float4 wv[7];
#pragma unroll
            for (int j = 0; j < 7; j++) {  // 392 float4 = 136 (previous) + 256 (this frame)
                const int i = u + 64 * j;
                const bool pv = i < 136, skip = i >= 392 || (firstr && i < 64);
                wv[j] = skip ? make_float4(0.f, 0.f, 0.f, 0.f) : pv ? prv4[i] : cur4[i - 136];
            }
#pragma unroll
            for (int j = 0; j < 7; j++)
                if (u + 64 * j < 392) w4[u + 64 * j] = wv[j];
        }
        if (u < NR) rd[u] = rv;
#pragma unroll
        for (int j = 0; j < KT; j++)
            if (u + 64 * j < NT) td[u + 64 * j] = tv[j];
        wave_sync();
        HF_STAMP(10);
    }
    const SbrRec& R = L.rec;
    const SbrTab& T = L.tab;
    // The fields that steer loops, branches and selects, read into SGPRs: a field read from the
    // LDS copy is a VGPR the compiler cannot prove wave-uniform, so every envelope-border test,
    // border walk and table-width loop over it was a VALU compare + select or an exec-masked
    // divergent loop (C4 HF 715 -> ~600 us, profiles/round5_hf_uniform/).
    auto ufl = [](int v) { return (int)__builtin_amdgcn_readfirstlane(v); };
    const int kx = ufl(T.kx), M = ufl(T.M), L_E = ufl(R.L_E);
    const uint32_t noise0 = (uint32_t)ufl(R.noise0), sine0 = (uint32_t)ufl(R.sine0);
    int tE[6];
#pragma unroll
    for (int k = 0; k < 6; k++) tE[k] = ufl(R.t_E[k]);
    const int first = tE[0], last = ufl(R.t_E[L_E]);
    const int s_lim = R.lim_bands;
    const float rel = __fdiv_rn(1.0f, 1.0f + 1e-6f);

    // rows 0..7 of a run's first record: the slot state's carry rows (issue_rows above)
    if constexpr (kFused) {
        // QMF analysis (A/sbr/AnalysisFilterbank.java:9-73, qmf_analysis_pass): pass p gives slots
        // 2p (lanes 0..31) and 2p + 1 (lanes 32..63); one v_permlane32_swap brings both to lane =
        // band.  Rows 8..39 = this frame's slots 0..31 (kx of this record); rows 0..7 = the previous
        // frame's slots 24..31 (its kx), i.e. this frame's "slots -8..-1"; a run's first record
        // takes them from the slot state below.
        const float* win = &L.ecurr[0][0] + 544;
        auto smp = [&](int g) { return win[g]; };
        const int kxc = (R.flags & kSbrProcess) ? kx : 32;
        const int kxp = (pflags & kSbrProcess) ? (int)A.tabs[ptable].kx : 32;
        const bool firstr = ufl(R.first) != 0;
#pragma unroll
        for (int p = -4; p < 16; p++) {
            if (p < 0 && firstr) continue;
            const float2 v = qmf_analysis_pass(smp, 2 * p + (hba >> 5), ea, hba, Ea, Ka, Qa, p < 0 ? kxp : kxc);
            const auto sr = __builtin_amdgcn_permlane32_swap(__float_as_int(v.x), __float_as_int(v.x), false, false);
            const auto si = __builtin_amdgcn_permlane32_swap(__float_as_int(v.y), __float_as_int(v.y), false, false);
            // lanes 0..31: own value = slot 2p, the swapped one = slot 2p + 1; bands >= 32 are zero
            const int r0 = 8 + 2 * p;
            x[r0] = u < 32 ? f2{v.x, v.y} : f2{0.0f, 0.0f};
            x[r0 + 1] = u < 32 ? f2{__int_as_float(sr[1]), __int_as_float(si[1])} : f2{0.0f, 0.0f};
        }
        wave_sync();  // (the window's LDS is the gain stage's scratch)
    } else {
        issue_rows(cf, true);
    }
    HF_STAMP(11);
    if (ufl(R.first)) load_rows(&A.state[(size_t)ufl(R.slot) * 2 + c].xcarry[0][0][0], 0, 8, 64, 512);
    // Parameter lookups issued now, while the Xlow rows are in flight: the generation's source band
    // and chirp factor, and calculate_gain's per-band inputs of every envelope (noise band ->
    // Q_div / Q_div2, resolution band -> E_orig).  Each is a two-level table walk in global memory;
    // fetched inside the envelope loop they were two dependent round trips per envelope.
    const int p_src = T.src_p[u];
    float bw_k, pEo[5];
    int nb_m;  // noise band of band m
    {
        const int gk = T.g_of_k[u];
        bw_k = R.bw[gk < 5 ? gk : 0];
        const int mi = (u - kx >= 0 && u - kx < M) ? u - kx : 0;
        const int nb = T.noise_map[s_lim][mi];
        nb_m = nb;
        const int rm0 = T.res_map[s_lim][0][mi], rm1 = T.res_map[s_lim][1][mi];
        int eo = (int)R.e_off;
#pragma unroll
        for (int l = 0; l < 5; l++) {
            const bool on = l < L_E;
            const int fl = on ? R.f[l] : 0;
            pEo[l] = on ? A.epool[eo + (fl ? rm1 : rm0)] : 0.0f;
            eo += on ? (fl ? T.n_hi : T.n_lo) : 0;
        }
    }
    // The G/Q smoothing ring in age order: gr[0] is the entry the frame's first assembled row
    // overwrites (ring position GQ_ringbuf_index = gq0), gr[4] the newest; each row shifts it by one
    // and appends, so its five filter taps are gr[0..4] in order -- compile-time registers instead
    // of a select over the ring per tap (positions read rotated once here, gq0 wave-uniform).
    f2 gq[5] = {};  // (G, Q) pairs: the smoothing filter runs packed
    const int gq0 = ufl(R.gq0);
    if ((P == 2 || (P == 3 && A.smoothing)) && !(R.flags & kSbrReset)) {
        const float* ring = R.first ? &A.state[(size_t)R.slot * 2 + c].gq[0][0][0] : A.gq + (size_t)(cf - A.nch) * 640;
        const int mm = u - kx >= 0 && u - kx < 64 ? u - kx : 0;
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const int pj = (gq0 + j) % 5;
            gq[j] = f2{ring[pj * 64 + mm], ring[320 + pj * 64 + mm]};
        }
        if (A.dbg && cf == 2)
            for (int j = 0; j < 5; j++) {
                A.dbg[((gq0 + j) % 5) * 64 + u] = gq[j].x;
                A.dbg[320 + ((gq0 + j) % 5) * 64 + u] = gq[j].y;
            }
    }

    HF_STAMP(2);
    // ---------- HF generation (A/sbr/HFGeneration.java:17-98, 100-196) ----------
    float a0r = 0, a0i = 0, a1r = 0, a1i = 0;
    {
        // r01 = (r01r, r01i) += (t3r t2r + t3i t2i, t3i t2r - t3r t2i), r02 likewise with t1:
        // 2 v_pk_mul + 2 v_pk_add each; r11r += t2r t2r + t2i t2i
        f2 r01 = {0.0f, 0.0f}, r02 = {0.0f, 0.0f};
        float r11r = 0;
        f2 t1, t2 = x[0], t3 = x[1];
        const f2 t4 = t2, t5 = t3;
#pragma unroll
        for (int j = 2; j < 40; j++) {
            t1 = t2;
            t2 = t3;
            t3 = x[j];
            r01 = pk_add(r01, pk_mul_conj(t3, t2));
            r02 = pk_add(r02, pk_mul_conj(t3, t1));
            const f2 sq = pk_mul(t2, t2);
            r11r += sq.x + sq.y;
        }
        const float r01r = r01.x, r01i = r01.y, r02r = r02.x, r02i = r02.y;
        const f2 c32 = pk_mul_conj(t3, t2), c54 = pk_mul_conj(t5, t4);
        const f2 s2 = pk_mul(t2, t2), s4 = pk_mul(t4, t4);
        const float r12r = r01r - c32.x + c54.x;
        const float r12i = r01i - c32.y + c54.y;
        const float r22r = r11r - (s2.x + s2.y) + (s4.x + s4.y);
        const float det = (r11r * r22r) - (rel * ((r12r * r12r) + (r12i * r12i)));
        if (det != 0.0f) {
            const float tmp = __fdiv_rn(1.0f, det);
            a1r = ((r01r * r12r) - (r01i * r12i) - (r02r * r11r)) * tmp;
            a1i = ((r01i * r12r) + (r01r * r12i) - (r02i * r11r)) * tmp;
        }
        if (r11r != 0.0f) {
            const float tmp = __fdiv_rn(1.0f, r11r);
            a0r = -(r01r + (a1r * r12r) + (a1i * r12i)) * tmp;
            a0i = -(r01i + (a1i * r12r) - (a1r * r12i)) * tmp;
        }
        if (((a0r * a0r) + (a0i * a0i) >= 16.0f) || ((a1r * a1r) + (a1i * a1i) >= 16.0f)) a0r = a0i = a1r = a1i = 0.0f;
    }
    HF_STAMP(3);
    {
        const int p = p_src;
        const bool gen = p != 0xFF;
        const int ps = gen ? p : u;
        const float bw = bw_k;
        const f2 bwp = f2{bw, bw * bw};  // (bw, bw2)
        const f2 A0 = pk_mul_bx(bwp, f2{shfl(a0r, ps), shfl(a0i, ps)});  // (A0r, A0i)
        const f2 A1 = pk_mul_by(bwp, f2{shfl(a1r, ps), shfl(a1i, ps)});  // (A1r, A1i)
        f2 p1 = {0.0f, 0.0f}, p2 = {0.0f, 0.0f};  // source rows r-2, r-1
        f2 sb[8];  // source rows, fetched 8 at a time
#pragma unroll
        for (int r = 0; r < 40; r++) {
            if ((r & 7) == 0) {
#pragma unroll
                for (int q = 0; q < 8; q++) sb[q] = f2{shfl(x[r + q].x, ps), shfl(x[r + q].y, ps)};
            }
            const f2 sv = sb[r & 7];
            const int l = r - 2;
            if (gen && l >= first && l < last) {
                if (bwp.y > 0.0f) {
                    // (A0r p2r - A0i p2i + A1r p1r - A1i p1i, A0i p2r + A0r p2i + A1i p1r + A1r p1i),
                    // left to right as the Java sums them, then added to the source row
                    f2 w = pk_add_nlo(pk_mul_xa(A0, p2), pk_mul_ya(A0, p2));
                    w = pk_add(w, pk_mul_xa(A1, p1));
                    w = pk_add_nlo(w, pk_mul_ya(A1, p1));
                    x[r] = pk_add(sv, w);
                } else {
                    x[r] = sv;
                }
            }
            p1 = p2;
            p2 = sv;
            if ((r & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        }
    }

    HF_STAMP(4);
    // ---------- HF adjustment (A/sbr/HFAdjustment.java) ----------
    const int m = u - kx;
    const bool band = m >= 0 && m < M;
    // estimate_current_envelope (:82-138)
    if (R.flags & kSbrInterpol) {
        float acc[5] = {0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 2; r < 40; r++) {
            const f2 sq = pk_mul(x[r], x[r]);
            const float en = sq.x + sq.y;
            const int i = r - 2;
#pragma unroll
            for (int l = 0; l < 5; l++)
                if (l < L_E && i >= tE[l] && i < tE[l + 1]) acc[l] += en;
        }
#pragma unroll
        for (int l = 0; l < 5; l++) {
            if (l < L_E && band) {
                float div = (float)(tE[l + 1] - tE[l]);
                if (div == 0.0f) div = 1.0f;
                L.ecurr[l][m] = __fdiv_rn(acc[l], div);
            }
        }
    } else {
        // band-group averages: nrg over rows (outer) and bands of the group (inner)
        for (int l = 0; l < L_E; l++) {
            const int fl = ufl(R.f[l]);
            const int nb = ufl(fl ? T.n_hi : T.n_lo);
            int k_l = -1, k_h = -1;
            for (int p = 0; p < nb; p++)
                if (u >= T.f_res[fl][p] && u < T.f_res[fl][p + 1]) {
                    k_l = T.f_res[fl][p];
                    k_h = T.f_res[fl][p + 1];
                }
            int maxw = 0;
            for (int p = 0; p < nb; p++) maxw = max(maxw, ufl((int)T.f_res[fl][p + 1] - (int)T.f_res[fl][p]));
            const int w = k_h - k_l;
            float nrg = 0.0f;
#pragma unroll
            for (int r = 2; r < 40; r++) {
                const f2 sq = pk_mul(x[r], x[r]);
                const float en = sq.x + sq.y;
                const int i = r - 2;
                if (i >= ufl(R.t_E[l]) && i < ufl(R.t_E[l + 1])) {
                    for (int d = 0; d < maxw; d++) {
                        const float v = shfl(en, (u + d) & 63);
                        if (u == k_l && d < w) nrg += v;
                    }
                }
            }
            int rows = R.t_E[l + 1] - R.t_E[l];
            float div = (float)(rows * w);
            if (div == 0.0f) div = 1.0f;
            const float own = __fdiv_rn(nrg, div);
            const float val = shfl(own, k_l >= 0 ? k_l : u);
            if (band && k_l >= 0) L.ecurr[l][m] = val;
        }
    }
    for (int i = u; i < 5 * 64; i += 64) {
        (&L.gl[0][0])[i] = 0.0f;
        (&L.ql[0][0])[i] = 0.0f;
        (&L.sl[0][0])[i] = 0.0f;
    }
    wave_sync();

    HF_STAMP(5);
    // calculate_gain (:240-415), per envelope, with every per-band step lane-parallel:
    //   (1) lane m: E_orig, E_curr, Q_M, S_M and the unlimited G;
    //   (2) lane kb (limiter band): acc1, acc2 as the Java's ordered sums over its bands -> G_max;
    //   (3) lane m: limiting (G_max vs G, Q_M*G_max/G) and its three den terms;
    //   (4) lane kb: den as the ordered sum of those terms -> G_boost;
    //   (5) lane m: the boosted square roots.
    // A skipped den term is written as +0: every term is >= 0 and den starts at +0, so adding
    // +0 leaves the sum bit-identical.  Ordered sums read up to 16 band values in one batch.
    {
        const int NL = T.N_L[s_lim];
        const float EPS = 1e-12f;
        // limiter band of band m (lane); bands outside every limiter band keep G = Q = S = 0
        int kbm = 0;
        for (int kb = 1; kb < NL; kb++)
            if (m >= (int)T.lim[s_lim][kb]) kbm = kb;
        const bool covered = band && m >= (int)T.lim[s_lim][0] && m < (int)T.lim[s_lim][NL];
        const int kb = u;
        const bool lim_lane = kb < NL;
        const int ml1 = lim_lane ? T.lim[s_lim][kb] : 0, ml2 = lim_lane ? T.lim[s_lim][kb + 1] : 0;
        int wmax = 0;
        for (int j = 0; j < NL; j++) wmax = max(wmax, (int)T.lim[s_lim][j + 1] - (int)T.lim[s_lim][j]);
#pragma unroll
        for (int l = 0; l < 5; l++) {
            if (l >= L_E) break;
            const bool delta1 = !((R.no_noise >> l) & 1);
            const uint64_t smask = R.s_index[l], mmask = R.s_mapped[l];
            const bool sidx = band && ((smask >> m) & 1);
            float Eom = 0.0f, Ec = 0.0f, Q_M = 0.0f, S_M = 0.0f, G = 0.0f;
            if (band) {  // (1)
                const int tnb = ufl(R.tnb[l]);
                const float Qd = R.q_div[tnb][nb_m], Qd2 = R.q_div2[tnb][nb_m];
                Eom = pEo[l];
                Ec = L.ecurr[l][m];
                const bool smap = (mmask >> m) & 1;
                G = __fdiv_rn(Eom, 1.0f + Ec);
                if (!smap && delta1) G *= Qd;
                else if (smap) G *= Qd2;
                L.gq_eo[m] = Eom;
                Q_M = Eom * Qd2;
                S_M = sidx ? Eom * Qd : 0.0f;
            }
            wave_sync();
            if (lim_lane) {  // (2)
                float acc1 = 0.0f, acc2 = 0.0f;
                if (wmax <= 16) {
#pragma unroll
                    for (int h = 0; h < 16; h += 8) {  // (8 reads in flight: fewer live VGPRs than 16)
                        float ve[8], vc[8];
#pragma unroll
                        for (int j = 0; j < 8; j++) {
                            const int mm = ml1 + h + j < ml2 ? ml1 + h + j : ml1;
                            ve[j] = L.gq_eo[mm];
                            vc[j] = L.ecurr[l][mm];
                        }
#pragma unroll
                        for (int j = 0; j < 8; j++)
                            if (ml1 + h + j < ml2) {
                                acc1 += ve[j];
                                acc2 += vc[j];
                            }
                    }
                } else {
                    for (int mm = ml1; mm < ml2; mm++) {
                        acc1 += L.gq_eo[mm];
                        acc2 += L.ecurr[l][mm];
                    }
                }
                float G_max = __fdiv_rn(EPS + acc1, EPS + acc2) * R.lim_gain;
                L.lim_gmax[kb] = java_minf(G_max, 1e10f);
                L.lim_acc1[kb] = acc1;
            }
            wave_sync();
            float Gl = 0.0f, Ql = 0.0f;
            if (covered) {  // (3)
                const float G_max = L.lim_gmax[kbm];
                if (G_max > G) {
                    Ql = Q_M;
                    Gl = G;
                } else {
                    Ql = __fdiv_rn(Q_M * G_max, G);
                    Gl = G_max;
                }
                L.den_s[m] = sidx ? S_M : 0.0f;
                L.den_e[m] = Ec * Gl;
                L.den_q[m] = (!sidx && l != R.l_A) ? Ql : 0.0f;
            }
            wave_sync();
            if (lim_lane) {  // (4)
                float den = 0.0f;
                if (wmax <= 16) {
#pragma unroll
                    for (int h = 0; h < 16; h += 8) {
                        float ts[8], te[8], tq[8];
#pragma unroll
                        for (int j = 0; j < 8; j++) {
                            const int mm = ml1 + h + j < ml2 ? ml1 + h + j : ml1;
                            ts[j] = L.den_s[mm];
                            te[j] = L.den_e[mm];
                            tq[j] = L.den_q[mm];
                        }
#pragma unroll
                        for (int j = 0; j < 8; j++)
                            if (ml1 + h + j < ml2) den = ((den + ts[j]) + te[j]) + tq[j];
                    }
                } else {
                    for (int mm = ml1; mm < ml2; mm++) den = ((den + L.den_s[mm]) + L.den_e[mm]) + L.den_q[mm];
                }
                const float G_boost = __fdiv_rn(L.lim_acc1[kb] + EPS, den + EPS);
                L.lim_boost[kb] = java_minf(G_boost, 2.51188643f);
            }
            wave_sync();
            if (covered) {  // (5)
                const float Gb = L.lim_boost[kbm];
                L.gl[l][m] = sqrtf(Gl * Gb);
                L.ql[l][m] = sqrtf(Ql * Gb);
                L.sl[l][m] = S_M != 0.0f ? sqrtf(S_M * Gb) : 0.0f;
            }
            wave_sync();
        }
    }

    HF_STAMP(6);
    // G/Q ring after this frame: the last 5 assembled rows (rows >= 26 always, see the host check).
    // Read by the next frame's smoothing (launches with smoothing) and, for a run's last record, by
    // sbr_state_kernel: other records of a launch without smoothing skip the 2.5 KB.
    if (A.smoothing || (ufl(R.flags) & kSbrLast)) {
        float* ring = A.gq + (size_t)cf * 640;
        const int rows = last - first;
        for (int j = 0; j < 5; j++) {
            const int i = last - 1 - j;                      // row
            const int pos = (R.gq0 + rows - 1 - j + 10) % 5;  // ring position it was written to
            int l = 0;
            for (int jj = 1; jj < L_E; jj++)
                if (i >= R.t_E[jj]) l = jj;
            ring[pos * 64 + u] = u < M ? L.gl[l][u] : 0.0f;
            ring[320 + pos * 64 + u] = u < M ? L.ql[l][u] : 0.0f;
        }
    }
    if (P == 1) return;

    HF_STAMP(7);
    // hf_assembly (:140-238): lane k = m + kx
    {
        const int mi = band ? m : 0;
        const bool smooth = (R.flags & kSbrSmooth) != 0;
        if (R.flags & kSbrReset) {  // ring positions 0..3 = the first envelope's values, position 4 (0) is written first
            const float g0 = L.gl[0][mi], q0 = L.ql[0][mi];
#pragma unroll
            for (int j = 1; j < 5; j++) {
                gq[j] = f2{g0, q0};
            }
        }
        const float rev = (u & 1) ? -1.0f : 1.0f;
        if (!smooth) {
            // bs_smoothing_mode == 1: G_filt/Q_filt are the row's envelope values, no ring
            // (the G/Q ring output above is built from gl/ql directly); the rows walk the
            // envelopes in order, so each envelope's values are read from LDS once
            int l = -1, next = first;  // next: first row of the envelope after l
            f2 gqf = {0.0f, 0.0f}, Sv = {0.0f, 0.0f};  // (G_filt, Q_filt), (S, rev * S)
            float2 nzv[8];  // noise entries of the next 8 rows
#pragma unroll
            for (int r = 2; r < 40; r++) {
                const int i = r - 2;
                if (((r - 2) & 7) == 0) {
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        nzv[q] = noise_s[(noise0 + (uint32_t)(i + q - first) * (uint32_t)M + (uint32_t)mi + 1u) & 511u];
                }
                if (i < first || i >= last) continue;
                if (i >= next) {  // wave-uniform
                    while (l + 1 < L_E && i >= ufl(R.t_E[l + 1])) l++;
                    next = l + 1 < L_E ? ufl(R.t_E[l + 1]) : 64;
                    const bool no_noise = (ufl(R.no_noise) >> l) & 1;
                    const float S = L.sl[l][mi];
                    gqf = f2{L.gl[l][mi], (S != 0.0f || no_noise) ? 0.0f : L.ql[l][mi]};
                    Sv = f2{S, rev * S};
                }
                const int fs = (int)((sine0 + (uint32_t)(i - first)) & 3u);
                if (band) {
                    const float2 nz = nzv[(r - 2) & 7];
                    // (G xr + Q nz.re + S phr, G xi + Q nz.im + (rev S) phi)
                    const f2 ph = f2{fs == 0 ? 1.0f : fs == 2 ? -1.0f : 0.0f, fs == 1 ? 1.0f : fs == 3 ? -1.0f : 0.0f};
                    const f2 v = pk_add(pk_mul_bx(gqf, x[r]), pk_mul_by(gqf, f2{nz.x, nz.y}));
                    x[r] = pk_add(v, pk_mul(Sv, ph));
                }
            }
        } else {
        int l = -1, next = first;  // envelope walk as above
        bool no_noise = false;
        float gnew = 0.0f, qnew = 0.0f, S = 0.0f;
        f2 Sv = {0.0f, 0.0f};  // (S, rev * S)
        float2 nzv[8];  // noise entries of the next 8 rows, read before them (no LDS wait per row)
#pragma unroll
        for (int r = 2; r < 40; r++) {
            const int i = r - 2;
            if (((r - 2) & 7) == 0) {
#pragma unroll
                for (int q = 0; q < 8; q++)
                    nzv[q] = noise_s[(noise0 + (uint32_t)(i + q - first) * (uint32_t)M + (uint32_t)mi + 1u) & 511u];
            }
            if (i < first || i >= last) continue;
            if (i >= next) {  // wave-uniform
                while (l + 1 < L_E && i >= ufl(R.t_E[l + 1])) l++;
                next = l + 1 < L_E ? ufl(R.t_E[l + 1]) : 64;
                no_noise = (ufl(R.no_noise) >> l) & 1;
                gnew = L.gl[l][mi];
                qnew = L.ql[l][mi];
                S = L.sl[l][mi];
                Sv = f2{S, rev * S};
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                gq[j] = gq[j + 1];
            }
            gq[4] = f2{gnew, qnew};
            float G_filt = 0.0f, Q_filt = 0.0f;
            if (smooth && !no_noise) {
                // taps from the oldest entry (ring position GQ_ringbuf_index + 1) to this row's
                // (A/sbr/HFAdjustment.java:188-195), G and Q in one packed accumulator
                f2 acc = f2{0.0f, 0.0f};
#pragma unroll
                for (int n = 0; n <= 4; n++) {
                    const float h = n == 0 ? 0.03183050093751f : n == 1 ? 0.11516383427084f
                                  : n == 2 ? 0.21816949906249f : n == 3 ? 0.30150283239582f : 0.33333333333333f;
                    acc += gq[n] * h;
                }
                G_filt = acc.x;
                Q_filt = acc.y;
            } else {
                G_filt = gnew;
                Q_filt = qnew;
            }
            Q_filt = (S != 0.0f || no_noise) ? 0.0f : Q_filt;
            const int fs = (int)((sine0 + (uint32_t)(i - first)) & 3u);
            if (band) {
                const float2 nz = nzv[(r - 2) & 7];
                const f2 gqf = f2{G_filt, Q_filt};
                const f2 ph = f2{fs == 0 ? 1.0f : fs == 2 ? -1.0f : 0.0f, fs == 1 ? 1.0f : fs == 3 ? -1.0f : 0.0f};
                const f2 v = pk_add(pk_mul_bx(gqf, x[r]), pk_mul_by(gqf, f2{nz.x, nz.y}));
                x[r] = pk_add(v, pk_mul(Sv, ph));
            }
            if (((r - 2) & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        }
        }
    }


    HF_STAMP(8);
    // ---------- outputs ----------
    // synthesis input X[l][k] = Xsbr[l + tHFAdj][k] for k < kx_band + M_band (Channel.java:619-645);
    // rows l < t_E[0] take kx_prev/M_prev and the carried rows, patched in by the synthesis kernel
    {
        // rows l < t_E[0] are Xsbr rows 2..7 as frame f-1 left them: its carry rows 2..7, which
        // the synthesis / PS analysis read (a later launch) with kx_prev + M_prev bands
        // (from the run's band limit up nothing is stored: no stage reads those bands, SbrRec::blim)
        // (PS: straight into X_left's place, xps[f][0], which the PS analysis patches rows
        // l < t_E[0] of; nch = 1 there)
        float2* xs = reinterpret_cast<float2*>(A.ps ? A.xps + (size_t)cf * 8192 : A.xsyn + (size_t)cf * 4096);
        const int kcur = kx + M, blim = ufl(R.blim);
        // bands below kx + M keep their rows, the rest up to the band limit are zero (two store
        // loops under complementary lane masks, no per-row select)
        if (u < min(blim, kcur)) {
#pragma unroll
            for (int l = 0; l < 32; l++) xs[l * 64 + u] = make_float2(x[l + 2].x, x[l + 2].y);
        } else if (u < blim) {
#pragma unroll
            for (int l = 0; l < 32; l++) xs[l * 64 + u] = make_float2(0.0f, 0.0f);
        }
        // Xsbr rows 32..39, every band (zero from kx + M up): the next frame's rows 0..7, the PS
        // look-ahead rows, the slot state
        float2* xc = reinterpret_cast<float2*>(A.xcarry + (size_t)cf * kSbrCarryFloats);
#pragma unroll
        for (int j = 0; j < 8; j++) xc[j * 64 + u] = make_float2(x[32 + j].x, x[32 + j].y);
    }
#if defined(JAAD_HF_STAMPS)
    HF_STAMP(9);
    if (kPhase == 0 && A.dbg && u < 12) reinterpret_cast<uint64_t*>(A.dbg)[(size_t)cf * 16 + u] = hf_t[u];
#endif
    };
    if constexpr (kPhase == 4) {
        for (uint32_t it = 0; it < n_iter; it++) {
            if (it) {
                __threadfence();  // the previous frame's carry rows and G/Q ring, before this frame reads them
                wave_sync();
            }
            frame(A.fix[o + it]);
        }
    } else {
        frame(cf);
    }
}

// ---------------------------------------------------------------------------------------------
// synthesis: where the rows of one frame of a chunk's sequence come from (all wave-uniform)
// ---------------------------------------------------------------------------------------------
struct SynSrc {
    const gfloat* xs;  // rows l >= t0 (64 bands, 128 floats a row)
    const gfloat* xc;  // rows l < t0: the carried Xsbr rows 2..7, kprev bands
    int t0, kprev, rows;
    int lo;            // rows below lo are clamped to it (the 64-band history's leading dummy slot)
    size_t n0;         // first output sample (emitting frames)
    bool emit, dup;
};
// the record fields the synthesis needs (dwords 0..3 and the slot), loaded one frame ahead
struct SynRec {
    uint32_t w0, w1, w2, w3, slot;
};

// SynthesisFilterbank32's DCT4_32 / DST4_32 (A/sbr/SynthesisFilterbank32.java:95-940): the
// reference's straight-line binary32 programs (tables/jaad_sbr_dct32.inc), unrolled at compile
// time over a register file r[] (in place on r[0..31], temporaries above), same ops, same order.
template <int kKind, int kD, int kA, int kB>
__device__ __forceinline__ void dct32_op(float* r, float k)
{
    if constexpr (kKind == 0) r[kD] = r[kA] - r[kB];
    else if constexpr (kKind == 1) r[kD] = r[kA] + r[kB];
    else r[kD] = k * r[kA];
}
template <size_t... I>
__device__ __forceinline__ void dct4_32(float* r, std::index_sequence<I...>)
{
    (dct32_op<JAAD_SBR_DCT4_32_OPS[I][0], JAAD_SBR_DCT4_32_OPS[I][1], JAAD_SBR_DCT4_32_OPS[I][2],
              JAAD_SBR_DCT4_32_OPS[I][3]>(r, JAAD_SBR_DCT4_32_K[I]),
     ...);
}
template <size_t... I>
__device__ __forceinline__ void dst4_32(float* r, std::index_sequence<I...>)
{
    (dct32_op<JAAD_SBR_DST4_32_OPS[I][0], JAAD_SBR_DST4_32_OPS[I][1], JAAD_SBR_DST4_32_OPS[I][2],
              JAAD_SBR_DST4_32_OPS[I][3]>(r, JAAD_SBR_DST4_32_K[I]),
     ...);
}

// Downsampled synthesis (SynthesisFilterbank32.synthesis, A/sbr/SynthesisFilterbank32.java:44-93),
// a frame at a time: lane (half, l) pre-twiddles row l of the frame and runs DCT4_32 (half 0, x1)
// or DST4_32 (half 1, x2) on it -- the 32 slots of a frame in parallel --, the v blocks go to an
// LDS ring of 41 (9 history + 32), then the 10-tap window makes 2 slots' 32 samples per pass.
constexpr int kRing32 = 41;
template <class HistSrc, class FrameSrc, class RecLoad, class StorePcm>
__device__ __forceinline__ void synthesis32(const SbrArgs& A, const SbrChunk& ck, int wave, HistSrc history_src,
                                            FrameSrc frame_src, RecLoad rec_load, const float (&cw)[10],
                                            StorePcm store_pcm)
{
    __shared__ float ring_s[kWavesPerBlock][kRing32][64];
    __shared__ float tr_s[kWavesPerBlock][2][32][33];  // DCT / DST outputs [half][slot][n] (+1 pad)
    float(*ring)[64] = ring_s[wave];
    float(*tr)[32][33] = tr_s[wave];
    const int u = lane_id();
    const int l = u & 31, half = u >> 5;
    const float scale = 1.f / 64.f;
    // v blocks of the frame's rows -> ring[(base + l) % kRing32]
    auto transform = [&](const SynSrc& S, int base) {
        if (l < S.rows) {
            const bool carry = l < S.t0;
            const gfloat* row = carry ? S.xc + (l + 2) * 128 : S.xs + l * 128;
            const int klim = carry ? S.kprev : 64;
            float r[JAAD_SBR_DCT4_32_NREG > JAAD_SBR_DST4_32_NREG ? JAAD_SBR_DCT4_32_NREG : JAAD_SBR_DST4_32_NREG];
#pragma unroll
            for (int k = 0; k < 32; k++) {
                const float re = k < klim ? row[2 * k] : 0.0f, im = k < klim ? row[2 * k + 1] : 0.0f;
                const float t0 = A.tw32[2 * k], t1 = A.tw32[2 * k + 1];  // qmf32_pre_twiddle[k]
                float x1 = (re * t0) - (im * t1);
                float x2 = (im * t0) + (re * t1);
                x1 *= scale;
                x2 *= scale;
                r[k] = half ? x2 : x1;
            }
            if (half) dst4_32(r, std::make_index_sequence<JAAD_SBR_DST4_32_NOPS>{});
            else dct4_32(r, std::make_index_sequence<JAAD_SBR_DCT4_32_NOPS>{});
#pragma unroll
            for (int n = 0; n < 32; n++) tr[half][l][n] = r[n];
        }
        wave_sync();
        if (l < S.rows) {
            float* vb = ring[(base + l) % kRing32];
#pragma unroll
            for (int n = 0; n < 32; n++) {
                const float c1 = tr[0][l][n], s2 = tr[1][l][n];
                if (!half) vb[n] = -c1 + s2;       // v[n] = -x1[n] + x2[n]
                else vb[63 - n] = c1 + s2;         // v[63 - n] = x1[n] + x2[n]
            }
        }
        wave_sync();
    };
    // the 10-tap window (:73-86) of slot s (block b = its ring block), sample l
    auto window = [&](int b) {
        float acc = 0.0f;
#pragma unroll
        for (int t = 0; t < 10; t++) {
            const float* vt = ring[(b - t + kRing32) % kRing32];
            const float p = vt[(t & 1) * 32 + l] * cw[t];
            acc = t == 0 ? p : acc + p;
        }
        return acc;
    };
    SynSrc S = history_src();
    SynRec W{};
    rec_load(0, W);
    transform(S, 0);
    int base = S.rows;  // ring block of the next frame's slot 0
    for (uint32_t j = 0; j < ck.n; j++) {
        S = frame_src((int)j, W);
        rec_load((int)j + 1, W);
        if (!S.rows) continue;
        transform(S, base);
        if (S.emit)
            for (int s = half; s < S.rows; s += 2) store_pcm(S, S.n0 + 32 * s + l, window(base + s));
        base = (base + S.rows) % kRing32;
        wave_sync();
    }
}

// ---------------------------------------------------------------------------------------------
// SynthesisFilterbank64.synthesis (A/sbr/SynthesisFilterbank64.java:9-79) + SampleBuffer PCM
// ---------------------------------------------------------------------------------------------
// kDown: SynthesisFilterbank32 (downsampled SBR, A/sbr/SynthesisFilterbank32.java:44-93), bands
// 0..31, 32 samples per slot.  Its DCT-IV / DST-IV run the reference's own generated DCT4_32 /
// DST4_32 op lists (tables/jaad_sbr_dct32.inc, unrolled at compile time above), and the
// pre-twiddle is the reference's qmf32_pre_twiddle, so oracle, kernel and reference perform the
// same binary32 operations in the same order.
template <bool kDown>
__global__ __launch_bounds__(256) void sbr_synthesis_kernel(SbrArgs A)
{
    // v ring: 10 blocks, each also kept 10 blocks up (a window reads ring blocks q+1..q+10 at fixed
    // offsets); half h of ring block q at [h][q][64], so the two slots of a pair read a tap's words
    // 256 bytes apart (one ds_read2st64 a tap, the pair's values in one register pair)
    __shared__ float vring_s[kWavesPerBlock][kDown ? 1 : 40][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ci = blockIdx.x * kWavesPerBlock + wave;
    if (ci >= A.n_chunks) return;
    float(*vring)[64] = vring_s[wave];
    const SbrChunk ck = A.chunks[ci];
    const int u = lane_id();
    const int e = u & 31, half = u >> 5;
    // PS: the SBR stages ran on the mono channel (nch = 1); channel c of the output is X_left' /
    // X_right from ps_kernel (xps), whose rows need no carry patch
    const int c = ck.ch, nch = A.nch, ps = A.ps;
    const int rc = ps ? 0 : c;  // channel of the SBR records
    const DctPairConst K = load_dct_pair_const(A.dct, e);
    // v-block words of this lane's DCT outputs (dct4_pair: elements n = E_S (.x) and E_S + 1 (.y) of
    // slot e >> 4; half 0 holds the x1 outputs and gets the x2 real parts, half 1 the x2 outputs
    // and gets the x1 imaginary parts): with a = x2 + x1, b = x2 - x1 (SynthesisFilterbank64.java:99-129)
    //   half 0: v[2n] = b, v[127-2n] = a       half 1: v[63-2n] = a, v[64+2n] = b
    const int es = bitrev5(e & 15), sl = 128 * ((e >> 4) & 1);
    auto ring_word = [&](int w) { return (w >> 6) * 20 * 64 + (w & 63) + (sl >> 1); };  // v[w] of ring block 0 (+ slot)
    const int wa_x = ring_word(half ? 63 - 2 * es : 127 - 2 * es), wb_x = ring_word(half ? 64 + 2 * es : 2 * es);
    const int wa_y = ring_word(half ? 61 - 2 * es : 125 - 2 * es), wb_y = ring_word(half ? 66 + 2 * es : 2 * es + 2);
    float cw[10];
#pragma unroll
    for (int t = 0; t < 10; t++) cw[t] = kDown ? A.qmf_c[64 * t + 2 * e] : A.qmf_c[u + 64 * t];
    const float scale = 1.f / 64.f;
    // This lane's two DCT inputs of a slot, gathered straight from the row of X (64 float2, band
    // order) instead of exchanged through cross-lane permutes:
    //   64 bands: half 0 (in_real1[e], in_imag1[e]) = (Re X[2e], Re X[63-2e]),
    //             half 1 (in_real2[e], in_imag2[e]) = (Im X[63-2e], Im X[2e])  (SynthesisFilterbank64.java:25-42)
    const int band_a = half ? 63 - 2 * e : 2 * e;
    const int band_b = half ? 2 * e : 63 - 2 * e;
    // Rows hold 64 bands in memory; bands >= klim read as zero.  The mask is applied where the
    // slot consumes the values (a select next to the load would wait for it).  From the run's band
    // limit up (SbrRec::blim; the same for every record of a chunk) nothing is read: those lanes
    // load the word of band 0 (fetched by other lanes anyway) and the mask zeroes it.
    const int kb = (int)__builtin_amdgcn_readfirstlane(A.recs[(size_t)ck.frame0 * nch + rc].blim);
    const int ia = band_a < kb ? 2 * band_a + half : half, ib = band_b < kb ? 2 * band_b + half : half;
    auto fetch = [&](const gfloat* r, float& a, float& b) {
        a = r[ia];
        b = r[ib];
    };
    auto mask = [&](int klim, float& a, float& b) {
        a = band_a < klim ? a : 0.0f;
        b = band_b < klim ? b : 0.0f;
    };

    // two slots at ring blocks p, p + 1 (p even): DCT-IV pairs -> v blocks (:99-129); emit: their
    // windows (:134-146), sample u in res0 / res1
    auto slot_pair = [&](float a0, float b0, float a1, float b1, int p, bool emit, float& res0, float& res1) {
        const f2 in_r = f2{a0, a1} * scale;  // (fetch) d = 0: in_real1[e] / d = 1: in_real2[e]
        const f2 in_i = f2{b0, b1} * scale;  //            in_imag1[e] /        in_imag2[e]
        f2 orr, oi;
        dct4_pair(K, e, in_r, in_i, orr, oi);
        // half 0 gets x2's real parts, half 1 x1's imaginary parts (v_permlane32_swap)
        const auto px = __builtin_amdgcn_permlane32_swap(__float_as_int(orr.x), __float_as_int(oi.x), false, false);
        const auto py = __builtin_amdgcn_permlane32_swap(__float_as_int(orr.y), __float_as_int(oi.y), false, false);
        const f2 x1 = f2{__int_as_float(px[0]), __int_as_float(py[0])};
        const f2 x2 = f2{__int_as_float(px[1]), __int_as_float(py[1])};
        const f2 a = x2 + x1, b = x2 - x1;
        // the pair's windows read blocks p+1..p+11 of the ring, i.e. the upper copies of both new
        // blocks and, at p+1, the old block p-9 that slot 0's last tap needs: the lower copies
        // (p, p+1) are written after the windows
        float* vb = vring[p];
        vb[wa_x + 640] = a.x;
        vb[wb_x + 640] = b.x;
        vb[wa_y + 640] = a.y;
        vb[wb_y + 640] = b.y;
        wave_sync();
        if (emit) {
            // tap t of the slot at block q reads block q - t = ring q + 10 - t, half t & 1
            const float* v = &vring[p][u];
            f2 acc;
#pragma unroll
            for (int t = 0; t < 10; t++) {
                const f2 x = f2{v[64 * (20 * (t & 1) + 10 - t)], v[64 * (20 * (t & 1) + 11 - t)]};
                const f2 pr = x * cw[t];
                acc = t == 0 ? pr : acc + pr;
            }
            res0 = acc.x;
            res1 = acc.y;
        }
        wave_sync();
        vb[wa_x] = a.x;
        vb[wb_x] = b.x;
        vb[wa_y] = a.y;
        vb[wb_y] = b.y;
    };

    const size_t spf = kDown ? 1024 : 2048, sps = kDown ? 32 : 64;  // output samples per frame / slot

    // The chunk's slots (9 history slots, then 32 per frame) run as a software pipeline of 4-slot
    // groups: the rows of group g+1 are loaded while group g computes, and group g's PCM is
    // stored after an explicit vmcnt(0) (vmem_drain): vmcnt counts loads and stores in issue order,
    // so a store issued before the next group's loads would otherwise make every row load wait for
    // the previous slot's PCM to reach memory (one global round trip per slot).
    auto uni = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane(x); };  // (int -> uint32, no sign extension)
    auto uptr = [&](const float* p) {
        const uint64_t v = reinterpret_cast<uint64_t>(p);
        return (const gfloat*)(((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v));
    };
    static_assert(offsetof(SbrRec, flags) == 2 && offsetof(SbrRec, kx_prev) == 6 && offsetof(SbrRec, M_prev) == 7 &&
                      offsetof(SbrRec, first) == 11 && offsetof(SbrRec, t_E) == 12 && offsetof(SbrRec, slot) == 64,
                  "SbrRec field offsets used by the synthesis");
    auto rec_load = [&](int j, SynRec& W) {
        if (j >= (int)ck.n) return;
        const uint32_t* r = reinterpret_cast<const uint32_t*>(A.recs + (size_t)(ck.frame0 + j) * nch + rc);
        W.w0 = r[0];
        W.w1 = r[1];
        W.w2 = r[2];
        W.w3 = r[3];
        W.slot = r[16];
    };
    // frame j >= 0 of the chunk from its record fields
    auto frame_src = [&](int j, const SynRec& W) {
        SynSrc S{};
        const uint32_t f = ck.frame0 + (uint32_t)j;
        const uint32_t cf = f * nch + rc;
        const uint32_t flags = uni(W.w0 >> 16) & 0xFF, first = uni(W.w2 >> 24) & 0xFF;
        S.rows = 32;
        S.emit = true;
        S.n0 = batch_frame(A, f) * spf;
        if (ps) {
            // a frame without PS data: SBR1.process synthesises X with qmfs0 and copies the left
            // channel to the right one (A/sbr/SBR1.java:75-81); qmfs1 does not run
            const bool ps_on = (flags & kSbrPsOn) != 0;
            if (c == 1 && !ps_on) S.rows = 0;
            S.dup = !ps_on;
            S.xs = uptr(A.xps + ((size_t)f * 2 + c) * 4096);
            return S;
        }
        S.xs = uptr(A.xsyn + (size_t)cf * 4096);
        // rows l < t_E[0]: Xsbr rows 2..7 carried from frame f-1 (its carry rows 2..7 = rows
        // 34..39), kx_prev + M_prev bands
        S.t0 = (int)(uni(W.w3) & 0xFF);
        S.xc = first ? uptr(&A.state[(size_t)uni(W.slot) * 2 + c].xcarry[0][0][0])
                     : uptr(A.xcarry + (size_t)(cf - nch) * kSbrCarryFloats);
        S.kprev = (int)((uni(W.w1) >> 16) & 0xFF) + (int)(uni(W.w1) >> 24);
        return S;
    };
    // frame -1: the v history (slots 23..31 of the frame before the chunk)
    auto history_src = [&]() {
        SynSrc S{};
        const uint32_t cf0 = uni(ck.frame0 * nch + rc);
        const SbrRec& R0 = A.recs[cf0];
        // PS right channel (qmfs1): history of the previous frame that carried PS data
        const uint32_t back = uni((ps && c == 1) ? R0.ps_back : (R0.first ? 0u : 1u));
        if (back == 0) S.xs = uptr(&A.state[(size_t)uni(R0.slot) * 2 + c].xsyn[0][0][0]);
        else if (ps) S.xs = uptr(A.xps + ((size_t)(ck.frame0 - back) * 2 + c) * 4096) + 23 * 128;
        else S.xs = uptr(A.xsyn + (size_t)(cf0 - nch) * 4096) + 23 * 128;
        S.rows = 9;
        return S;
    };
    // slots per software-pipeline group: the next group's rows are loaded while this one computes
#ifndef JAAD_SYN_GROUP
#define JAAD_SYN_GROUP 4
#endif
    constexpr int kG = JAAD_SYN_GROUP;
    static_assert(kG % 2 == 0, "slots run in pairs");
    auto load_group = [&](const SynSrc& S, int l0, float (&ga)[kG], float (&gb)[kG], int (&kl)[kG]) {
#pragma unroll
        for (int i = 0; i < kG; i++) {
            const int l = max(min(l0 + i, S.rows - 1), S.lo);  // (rows past the frame's last are not used)
            const bool carry = l < S.t0;
            kl[i] = carry ? S.kprev : kb;
            fetch(carry ? S.xc + (l + 2) * 128 : S.xs + l * 128, ga[i], gb[i]);
        }
    };
    const bool f32 = (A.out_mode & JAAD_PCM_FLOAT32) != 0;
    const bool swap = !(A.out_mode & JAAD_PCM_LITTLE_ENDIAN);
    // PCM sample n (frame-major, 2 channels) of this channel; a frame without PS data or a mono
    // core writes both channels (SampleBuffer duplicates an SCE, SBR1 copies L to R)
    auto store_pcm = [&](const SynSrc& S, size_t n, float v) {
        const bool one = (nch == 2 || ps) && !S.dup;  // this channel's half of the word
        if (f32) {
            float* o = reinterpret_cast<float*>(A.pcm) + 2 * n;
            if (one) o[c] = v;
            else *reinterpret_cast<float2*>(o) = make_float2(v, v);
        } else {
            const uint32_t w = java_round16_pair(v, swap);
            if (one) reinterpret_cast<uint16_t*>(A.pcm)[2 * n + c] = (uint16_t)w;
            else reinterpret_cast<uint32_t*>(A.pcm)[n] = w;
        }
    };
    auto store_group = [&](const SynSrc& S, int l0, const float (&res)[kG]) {
        if (!S.emit) return;
#pragma unroll
        for (int i = 0; i < kG; i++) {
            const int l = l0 + i;
            if (l >= S.rows) break;
            store_pcm(S, S.n0 + sps * l + u, res[i]);
        }
    };

    if constexpr (kDown) {
        synthesis32(A, ck, wave, history_src, frame_src, rec_load, cw, store_pcm);
        return;
    }

    // the history's 9 slots go to ring blocks 1..9 behind a dummy slot at block 0 (overwritten by
    // the first frame's slot 0 before any window reads it), so every frame's slot pairs start at
    // an even block
    SynSrc S = history_src();
    S.xs -= 128;
    S.rows = 10;
    S.lo = 1;
    SynRec W{};                  // record fields of frame j + 1
    rec_load(0, W);
    int p = 0;                   // ring block of the next pair's first slot
    float ga[kG] = {}, gb[kG] = {};
    int kl[kG];
    load_group(S, 0, ga, gb, kl);
    vmem_drain();
    bool have = true;            // ga/gb hold the rows of the group about to run
    for (int j = -1;;) {
        for (int l0 = 0; l0 < S.rows; l0 += kG) {
            if (!have) {         // first group after a frame without rows
                load_group(S, l0, ga, gb, kl);
                vmem_drain();
            }
            have = false;
            float na[kG] = {}, nb[kG] = {};
            int nk[kG];
            // the next group: later rows of this frame or the first rows of the next one (only
            // scalar selects branch; the loads themselves are unconditional, a reload of the
            // current rows when there is nothing to fetch)
            SynSrc Sn = S;
            int ln = l0 + kG;
            if (ln >= S.rows) {
                have = false;
                if (j + 1 < (int)ck.n) {
                    const SynSrc F = frame_src(j + 1, W);
                    if (F.rows) {
                        Sn = F;
                        ln = 0;
                        have = true;
                    }
                }
                if (!have) ln = l0;
            } else {
                have = true;
            }
            load_group(Sn, ln, na, nb, nk);
            float res[kG] = {};
#pragma unroll
            for (int i = 0; i < kG; i += 2) {
                if (l0 + i >= S.rows) break;  // (rows come in pairs: 10 or 32)
                mask(kl[i], ga[i], gb[i]);
                mask(kl[i + 1], ga[i + 1], gb[i + 1]);
                slot_pair(ga[i], gb[i], ga[i + 1], gb[i + 1], p, S.emit, res[i], res[i + 1]);
                p = p == 8 ? 0 : p + 2;
            }
            vmem_drain();
            store_group(S, l0, res);
#pragma unroll
            for (int i = 0; i < kG; i++) {
                ga[i] = na[i];
                gb[i] = nb[i];
                kl[i] = nk[i];
            }
        }
        if (++j >= (int)ck.n) break;
        S = frame_src(j, W);
        rec_load(j + 1, W);
    }
}

// ---------------------------------------------------------------------------------------------
// slot state after the last frame of each run
// ---------------------------------------------------------------------------------------------
// A wave's copy of N floats (N % 4 == 0, both ends 16-byte aligned) in two halves: wave_load issues
// the float4 loads into registers (unconditional: a clamped duplicate instead of a branch per load),
// wave_store writes them.  sbr_state_kernel issues every load of a slot's state before the first
// store: copied element by element, each store would make the next load wait a memory round trip
// behind it (the state and the rows may alias as far as the compiler knows) -- 49 round trips per wave.
template <int N>
constexpr int wave_copy_regs() { return (N / 4 + 63) / 64; }
template <int N>
__device__ __forceinline__ void wave_load(float4 (&v)[wave_copy_regs<N>()], const float* src, int u)
{
    static_assert(N % 4 == 0, "wave_load: float4 units");
    const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
    for (int i = 0; i < wave_copy_regs<N>(); i++) v[i] = s4[min(u + 64 * i, N / 4 - 1)];
}
template <int N>
__device__ __forceinline__ void wave_store(const float4 (&v)[wave_copy_regs<N>()], float* dst, int u)
{
    float4* d4 = reinterpret_cast<float4*>(dst);
#pragma unroll
    for (int i = 0; i < wave_copy_regs<N>(); i++)
        if (u + 64 * i < N / 4) d4[u + 64 * i] = v[i];
}
static_assert(offsetof(SbrChState, xcarry) % 16 == 0 && offsetof(SbrChState, xsyn) % 16 == 0 &&
                  offsetof(SbrChState, gq) % 16 == 0 && sizeof(SbrChState) % 16 == 0,
              "sbr_state_kernel copies float4s");

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void sbr_state_kernel(SbrArgs A)
{
    const uint32_t i = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (i >= A.n_last) return;
    const int u = lane_id();
    const uint32_t cf = A.last_cf[i];
    const int c = (int)(cf % (uint32_t)A.nch);
    // the record's fields first (vmcnt counts in issue order: a wait for them must not wait for the
    // rows), then the parts whose source depends on cf alone, in flight while the record arrives
    const SbrRec& R = A.recs[cf];
    const uint32_t slot = R.slot, flags = R.flags, ps_back = R.ps_back, kb = R.blim;
    float4 vt[wave_copy_regs<288>()], vc[wave_copy_regs<kSbrCarryFloats>()], vg[wave_copy_regs<640>()];
    wave_load<288>(vt, A.time + batch_cf(A, cf) * 1024 + 736, u);
    wave_load<kSbrCarryFloats>(vc, A.xcarry + (size_t)cf * kSbrCarryFloats, u);
    wave_load<640>(vg, A.gq + (size_t)cf * 640, u);
    // synthesis history: the channel's own rows, or with PS both output channels' from xps -- the
    // right channel's synthesis (qmfs1) last ran on the run's last PS frame (none in this call:
    // its history stays)
    float4 vs0[wave_copy_regs<9 * 128>()], vs1[wave_copy_regs<9 * 128>()];
    const bool ps_right = A.ps && ((flags & kSbrPsOn) || ps_back != 0);
    const size_t fs1 = (flags & kSbrPsOn) ? cf : cf - ps_back;
    wave_load<9 * 128>(vs0, A.ps ? A.xps + (size_t)cf * 2 * 4096 + 23 * 128 : A.xsyn + (size_t)cf * 4096 + 23 * 128, u);
    if (A.ps) wave_load<9 * 128>(vs1, A.xps + ((ps_right ? fs1 : cf) * 2 + 1) * 4096 + 23 * 128, u);  // (xps is null without PS)
    // bands from the run's limit up are not written by the stages (SbrRec::blim): the state keeps
    // them zero, as a later call with a higher limit reads them
    auto band_mask = [&](float4 (&v)[wave_copy_regs<9 * 128>()]) {
#pragma unroll
        for (int i = 0; i < wave_copy_regs<9 * 128>(); i++) {
            const uint32_t b = 2 * ((uint32_t)(u + 64 * i) & 31);  // float4 = bands b, b + 1 of a row
            if (b >= kb) v[i].x = v[i].y = 0.0f;
            if (b + 1 >= kb) v[i].z = v[i].w = 0.0f;
        }
    };
    band_mask(vs0);
    if (A.ps) band_mask(vs1);
    SbrChState& S = A.state[(size_t)slot * 2 + c];
    wave_store<288>(vt, S.tail, u);
    wave_store<kSbrCarryFloats>(vc, &S.xcarry[0][0][0], u);
    wave_store<640>(vg, &S.gq[0][0][0], u);
    wave_store<9 * 128>(vs0, &S.xsyn[0][0][0], u);  // (PS: c = 0, the left output channel)
    if (ps_right) wave_store<9 * 128>(vs1, &A.state[(size_t)slot * 2 + 1].xsyn[0][0][0], u);
}

// ---------------------------------------------------------------------------------------------
// JAAD_SBR_UPSAMPLE frames: SBR.upsample (A/sbr/SBR.java:302-309) of the core output -- data[2i] =
// data[2i+1] = core[i] for i = len/2-1 .. 1, data[0] and data[1] keep core[0] and core[1] -- then
// SampleBuffer.accept; one channel (SCE, PS) is accepted once and duplicated to stereo
// (A/syntax/SyntacticElements.java:243-245).  Downsampled SBR (frame length = sample length):
// the core as it is (A/syntax/CPE.java:201).  One block per frame.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sbr_upsample_kernel(SbrArgs A)
{
    const size_t f = A.ups[blockIdx.x];
    const int nch = A.nch;
    const float* c0 = A.time + (size_t)f * nch * 1024;
    const float* c1 = nch == 2 ? c0 + 1024 : c0;
    const int spf = A.down ? 1024 : 2048;
    for (int n = threadIdx.x; n < spf; n += blockDim.x) {
        const int k = A.down ? n : (n == 1 ? 1 : n >> 1);
        const float l = c0[k], r = c1[k];
        const size_t o = (size_t)f * spf + n;
        if (A.out_mode & JAAD_PCM_FLOAT32) {
            reinterpret_cast<float2*>(A.pcm)[o] = make_float2(l, r);
        } else {
            uint32_t sl = (uint32_t)(uint16_t)(int16_t)java_round16(l), sr = (uint32_t)(uint16_t)(int16_t)java_round16(r);
            if (!(A.out_mode & JAAD_PCM_LITTLE_ENDIAN)) {
                sl = ((sl & 0xFF) << 8) | (sl >> 8);
                sr = ((sr & 0xFF) << 8) | (sr >> 8);
            }
            reinterpret_cast<uint32_t*>(A.pcm)[o] = sl | (sr << 16);
        }
    }
}

}  // namespace

hipError_t launch_sbr(const SbrArgs& a, hipStream_t stream, const uint32_t* fix_dev, const uint32_t* fix_counts,
                      int n_fix_passes)
{
    if (a.n_ups) hipLaunchKernelGGL(sbr_upsample_kernel, dim3(a.n_ups), dim3(256), 0, stream, a);
    const dim3 blk(256);
    if (a.n_cf) {
        const dim3 g((a.n_cf + kWavesPerBlock - 1) / kWavesPerBlock);
        // no smoothing and no fix pass: the analysis runs inside the HF kernel (phase 5), X_low never
        // goes through HBM (JAAD_SBR_FUSED=0: the separate kernels, for A/B)
        const char* fz = std::getenv("JAAD_SBR_FUSED");  // (read per launch: tests switch it)
        const bool fuse_ok = !(fz && fz[0] == '0');
        if (fuse_ok && !a.smoothing && n_fix_passes == 0 && !a.n_chains) {
            hipLaunchKernelGGL(sbr_hf_kernel<5>, g, blk, 0, stream, a);
        } else {
        hipLaunchKernelGGL(sbr_analysis_kernel, g, blk, 0, stream, a);
        if (a.smoothing) {
            hipLaunchKernelGGL(sbr_hf_kernel<1>, g, blk, 0, stream, a);
            hipLaunchKernelGGL(sbr_hf_kernel<2>, g, blk, 0, stream, a);
        } else {
            hipLaunchKernelGGL(sbr_hf_kernel<0>, g, blk, 0, stream, a);
        }
        // pass p recomputes the kSbrDep frames p links down a chain: frame f-1's carry rows (and
        // G/Q ring) are final by then
        SbrArgs fa = a;
        fa.fix = fix_dev;
        for (int p = 0; p < n_fix_passes; p++) {
            fa.n_fix = fix_counts[p];
            if (fa.n_fix)
                hipLaunchKernelGGL(sbr_hf_kernel<3>, dim3((fa.n_fix + kWavesPerBlock - 1) / kWavesPerBlock), blk, 0,
                                   stream, fa);
            fa.fix += fix_counts[p];
        }
        if (a.n_chains)  // links past kSbrFixPasses: fa.fix now points at the walker's lists
            hipLaunchKernelGGL(sbr_hf_kernel<4>, dim3((a.n_chains + kWavesPerBlock - 1) / kWavesPerBlock), blk, 0,
                               stream, fa);
        }
    }
    if (a.ps) {
        const hipError_t e = launch_ps(a, stream);
        if (e != hipSuccess) return e;
    }
    if (a.n_chunks) {
        const dim3 g((a.n_chunks + kWavesPerBlock - 1) / kWavesPerBlock);
        if (a.down) hipLaunchKernelGGL(sbr_synthesis_kernel<true>, g, blk, 0, stream, a);
        else hipLaunchKernelGGL(sbr_synthesis_kernel<false>, g, blk, 0, stream, a);
    }
    if (a.n_last)
        hipLaunchKernelGGL(sbr_state_kernel, dim3((a.n_last + kWavesPerBlock - 1) / kWavesPerBlock), blk, 0, stream, a);
    return hipGetLastError();
}

}  // namespace jaad

// ---------------------------------------------------------------------------------------------
// internal self-test entry points (not in the public header): the distributed DCT-IV on its own
// ---------------------------------------------------------------------------------------------
namespace jaad {
namespace {
__global__ void dct_test_kernel(const float* dct, const float* in_re, const float* in_im, float* out_re,
                                float* out_im, int n)
{
    const int u = lane_id();
    const int e = u & 31, E = bitrev5(e);
    const int v = blockIdx.x * 2 + (u >> 5);
    const DctConst K = load_dct_const(dct, e, E);
    const int vv = v < n ? v : n - 1;
    float orr, oi;
    dct4(K, e, E, in_re[32 * vv + e], in_im[32 * vv + e], orr, oi);
    if (v < n) {  // lane e holds output element E
        out_re[32 * v + E] = orr;
        out_im[32 * v + E] = oi;
    }
}
}  // namespace
}  // namespace jaad

extern "C" int jaad__sbr_dct_test(const float* dct_dev, const float* in_re, const float* in_im, float* out_re,
                                  float* out_im, int n)
{
    hipLaunchKernelGGL(jaad::dct_test_kernel, dim3((n + 1) / 2), dim3(64), 0, nullptr, dct_dev, in_re, in_im, out_re,
                       out_im, n);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

namespace jaad {
namespace {
__global__ void math_test_kernel(const float* a, const float* b, float* sq, float* dv, int n)
{
    const int i = blockIdx.x * 64 + lane_id();
    if (i < n) {
        sq[i] = (float)__dsqrt_rn((double)a[i]);
        dv[i] = sqrtf(a[i]);
    }
}
}  // namespace
}  // namespace jaad

extern "C" int jaad__math_test(const float* a, const float* b, float* sq, float* dv, int n)
{
    hipLaunchKernelGGL(jaad::math_test_kernel, dim3((n + 63) / 64), dim3(64), 0, nullptr, a, b, sq, dv, n);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
