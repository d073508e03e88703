// Parametric stereo (HE-AAC v2) for gfx950, A/ = aac/src/main/java/net/sourceforge/jaad/aac/ of the
// reference: PSImpl.process (A/ps/PSImpl.java:685-707) = hybrid analysis (A/ps/Filterbank.java:
// 18-68, T20), decorrelation (:202-400), mixing (:406-681), hybrid synthesis
// (A/ps/Filterbank.java:70-86).  Same binary32 evaluation order as the Java (-ffp-contract=off).
// IPD/OPD phase rotation included (nr_ipdopd_par 11 / 17), with the reference's index quirks.
//
// Only two parts of PS are recurrences across frames: the all-pass / delay lines of the
// decorrelator and the transient detector's peak/smooth IIRs.  Everything else reaches back at
// most one frame and runs frame-parallel (one wave per frame) on what the previous stage left in
// HBM:
//   ps_analysis_kernel  X_left = the SBR output the HF kernel wrote into xps[f][0], rows l < t_E[0]
//                       patched with the carried rows; hybrid analysis -> xhl;
//                       band energies P -> pg                                  (wave per frame)
//   ps_decor_kernel     per run, eight waves: the three all-pass links of the QMF bands (lane =
//                       band) and of the hybrid groups pipelined over waves, transient detector,
//                       mixing-parameter scan (IPD/OPD phase history, h_prev), sequential over
//                       the run's frames; rings in VGPRs with compile-time indices (32 slots per
//                       frame), raw all-pass output -> xps[f][1], xhr; G_TransientRatio -> pg;
//                       H start/delta per (env, group) -> hb (block per run)
//   ps_mix_kernel       H interpolation, G scaling, mixing (+ IPD/OPD rotation), hybrid
//                       synthesis -> xps[f][0..1]                              (wave per frame)
//   ps_state_kernel     filterbank history of each run's last frame -> slot state
#include <hip/hip_runtime.h>

#include <type_traits>

#include "jaad_ps_mix.h"
#include "jaad_sbr.h"
#include "jaad_wave.h"

namespace jaad {
namespace {

constexpr int kBorder[23] = {6, 7, 0, 1, 2, 3, 9, 8, 10, 11, 3, 4, 5, 6, 7, 8, 9, 11, 14, 18, 23, 35, 64};
constexpr float kAlphaDecay = 0.76592833836465f, kAlphaSmooth = 0.25f, kDecaySlope = 0.05f;
constexpr float kCoefSqrt2 = 1.4142135623731f;
constexpr int kPsWaves = 4;  // frames per block of the frame-parallel kernels

__device__ __forceinline__ int group_bk(int gr) { return gr == 0 ? 1 : (gr == 1 ? 0 : gr - 2); }

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// ---------------------------------------------------------------------------------------------
// hybrid filterbank
// ---------------------------------------------------------------------------------------------
// Filter8.DCT3_4_unscaled (A/ps/Filter8.java:122-137)
__device__ __forceinline__ void dct3_4(float x[4])
{
    const float f0 = (x[2] * 0.7071067811865476f);
    const float f1 = x[0] - f0;
    const float f2 = x[0] + f0;
    const float f3 = x[1] + x[3];
    const float f4 = (x[1] * 1.3065629648763766f);
    const float f5 = (f3 * (-0.9238795325112866f));
    const float f6 = (x[3] * (-0.5411961001461967f));
    const float f7 = f4 + f5;
    const float f8 = f6 - f5;
    x[3] = f2 - f8;
    x[0] = f2 + f8;
    x[2] = f1 - f7;
    x[1] = f1 + f7;
}

// Filter8.filter for one time slot (A/ps/Filter8.java:54-119), b = 13 window samples; sub-bands
// 3+4 and 2+5 merged afterwards (A/ps/Filterbank.java:55-67)
__device__ __forceinline__ void filter8(const float2 b[13], const float* c, float2 out[8])
{
    float r1[4], i1[4], r2[4], i2[4], x[4], re[8], im[8];
    r1[0] = (c[6] * b[6].x);
    r1[1] = (c[5] * (b[5].x + b[7].x));
    r1[2] = -(c[0] * (b[0].x + b[12].x)) + (c[4] * (b[4].x + b[8].x));
    r1[3] = -(c[1] * (b[1].x + b[11].x)) + (c[3] * (b[3].x + b[9].x));
    i1[0] = (c[5] * (b[7].y - b[5].y));
    i1[1] = (c[0] * (b[12].y - b[0].y)) + (c[4] * (b[8].y - b[4].y));
    i1[2] = (c[1] * (b[11].y - b[1].y)) + (c[3] * (b[9].y - b[3].y));
    i1[3] = (c[2] * (b[10].y - b[2].y));
    for (int n = 0; n < 4; n++) x[n] = r1[n] - i1[3 - n];
    dct3_4(x);
    re[7] = x[0]; re[5] = x[2]; re[3] = x[3]; re[1] = x[1];
    for (int n = 0; n < 4; n++) x[n] = r1[n] + i1[3 - n];
    dct3_4(x);
    re[6] = x[1]; re[4] = x[3]; re[2] = x[2]; re[0] = x[0];
    i2[0] = (c[6] * b[6].y);
    i2[1] = (c[5] * (b[5].y + b[7].y));
    i2[2] = -(c[0] * (b[0].y + b[12].y)) + (c[4] * (b[4].y + b[8].y));
    i2[3] = -(c[1] * (b[1].y + b[11].y)) + (c[3] * (b[3].y + b[9].y));
    r2[0] = (c[5] * (b[7].x - b[5].x));
    r2[1] = (c[0] * (b[12].x - b[0].x)) + (c[4] * (b[8].x - b[4].x));
    r2[2] = (c[1] * (b[11].x - b[1].x)) + (c[3] * (b[9].x - b[3].x));
    r2[3] = (c[2] * (b[10].x - b[2].x));
    for (int n = 0; n < 4; n++) x[n] = i2[n] + r2[3 - n];
    dct3_4(x);
    im[7] = x[0]; im[5] = x[2]; im[3] = x[3]; im[1] = x[1];
    for (int n = 0; n < 4; n++) x[n] = i2[n] - r2[3 - n];
    dct3_4(x);
    im[6] = x[1]; im[4] = x[3]; im[2] = x[2]; im[0] = x[0];
    for (int k = 0; k < 8; k++) out[k] = make_float2(re[k], im[k]);
    out[3] = make_float2(out[3].x + out[4].x, out[3].y + out[4].y);
    out[4] = make_float2(0.0f, 0.0f);
    out[2] = make_float2(out[2].x + out[5].x, out[2].y + out[5].y);
    out[5] = make_float2(0.0f, 0.0f);
}

// Filter2.filter for one time slot (A/ps/Filter2.java:40-67)
__device__ __forceinline__ void filter2(const float2 b[13], const float* c, float2 out[2])
{
    const float r0 = (c[0] * (b[0].x + b[12].x)), r1 = (c[1] * (b[1].x + b[11].x));
    const float r2 = (c[2] * (b[2].x + b[10].x)), r3 = (c[3] * (b[3].x + b[9].x));
    const float r4 = (c[4] * (b[4].x + b[8].x)), r5 = (c[5] * (b[5].x + b[7].x)), r6 = (c[6] * b[6].x);
    const float i0 = (c[0] * (b[0].y + b[12].y)), i1 = (c[1] * (b[1].y + b[11].y));
    const float i2 = (c[2] * (b[2].y + b[10].y)), i3 = (c[3] * (b[3].y + b[9].y));
    const float i4 = (c[4] * (b[4].y + b[8].y)), i5 = (c[5] * (b[5].y + b[7].y)), i6 = (c[6] * b[6].y);
    out[0] = make_float2(r0 + r1 + r2 + r3 + r4 + r5 + r6, i0 + i1 + i2 + i3 + i4 + i5 + i6);
    out[1] = make_float2(r0 - r1 + r2 - r3 + r4 - r5 + r6, i0 - i1 + i2 - i3 + i4 - i5 + i6);
}

// X_left row l < 38 of frame f for QMF band u: Xsbr rows l + 2 as SBR1.processPS assembles them
// (A/sbr/SBR1.java:102-120): rows l < t_E[0] carried from frame f-1 (its carry rows l + 2) with
// kx_prev + M_prev bands, rows 32..37 = Xsbr rows 34..39 (carry rows 2..7) for bands < 5
__device__ __forceinline__ const float2* x_carry_prev(const SbrArgs& A, const SbrRec& R, uint32_t f)
{
    return R.first ? reinterpret_cast<const float2*>(&A.state[(size_t)R.slot * 2].xcarry[0][0][0])
                   : reinterpret_cast<const float2*>(A.xcarry + (size_t)(f - 1) * kSbrCarryFloats);
}

// Filterbank.buffer after frame f, element i of band b: work[32 + i] = X_left[26 + i][b] (b < 3)
__device__ __forceinline__ float2 hyb_history_after(const SbrArgs& A, uint32_t f, int b, int i)
{
    return i < 6 ? reinterpret_cast<const float2*>(A.xps + (size_t)f * 8192)[(26 + i) * 64 + b]
                 : reinterpret_cast<const float2*>(A.xcarry + (size_t)f * kSbrCarryFloats)[(i - 4) * 64 + b];
}

// (rows transposed through LDS: the hybrid analysis reads bands 0..2 of rows 0..37, the band
// energies |X|^2 of rows 0..31 -- stored as energies, not complex rows, so four waves fit a CU's
// LDS per block and four blocks a CU instead of two)
struct AnaLds {
    float2 xl3[38][3];
    float en[32][65];
    float2 hist[3][12];
};

__global__ __launch_bounds__(256) void ps_analysis_kernel(SbrArgs A)
{
    __shared__ AnaLds lds_s[kPsWaves];
    const int wave = threadIdx.x >> 6, u = lane_id();
    const uint32_t f = blockIdx.x * kPsWaves + wave;
    if (f >= A.n_cf) return;
    AnaLds& L = lds_s[wave];
    const SbrRec& R = A.recs[f];
    const PsConst& K = *A.psc;
    {
        const int t0 = R.t_E[0], kprev = R.kx_prev + R.M_prev, K = R.blim;
        // The HF kernel wrote this frame's X rows into X_left's place (xs = xo): only rows
        // l < t_E[0] are replaced, by the carried ones.
        float2* xo = reinterpret_cast<float2*>(A.xps + (size_t)f * 8192);
        const float2* xs = xo;
        const float2* xc = x_carry_prev(A, R, f);
        const float2* xn = reinterpret_cast<const float2*>(A.xcarry + (size_t)f * kSbrCarryFloats);
        // every row load is issued before the first store: a load-store-load loop would wait out
        // one global round trip per row.  Bands >= the run's limit K are zero (SbrRec::blim): their
        // lanes read lane 0's word (no extra bytes) and store nothing.
        const bool ps_on = (R.flags & kSbrPsOn) != 0;
        float2 v[38];
#pragma unroll
        for (int l = 0; l < 38; l++) {
            const float2* src = l >= 32 ? xn + (l - 30) * 64 : l < t0 ? xc + (l + 2) * 64 : xs + l * 64;
            const bool ok = l >= 32 ? u < 5 && ps_on : l < t0 ? u < kprev : u < K;
            const float2 t = src[ok ? u : 0];
            v[l] = ok ? t : make_float2(0.0f, 0.0f);
        }
#pragma unroll
        for (int l = 0; l < 32; l++) {
            L.en[l][u] = (v[l].x * v[l].x) + (v[l].y * v[l].y);
            if (u < 3) L.xl3[l][u] = v[l];
        }
        if (u < K)
#pragma unroll
            for (int l = 0; l < 32; l++)
                if (l < t0) xo[l * 64 + u] = v[l];
        // a frame without PS data only hands its X (qmfs0 input) to the synthesis
        if (!ps_on) return;
        if (u < 3)
#pragma unroll
            for (int l = 32; l < 38; l++) L.xl3[l][u] = v[l];
        if (u < 36) {
            // Filterbank.buffer as the previous PS frame left it (frames without PS data do not
            // run the hybrid analysis)
            const int b = u / 12, i = u % 12;
            float2 h;
            if (R.ps_back == 0) {
                const PsState& S = A.pss[R.slot];
                h = S.init ? make_float2(S.hyb[b][i][0], S.hyb[b][i][1]) : make_float2(0.0f, 0.0f);
            } else {
                h = hyb_history_after(A, f - R.ps_back, b, i);
            }
            L.hist[b][i] = h;
        }
    }
    wave_sync();
    if (u >= 32) return;
    const int n = u;
    float2 hy[12];
    {
        float2 b[13];
        for (int band = 0; band < 3; band++) {
#pragma unroll
            for (int i = 0; i < 13; i++) {
                const int w = n + i;  // work[w]: history (w < 12) or X_left[w - 6]
                b[i] = w < 12 ? L.hist[band][w] : L.xl3[w - 6][band];
            }
            if (band == 0) filter8(b, K.p8, hy);
            else filter2(b, K.p2, hy + 6 + 2 * band);
        }
    }
    float2* xh = reinterpret_cast<float2*>(A.xhl + (size_t)f * 768) + n * 12;
#pragma unroll
    for (int k = 0; k < 12; k++) xh[k] = hy[k];
    // P[n][bk] in group order (PSImpl.java:213-236)
    float P[20];
#pragma unroll
    for (int k = 0; k < 20; k++) P[k] = 0.0f;
#pragma unroll
    for (int gr = 0; gr < 22; gr++) {
        const int bk = group_bk(gr);
        if (gr < 10) {
            const float2 v = hy[kBorder[gr]];
            P[bk] += (v.x * v.x) + (v.y * v.y);
        } else {
#pragma unroll
            for (int sb = kBorder[gr]; sb < kBorder[gr + 1]; sb++) P[bk] += L.en[n][sb];
        }
    }
    float* pg = A.pg + (size_t)f * 640 + n * 20;
#pragma unroll
    for (int k = 0; k < 20; k++) pg[k] = P[k];
}

// ---------------------------------------------------------------------------------------------
// mixing parameters (PSImpl.ps_mix_phase :419-590): parameter-only, but the IPD/OPD phase history
// and h_prev run through every frame, so one wave per run scans them (lane = parameter band)
// ---------------------------------------------------------------------------------------------
// target mixing coefficients (real parts) of envelope env, group gr (:433-482)
__device__ __forceinline__ void ps_h(const PsConst& K, const jaad_ps_frame& P, int env, int gr, float h[4])
{
    const int bk = group_bk(gr);
    const int fine = P.iid_mode >= 3;
    const int steps = fine ? 15 : 7;
    int iid = P.iid[env][bk];
    const int sign = iid < 0 ? -1 : 1;
    iid = iid < 0 ? -iid : iid;
    const int icc = P.icc[env][bk];
    if (P.icc_mode < 3) {  // type 'A'
        const float c1 = K.sf_iid[fine][steps + iid], c2 = K.sf_iid[fine][steps - iid];
        const float cosa = K.cos_alphas[icc], sina = K.sin_alphas[icc];
        const float cosb = K.cos_betas[fine][iid][icc];
        const float sinb = K.sin_betas[fine][iid][icc] * (float)sign;
        const float ab1 = (cosb * cosa), ab2 = (sinb * sina), ab3 = (sinb * cosa), ab4 = (cosb * sina);
        h[0] = (c2 * (ab1 - ab2));
        h[1] = (c1 * (ab1 + ab2));
        h[2] = (c2 * (ab3 + ab4));
        h[3] = (c1 * (ab3 - ab4));
    } else {  // type 'B'
        const float cosa = K.sincos_b[fine][steps + iid][icc];
        const float sina = K.sincos_b[fine][2 * steps - (steps + iid)][icc];
        const float cosg = K.cos_gammas[fine][iid][icc], sing = K.sin_gammas[fine][iid][icc];
        h[0] = (kCoefSqrt2 * (cosa * cosg));
        h[1] = (kCoefSqrt2 * (sina * cosg));
        h[2] = (kCoefSqrt2 * (-cosa * sing));
        h[3] = (kCoefSqrt2 * (sina * sing));
    }
}

__device__ __forceinline__ float magnitude_c(float re, float im)
{
    // (float)Math.sqrt(double) of a float argument == correctly rounded sqrtf (:402-404)
    return sqrtf((re * re) + (im * im));
}

// Lane bk walks its groups in group order (bk 0: groups 1, 2; bk 1: groups 0, 3; else bk + 2)
// over every envelope of every frame of the run.  The shared phase_hist counter flips once per
// (group, envelope) with bk < nr_ipdopd_par; those groups are always 0 .. nr + 1, so the
// counter at (gr, env) is phase_hist(frame start) + gr * num_env + env.
// The walk is sequential over the run's frames and each (envelope, group) step reads the frame
// record and then table entries it indexes: the record of frame j+1 is fetched into registers
// while frame j is scanned and parked in LDS (pbuf, double-buffered) at its end; K is the
// block's LDS copy of PsConst.
constexpr int kPsFrameDw = (int)(sizeof(jaad_ps_frame) / 4);
constexpr int kPsFrameDwPerLane = (kPsFrameDw + 19) / 20;
static_assert(sizeof(jaad_ps_frame) % 4 == 0, "PS records are copied dword-wise");

// One lane per parameter band (u < 20), frame by frame: scan_init, scan_frame(j) for j = 0 ..
// nfr-1, scan_finish.  The scan's arrays are the caller's locals (kept out of a struct so that they
// stay in registers: a dynamically indexed array member would go to scratch).
struct ScanCtx {
    const SbrArgs& A;
    const PsConst& K;
    const uint32_t* fl;
    uint32_t nfr;
    PsState& S;
    int u;
    uint32_t (*pbuf)[kPsFrameDw];
};
struct ScanArrays {
    uint32_t (&pre)[kPsFrameDwPerLane];
    int (&grs)[2];
    float (&hp)[2][8];
    float (&ipd)[2][2];
    float (&opd)[2][2];
    int& phase;
};

__device__ __forceinline__ void scan_fetch(const ScanCtx& C, const ScanArrays& Z, uint32_t f)
{
    const uint32_t* src = reinterpret_cast<const uint32_t*>(C.A.psf + f);
#pragma unroll
    for (int i = 0; i < kPsFrameDwPerLane; i++) {
        const int d = C.u + 20 * i;
        Z.pre[i] = d < kPsFrameDw ? src[d] : 0u;
    }
}
__device__ __forceinline__ void scan_park(const ScanCtx& C, const ScanArrays& Z, uint32_t* dst)
{
#pragma unroll
    for (int i = 0; i < kPsFrameDwPerLane; i++) {
        const int d = C.u + 20 * i;
        if (d < kPsFrameDw) dst[d] = Z.pre[i];
    }
}
__device__ __forceinline__ void scan_init(const ScanCtx& C, const ScanArrays& Z, bool fresh)
{
    scan_fetch(C, Z, C.fl[0]);
    scan_park(C, Z, C.pbuf[0]);
    wave_sync();
    const int bk = C.u;
    Z.grs[0] = bk == 0 ? 1 : (bk == 1 ? 0 : bk + 2);
    Z.grs[1] = bk == 0 ? 2 : (bk == 1 ? 3 : -1);
    for (int j = 0; j < 2; j++)
        for (int k = 0; k < 8; k++) {
            const int gr = Z.grs[j] < 0 ? 0 : Z.grs[j];
            // PSImpl constructor (:87-92): h11_prev = (1, 0), h12_prev = (0, 1), h21/h22 = 0
            Z.hp[j][k] = fresh ? (k == 0 || k == 5 ? 1.0f : 0.0f) : C.S.h_prev[gr][k];
        }
    for (int ph = 0; ph < 2; ph++)
        for (int c = 0; c < 2; c++) {
            Z.ipd[ph][c] = fresh ? 0.0f : C.S.ipd_prev[bk][ph][c];
            Z.opd[ph][c] = fresh ? 0.0f : C.S.opd_prev[bk][ph][c];
        }
    Z.phase = fresh ? 0 : C.S.phase_hist;
    if (C.nfr > 1) scan_fetch(C, Z, C.fl[1]);  // lands during frame 0's scan
}
// frame j (its record parked in pbuf[j & 1]); frame j + 1's record (fetched during frame j) is
// parked at its end and frame j + 2's fetched
__device__ __forceinline__ void scan_frame(const ScanCtx& C, const ScanArrays& Z, uint32_t j)
{
    const SbrArgs& A = C.A;
    const PsConst& K = C.K;
    const int bk = C.u;
    float (&hp)[2][8] = Z.hp;
    float (&ipd)[2][2] = Z.ipd;
    float (&opd)[2][2] = Z.opd;
    const uint32_t f = C.fl[j];
    const jaad_ps_frame& P = *reinterpret_cast<const jaad_ps_frame*>(C.pbuf[j & 1]);
    const int E = P.num_env, nr = P.nr_ipdopd_par;
    const bool elig = bk < nr;
    float* hbf = A.hb + (size_t)f * (5 * 22 * 16);
    for (int g = 0; g < 2; g++) {
        const int gr = Z.grs[g];
        if (gr < 0) break;
        for (int env = 0; env < E; env++) {
            float h[8];
            ps_h(K, P, env, gr, h);
            h[4] = h[5] = h[6] = h[7] = 0.0f;
            if (elig) {  // phase rotation (:484-567)
                const int ph = (Z.phase + gr * E + env) & 1;
                float* ip = ipd[ph];
                float* op = opd[ph];
                float tl0 = (ip[0] * 0.25f), tl1 = (ip[1] * 0.25f);
                float tr0 = (op[0] * 0.25f), tr1 = (op[1] * 0.25f);
                const int idx = P.ipd[env][bk] < 0 ? -P.ipd[env][bk] : P.ipd[env][bk];  // IPD for both
                ip[0] = K.ipdopd_cos[idx];
                ip[1] = K.ipdopd_sin[idx];
                op[0] = K.ipdopd_cos[idx];
                op[1] = K.ipdopd_sin[idx];
                tl0 += ip[0];
                tl1 += ip[1];
                tr0 += op[0];
                tr1 += op[1];
                const float* pp = opd[ph ^ 1];  // value before previous: opd.prev for both
                tl0 += (pp[0] * 0.5f);
                tl1 += (pp[1] * 0.5f);
                tr0 += (pp[0] * 0.5f);
                tr1 += (pp[1] * 0.5f);
                const float xy = magnitude_c(tr0, tr1), pq = magnitude_c(tl0, tl1);
                float pl0 = 0.0f, pl1 = 0.0f, pr0 = 0.0f, pr1 = 0.0f;
                if (xy != 0.0f) {
                    pl0 = __fdiv_rn(tr0, xy);
                    pl1 = __fdiv_rn(tr1, xy);
                }
                const float xypq = (xy * pq);
                if (xypq != 0.0f) {
                    const float tmp1 = (tr0 * tl0) + (tr1 * tl1);
                    const float tmp2 = (tr1 * tl0) - (tr0 * tl1);
                    pr0 = __fdiv_rn(tmp1, xypq);
                    pr1 = __fdiv_rn(tmp2, xypq);
                }
                h[4] = (h[0] * pl1);
                h[5] = (h[1] * pr1);
                h[6] = (h[2] * pl1);
                h[7] = (h[3] * pr1);
                h[0] = (h[0] * pl0);
                h[1] = (h[1] * pr0);
                h[2] = (h[2] * pl0);
                h[3] = (h[3] * pr0);
            }
            const float Lf = (float)(P.border[env + 1] - P.border[env]);
            float* o = hbf + (env * 22 + gr) * 16;
            for (int k = 0; k < 4; k++) {
                o[8 + k] = __fdiv_rn(h[k] - hp[g][k], Lf);
                o[k] = hp[g][k];
                hp[g][k] = h[k];
            }
            for (int k = 4; k < 8; k++) {
                float d = 0.0f, st = 0.0f;
                if (elig) {
                    d = __fdiv_rn(h[k] - hp[g][k], Lf);
                    st = hp[g][k];
                    if (bk != 0) {  // FBType.bkm tests the band bits (A/ps/FBType.java:71-73)
                        d = -d;
                        st = -st;
                    }
                    hp[g][k] = h[k];
                }
                o[8 + k] = d;
                o[k] = st;
            }
        }
    }
    if (nr) Z.phase = (Z.phase + (nr + 2) * E) & 1;
    if (j + 1 < C.nfr) {
        wave_sync();  // every lane is done with buffer (j + 1) & 1's previous frame
        scan_park(C, Z, C.pbuf[(j + 1) & 1]);
        wave_sync();
        if (j + 2 < C.nfr) scan_fetch(C, Z, C.fl[j + 2]);  // lands during frame j + 1's scan
    }
}
__device__ __forceinline__ void scan_finish(const ScanCtx& C, const ScanArrays& Z)
{
    const int bk = C.u;
    for (int g = 0; g < 2; g++)
        if (Z.grs[g] >= 0)
            for (int k = 0; k < 8; k++) C.S.h_prev[Z.grs[g]][k] = Z.hp[g][k];
    for (int ph = 0; ph < 2; ph++)
        for (int c = 0; c < 2; c++) {
            C.S.ipd_prev[bk][ph][c] = Z.ipd[ph][c];
            C.S.opd_prev[bk][ph][c] = Z.opd[ph][c];
        }
    if (C.u == 0) C.S.phase_hist = Z.phase;
}

__device__ void ps_param_scan(const SbrArgs& A, const PsConst& K, const uint32_t* fl, uint32_t nfr, PsState& S,
                              bool fresh, int u, uint32_t (*pbuf)[kPsFrameDw])
{
    if (u >= 20) return;
    uint32_t pre[kPsFrameDwPerLane];
    int grs[2], phase;
    float hp[2][8], ipd[2][2], opd[2][2];
    const ScanCtx C{A, K, fl, nfr, S, u, pbuf};
    const ScanArrays Z{pre, grs, hp, ipd, opd, phase};
    scan_init(C, Z, fresh);
    for (uint32_t j = 0; j < nfr; j++) scan_frame(C, Z, j);
    scan_finish(C, Z);
}

// ---------------------------------------------------------------------------------------------
// decorrelator recurrences
// ---------------------------------------------------------------------------------------------
// ring layout of one all-pass lane: [0..1] 2-slot delay, [2..4] link 0, [5..8] link 1, [9..13] link 2
template <int N>
__device__ __forceinline__ float2 allpass_step(float2 (&d)[14], float2 x, const float phi[2], const float q[3][2],
                                               const float g[3])
{
    constexpr int p0 = N % 2, pl[3] = {2 + N % 3, 5 + N % 4, 9 + N % 5};
    const float2 t0 = d[p0];
    d[p0] = x;
    float r0r = (t0.x * phi[0]) + (t0.y * phi[1]);
    float r0i = (t0.y * phi[0]) - (t0.x * phi[1]);
#pragma unroll
    for (int m = 0; m < 3; m++) {
        const float2 t = d[pl[m]];
        float tr = (t.x * q[m][0]) + (t.y * q[m][1]);
        float ti = (t.y * q[m][0]) - (t.x * q[m][1]);
        tr -= g[m] * r0r;
        ti -= g[m] * r0i;
        d[pl[m]] = make_float2(r0r + (g[m] * tr), r0i + (g[m] * ti));
        r0r = tr;
        r0i = ti;
    }
    return make_float2(r0r, r0i);
}

// after 32 slots the read positions sit at 32 mod L: rotate back to 0 (compile-time permutation)
template <int Off, int Len, int Shift, int Size>
__device__ __forceinline__ void rotate(float2 (&d)[Size])
{
    if constexpr (Shift != 0) {
        float2 t[Len];
#pragma unroll
        for (int k = 0; k < Len; k++) t[k] = d[Off + (k + Shift) % Len];
#pragma unroll
        for (int k = 0; k < Len; k++) d[Off + k] = t[k];
    }
}
__device__ __forceinline__ void rotate_allpass(float2 (&d)[14])
{
    rotate<0, 2, 32 % 2>(d);
    rotate<2, 3, 32 % 3>(d);
    rotate<5, 4, 32 % 4>(d);
    rotate<9, 5, 32 % 5>(d);
}

// ---------------------------------------------------------------------------------------------
// Pipelined decorrelator: the all-pass chain of a band (2-slot delay, then links 0, 1, 2:
// PSImpl.java:283-344) is a sequence of three independent recurrences -- link m's ring holds only
// link m's own past inputs and outputs -- so each link runs on its own wave, one frame behind the
// link before it, the links' outputs handed over through LDS.  Eight waves per run (two per SIMD:
// 256 VGPRs each), in lockstep steps separated by a workgroup barrier; at step k the roles do:
//   role 0 (Q0) QMF bands: 2-slot delay + link 0 of frame k
//   role 1 (Q1) QMF link 1 of frame k-1, and the plain delay lines of bands >= 23 (-> xps[f][1])
//   role 2 (Q2) QMF link 2 of frame k-2 (-> xps[f][1])
//   roles 3-5   the same three links for the hybrid groups 0..9 (-> xhr); role 4 also computes
//               G_TransientRatio of frame k-1 (the compare and the division, -> pg)
//   role 6      transient detector recurrences of frame k (peak, smooth, energy)
//   role 7      mixing-parameter scan of frame k (-> hb)
// Every value is computed by the same binary32 operations as the round-3 one-wave-per-recurrence form
// (measured 0.72 ms per C5 call; removed), bit-exact;
// only the waves that compute them differ.  The run's critical path drops from the whole chain
// of a QMF band (2-slot delay + 3 links per slot) to one link per slot.
// ---------------------------------------------------------------------------------------------
constexpr int kDecorWaves = 8;
constexpr int kApBands = 23;  // QMF bands 0..22 run the all-pass chain

// link m (0, 1, 2) of the all-pass chain at slot N: ring length 3, 4, 5; r = input (after the
// 2-slot delay's phi rotation for link 0, the previous link's output otherwise) -> output
// (packed: both components of each step in one v_pk_* instruction, the same binary32 operations --
// x + (-y) is x - y exactly)
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 pk(float2 v) { return pf2{v.x, v.y}; }
__device__ __forceinline__ float2 unpk(pf2 v) { return make_float2(v.x, v.y); }
// (t.x * c0) + (t.y * c1), (t.y * c0) - (t.x * c1)
__device__ __forceinline__ pf2 rot_conj(pf2 t, float c0, float c1)
{
    return (t * c0) + (pf2{t.y, t.x} * pf2{c1, -c1});  // (-c1 * x is -(c1 * x) exactly)
}
template <int M, int N, int Len>
__device__ __forceinline__ float2 ap_link(float2 (&d)[Len], float2 r, const float q[2], float g)
{
    const pf2 R = pk(r);
    pf2 T = rot_conj(pk(d[N % Len]), q[0], q[1]);
    T = T - (R * g);                    // tr -= g * r.x; ti -= g * r.y
    d[N % Len] = unpk(R + (T * g));     // r.x + (g * tr), r.y + (g * ti)
    return unpk(T);
}
// the 2-slot delay and its phi rotation (the input of link 0)
template <int N>
__device__ __forceinline__ float2 ap_delay2(float2 (&d)[2], float2 x, const float phi[2])
{
    const float2 t0 = d[N % 2];
    d[N % 2] = x;
    return unpk(rot_conj(pk(t0), phi[0], phi[1]));
}

// the lane index as an opaque value: each role recomputes it (two VALU) instead of the compiler
// keeping one copy alive across the whole kernel (which it spilled to scratch and reloaded per slot)
__device__ __forceinline__ int lane_id_fresh()
{
    int v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    return v;
}

// lanes of mask m take a, the others b, as one v_cndmask per float: a plain ?: on two array
// elements is turned into a load from a selected address, which puts the arrays in scratch
__device__ __forceinline__ float2 lane_sel(uint64_t m, float2 a, float2 b)
{
    float2 r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.x) : "v"(b.x), "v"(a.x), "s"(m));
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.y) : "v"(b.y), "v"(a.y), "s"(m));
    return r;
}

struct DecorLds {
    float2 q01[2][32][64], q12[2][32][64];  // QMF link outputs, [frame & 1][slot][band]
    float2 h01[2][32][10], h12[2][32][10];              // hybrid groups
    float2 tr[2][32][20];                               // (sm * gamma, nrg) per slot and parameter band
};

// The lockstep: nfr + 2 steps, a workgroup barrier after each; body(j, x, xn) runs for this wave's
// frame j = k - lag when there is one.  Readers (lag 0) find frame j's inputs in x and load frame
// j + 1's into xn; the two buffers alternate with the step's parity, as compile-time choices.
#ifdef JAAD_DECOR_STAMPS  // profiling build: per-wave busy (body) and total ticks of the steps
#define DECOR_T(v) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory")
#else
#define DECOR_T(v)
#endif
template <typename Body>
__device__ __forceinline__ void decor_steps(uint64_t& busy, uint32_t nfr, int lag, float2 (&xa)[32], float2 (&xb)[32],
                                            Body&& body)
{
    [[maybe_unused]] uint64_t t0 = 0, t1 = 0, acc = 0;
    for (uint32_t k = 0; k < nfr + 2; k += 2) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int64_t j = (int64_t)k + h - lag;
            DECOR_T(t0);
            if (j >= 0 && j < (int64_t)nfr) {
                if ((j & 1) == 0) body((uint32_t)j, xa, xb);
                else body((uint32_t)j, xb, xa);
            }
            DECOR_T(t1);
            acc += t1 - t0;
            __syncthreads();
        }
    }
    busy = acc;
}

__global__ __launch_bounds__(64 * kDecorWaves) __attribute__((amdgpu_waves_per_eu(1, 2))) void ps_decor_kernel(SbrArgs A)
{
    const uint32_t run = blockIdx.x;
    const uint32_t* fl = A.ps_list + A.runs[2 * run];
    const uint32_t nfr = A.runs[2 * run + 1];
    if (nfr == 0) return;  // uniform over the block
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __shared__ PsConst Ks;
    __shared__ uint32_t pbuf[2][kPsFrameDw];
    __shared__ DecorLds L;
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(A.psc);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&Ks);
        for (int i = threadIdx.x; i < (int)(sizeof(PsConst) / 4); i += 64 * kDecorWaves) dst[i] = src[i];
    }
    __syncthreads();
    PsState& S = A.pss[A.recs[fl[0]].slot];
    const PsConst& K = Ks;
    const bool fresh = S.init == 0;
    // the run's band limit: X_left is zero from band kb up and so is every all-pass ring there
    // (SbrRec::blim), so those lanes read a block of zeros and store nothing
    const int kb = (int)__builtin_amdgcn_readfirstlane(A.recs[fl[0]].blim);
    const float2 zero = make_float2(0.0f, 0.0f);
    float2 xa[32], xb[32];
    uint64_t busy = 0;
#ifdef JAAD_DECOR_STAMPS
    uint64_t t_start;
    DECOR_T(t_start);
#endif

    // role of this wave: 0..2 QMF links, 3..5 hybrid links, 6 transient detector, 7 parameter
    // scan.  Waves w and w + 4 share a SIMD when waves are placed round robin, so the roles are
    // paired for similar issue counts per step (profiles/round4_decor_stamps.txt):
    // (hybrid 0, hybrid 1), (QMF 0, hybrid 2), (QMF 1, scan), (QMF 2, transient).
#ifndef JAAD_DECOR_ROLES_PLAIN
    constexpr int kRole[kDecorWaves] = {3, 0, 1, 2, 4, 5, 7, 6};
#else
    constexpr int kRole[kDecorWaves] = {0, 1, 2, 3, 4, 5, 6, 7};
#endif
    const int role = kRole[wave];
    if (role <= 5) {
        const int u = lane_id_fresh();
        // ---- all-pass waves: QMF bands (waves 0-2, lane = band) / hybrid groups (3-5, lane = group)
        const bool hyb = role >= 3;
        const int link = hyb ? role - 3 : role;
        const int sb = hyb && u < 10 ? kBorder[u] : 0;
        // lanes that run the chain: every QMF lane (bands >= 23 too: v1 kept their rings running,
        // so the exported slot state is the same), the hybrid lanes with a group
        const bool act = hyb ? u < 10 : true;
        float phi[2], q[2], g;
        if (!hyb) {
            float slope = 1.0f;
            if (u > 3) {
                const int decay = 3 - u;
                slope = decay <= -20 ? 0.0f : 1.0f + kDecaySlope * (float)decay;
            }
            phi[0] = K.phi_qmf[u][0];
            phi[1] = K.phi_qmf[u][1];
            q[0] = K.q_qmf[u][link][0];
            q[1] = K.q_qmf[u][link][1];
            g = slope * K.filter_a[link];
        } else {
            phi[0] = K.phi_sub[sb][0];
            phi[1] = K.phi_sub[sb][1];
            q[0] = K.q_sub[sb][link][0];
            q[1] = K.q_sub[sb][link][1];
            g = 1.0f * K.filter_a[link];
        }
        const int hu = u < 10 ? u : 0;
        float2* const apst = hyb ? &S.aph[0][hu] : &S.ap[0][u];  // ring k at apst[k * stride]
        const int apstride = hyb ? 16 : 64;
        auto st_ap = [&](int k) -> float2& { return apst[k * apstride]; };
        if (link == 0) {
            // 2-slot delay + link 0
            float2 d2[2], r3[3];
            for (int k = 0; k < 2; k++) d2[k] = zero;
            for (int k = 0; k < 3; k++) r3[k] = zero;
            if (!fresh) {
                for (int k = 0; k < 2; k++) d2[k] = st_ap(k);
                for (int k = 0; k < 3; k++) r3[k] = st_ap(2 + k);
            }
            auto load = [&](float2 (&x)[32], uint32_t f) {
                if (!hyb) {
                    const float2* src = reinterpret_cast<const float2*>(u < kb ? A.xps + (size_t)f * 8192 : A.zero);
#pragma unroll
                    for (int n = 0; n < 32; n++) x[n] = src[n * 64 + u];
                } else {
                    const float2* src = reinterpret_cast<const float2*>(A.xhl + (size_t)f * 768);
#pragma unroll
                    for (int n = 0; n < 32; n++) x[n] = src[n * 12 + sb];
                }
            };
            load(xa, fl[0]);
            decor_steps(busy, nfr, 0, xa, xb, [&](uint32_t j, float2 (&x)[32], float2 (&xn)[32]) __attribute__((always_inline)) {
                const int u = lane_id_fresh();  // per step: a short live range
                const uint32_t pj = j & 1;
                if (j + 1 < nfr) load(xn, fl[j + 1]);  // lands during this frame
                if (!hyb) {
                    static_for<0, 32>([&](auto I) {
                        constexpr int n = decltype(I)::value;
                        L.q01[pj][n][u] = ap_link<0, n>(r3, ap_delay2<n>(d2, x[n], phi), q, g);
                    });
                } else if (act) {
                    static_for<0, 32>([&](auto I) {
                        constexpr int n = decltype(I)::value;
                        L.h01[pj][n][u] = ap_link<0, n>(r3, ap_delay2<n>(d2, x[n], phi), q, g);
                    });
                }
                rotate<0, 2, 32 % 2>(d2);
                rotate<0, 3, 32 % 3>(r3);
            });
            if (act) {
                for (int k = 0; k < 2; k++) st_ap(k) = d2[k];
                for (int k = 0; k < 3; k++) st_ap(2 + k) = r3[k];
            }
        } else if (link == 1) {
            // link 1 (+ the plain delay lines of QMF bands >= 23: 14 slots to band 34, 1 above, on
            // the frame's inputs, loaded at the step's start for those lanes and used after link 1)
            float2 r4[4], dl[14], d1 = zero;
            for (int k = 0; k < 4; k++) r4[k] = zero;
            for (int k = 0; k < 14; k++) dl[k] = zero;
            const bool dlane = !hyb && u >= kApBands && u < kb, is14 = u < 35;
            if (!fresh) {
                for (int k = 0; k < 4; k++) r4[k] = st_ap(5 + k);
                if (!hyb)
                    for (int k = 0; k < 14; k++) dl[k] = S.dl[k][u];
            }
            d1 = dl[0];
            // (only the plain delay lanes use the inputs: the others read the zero block, and their
            // unused delay slots in the state stay zero)
            auto load = [&](float2 (&x)[32], uint32_t f) {
                const float2* src = reinterpret_cast<const float2*>(dlane ? A.xps + (size_t)f * 8192 : A.zero);
#pragma unroll
                for (int n = 0; n < 32; n++) x[n] = src[n * 64 + u];
            };
            decor_steps(busy, nfr, 1, xa, xb, [&](uint32_t j, float2 (&)[32], float2 (&)[32]) __attribute__((always_inline)) {
                const int u = lane_id_fresh();  // per step: a short live range
                const uint32_t f = fl[j], pj = j & 1;
                if (!hyb) {
                    float2 x[32];
                    load(x, f);  // lands during link 1
                    static_for<0, 32>([&](auto I) {
                        constexpr int n = decltype(I)::value;
                        L.q12[pj][n][u] = ap_link<1, n>(r4, L.q01[pj][n][u], q, g);
                    });
                    rotate<0, 4, 32 % 4>(r4);
                    float2* dst = reinterpret_cast<float2*>(A.xps + (size_t)f * 8192) + 2048;
                    constexpr uint64_t kIs14 = (1ull << 35) - 1;  // lanes (bands) < 35: 14-slot delay
                    static_for<0, 32>([&](auto I) {
                        constexpr int n = decltype(I)::value;
                        const float2 rl = lane_sel(kIs14, dl[n % 14], d1);
                        dl[n % 14] = lane_sel(kIs14, x[n], dl[n % 14]);
                        d1 = x[n];
                        if (dlane) dst[n * 64 + u] = rl;
                    });
                    rotate<0, 14, 32 % 14>(dl);
                } else {
                    if (act) {
                        static_for<0, 32>([&](auto I) {
                            constexpr int n = decltype(I)::value;
                            L.h12[pj][n][u] = ap_link<1, n>(r4, L.h01[pj][n][u], q, g);
                        });
                        rotate<0, 4, 32 % 4>(r4);
                    }
                    if (u < 20) {  // G_TransientRatio (PSImpl.java:264-269), one frame behind role 6
                        float* dst = A.pg + (size_t)f * 640;
#pragma unroll
                        for (int n = 0; n < 32; n++) {
                            const float2 t = L.tr[pj][n][u];
                            dst[n * 20 + u] = t.x <= t.y ? 1.0f : __fdiv_rn(t.y, t.x);
                        }
                    }
                }
            });
            if (act)
                for (int k = 0; k < 4; k++) st_ap(5 + k) = r4[k];
            if (!hyb) {
                if (!is14) dl[0] = d1;
                for (int k = 0; k < 14; k++) S.dl[k][u] = dl[k];
            }
        } else {
            float2 r5[5];
            for (int k = 0; k < 5; k++) r5[k] = zero;
            if (!fresh)
                for (int k = 0; k < 5; k++) r5[k] = st_ap(9 + k);
            decor_steps(busy, nfr, 2, xa, xb, [&](uint32_t j, float2 (&)[32], float2 (&)[32]) {
                const int u = lane_id_fresh();  // per step: a short live range
                const uint32_t f = fl[j], pj = j & 1;
                if (!act) return;
                if (!hyb) {
                    float2* dst = reinterpret_cast<float2*>(A.xps + (size_t)f * 8192) + 2048;
                    static_for<0, 32>([&](auto I) {
                        constexpr int n = decltype(I)::value;
                        const float2 o = ap_link<2, n>(r5, L.q12[pj][n][u], q, g);
                        if (u >= 3 && u < kApBands) dst[n * 64 + u] = o;
                    });
                } else {
                    float2* dst = reinterpret_cast<float2*>(A.xhr + (size_t)f * 768);
                    static_for<0, 32>([&](auto I) {
                        constexpr int n = decltype(I)::value;
                        dst[n * 12 + sb] = ap_link<2, n>(r5, L.h12[pj][n][u], q, g);
                    });
                }
                rotate<0, 5, 32 % 5>(r5);
            });
            if (act)
                for (int k = 0; k < 5; k++) st_ap(9 + k) = r5[k];
        }
    } else if (role == 6) {
        const int u = lane_id_fresh();
        // ---- transient detector recurrences (lane = parameter band), PSImpl.java:238-270 ----
        const bool act = u < 20;
        const int pu = act ? u : 0;
        float peak = fresh ? 0.0f : S.peak[pu], smooth = fresh ? 0.0f : S.smooth[pu], pprev = fresh ? 0.0f : S.pprev[pu];
        auto load = [&](float2 (&x)[32], uint32_t f) {
            const float* src = A.pg + (size_t)f * 640;
#pragma unroll
            for (int n = 0; n < 32; n++) x[n].x = src[n * 20 + pu];
        };
        load(xa, fl[0]);
        decor_steps(busy, nfr, 0, xa, xb, [&](uint32_t j, float2 (&x)[32], float2 (&xn)[32]) __attribute__((always_inline)) {
            const int u = lane_id_fresh();  // per step: a short live range
            const uint32_t pj = j & 1;
            if (j + 1 < nfr) load(xn, fl[j + 1]);
#pragma unroll
            for (int n = 0; n < 32; n++) {
                const float Pn = x[n].x;
                const float gamma = 1.5f;
                peak = (peak * kAlphaDecay);
                if (peak < Pn) peak = Pn;
                float sm = smooth;
                sm += ((peak - Pn - smooth) * kAlphaSmooth);
                smooth = sm;
                float nrg = pprev;
                nrg += ((Pn - pprev) * kAlphaSmooth);
                pprev = nrg;
                if (act) L.tr[pj][n][u] = make_float2((sm * gamma), nrg);
            }
        });
        if (act) {
            S.peak[u] = peak;
            S.smooth[u] = smooth;
            S.pprev[u] = pprev;
        }
    } else {
        const int u = lane_id_fresh();
        // ---- mixing-parameter scan ----
        const bool act = u < 20;
        uint32_t sc_pre[kPsFrameDwPerLane];
        int sc_grs[2], sc_phase;
        float sc_hp[2][8], sc_ipd[2][2], sc_opd[2][2];
        const ScanCtx SC{A, K, fl, nfr, S, act ? u : 0, pbuf};
        const ScanArrays SZ{sc_pre, sc_grs, sc_hp, sc_ipd, sc_opd, sc_phase};
        if (act) scan_init(SC, SZ, fresh);
        decor_steps(busy, nfr, 0, xa, xb, [&](uint32_t j, float2 (&)[32], float2 (&)[32]) {
            if (act) scan_frame(SC, SZ, j);
        });
        if (act) scan_finish(SC, SZ);
    }
#ifdef JAAD_DECOR_STAMPS
    uint64_t t_end;
    DECOR_T(t_end);
    if (A.dbg && lane_id_fresh() == 0) {
        uint32_t* d = reinterpret_cast<uint32_t*>(A.dbg) + 4096 + (blockIdx.x * kDecorWaves + wave) * 4;
        d[0] = (uint32_t)busy;
        d[1] = (uint32_t)(t_end - t_start);
        d[2] = (uint32_t)kRole[wave];
        d[3] = nfr;
    }
#endif
}

// ---------------------------------------------------------------------------------------------
// mixing (PSImpl.ps_mix_phase :592-679) + hybrid synthesis (A/ps/Filterbank.java:70-86)
// ---------------------------------------------------------------------------------------------
// One wave per frame, in place on xps.  QMF bands 3..63 (lane = band), then the hybrid groups
// (lane = sub-band), each as four chunks of 8 slots with the next chunk's inputs in flight while
// this one mixes (two 8-slot buffers instead of all 32 slots in registers: 4 waves/SIMD); H walks
// the slots in order (PsHWalk: restart at each envelope border, one delta step per slot).
static_assert(offsetof(jaad_ps_frame, num_env) == 2 && offsetof(jaad_ps_frame, nr_ipdopd_par) == 3 &&
                  offsetof(jaad_ps_frame, border) == 4 && sizeof(jaad_ps_frame) % 4 == 0,
              "ps_mix_kernel reads the frame header as three dwords");

constexpr int kMixChunk = 8;
struct MixLds {
    float4 hb[5 * 22 * 16 / 4];                 // the frame's H start/delta rows (ps_decor_kernel's hb)
    float2 ml[kMixChunk][12], mr[kMixChunk][12];  // a chunk's mixed sub-bands (hybrid synthesis)
};
struct MixBuf {
    float2 x[kMixChunk], r[kMixChunk];
    float G[kMixChunk];
};

__global__ __launch_bounds__(256) void ps_mix_kernel(SbrArgs A)
{
    __shared__ MixLds lds_s[kPsWaves];
    const int wave = threadIdx.x >> 6, u = lane_id();
    const uint32_t f = blockIdx.x * kPsWaves + wave;
    if (f >= A.n_cf) return;
    if (!(A.recs[f].flags & kSbrPsOn)) return;  // X_left stays as the analysis wrote it
    MixLds& L = lds_s[wave];
    // frame parameters and H rows read once (the slot walks below would otherwise wait on a
    // global round trip at every envelope border): the first 12 bytes of jaad_ps_frame are
    // (iid_mode, icc_mode, num_env, nr_ipdopd_par, border[6], reserved[2])
    const uint32_t* ph = reinterpret_cast<const uint32_t*>(A.psf + f);
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(ph[0]);
    const uint64_t bw = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(ph[1]) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(ph[2]) << 32);
    const int nr = (int)(w0 >> 24), num_env = (int)((w0 >> 16) & 255u);
    {
        const float4* src = reinterpret_cast<const float4*>(A.hb + (size_t)f * (5 * 22 * 16));
        const int n4 = (num_env < 5 ? num_env : 5) * (22 * 16 / 4);
        for (int i = u; i < n4; i += 64) L.hb[i] = src[i];
        wave_sync();
    }
    const float* hbf = reinterpret_cast<const float*>(L.hb);
    const float* pg = A.pg + (size_t)f * 640;
    float2* xl = reinterpret_cast<float2*>(A.xps + (size_t)f * 8192);
    float2* xr = xl + 2048;
    // (chunks c = 0..3 unrolled, so the two buffers are compile-time choices)
    auto chunks = [&](auto&& load, auto&& mix) {
        MixBuf b0, b1;
        load(b0, 0);
        static_for<0, 4>([&](auto C) {
            constexpr int c = decltype(C)::value;
            MixBuf& cur = (c & 1) ? b1 : b0;
            MixBuf& nxt = (c & 1) ? b0 : b1;
            if constexpr (c < 3) load(nxt, kMixChunk * (c + 1));
            mix(cur, kMixChunk * c);
        });
    };
    // ---- QMF bands 3..K-1, lane = band (from the run's band limit up X_left and the all-pass
    // output are zero, and so are the mixed rows: nothing to load or store) ----
    if (u >= 3 && u < (int)A.recs[f].blim) {
        const int gr = ps_qmf_group(u), bk = gr - 2;
        const bool rot = bk < nr;
        PsHWalk W;
        W.begin();
        chunks(
            [&](MixBuf& b, int s0) {
#pragma unroll
                for (int i = 0; i < kMixChunk; i++) {
                    b.x[i] = xl[(s0 + i) * 64 + u];
                    b.r[i] = xr[(s0 + i) * 64 + u];
                    b.G[i] = pg[(s0 + i) * 20 + bk];
                }
            },
            [&](const MixBuf& b, int s0) {
#pragma unroll
                for (int i = 0; i < kMixChunk; i++) {
                    const int n = s0 + i;
                    W.step(hbf, bw, gr, rot, n);
                    float2 ol, orr;
                    ps_mix_slot(W.H, rot, b.x[i], b.r[i], b.G[i], ol, orr);
                    xl[n * 64 + u] = ol;
                    xr[n * 64 + u] = orr;
                }
            });
    }
    // ---- hybrid groups 0..9 (lane = group, sub-band kBorder[group]) and sub-bands 4, 5 (zero
    // after grouping, never decorrelated or mixed), a chunk at a time into LDS, then the hybrid
    // synthesis of the chunk's slots (lane = slot + 8 channel) into bands 0..2 ----
    const float2* hl = reinterpret_cast<const float2*>(A.xhl + (size_t)f * 768);
    const float2* hr = reinterpret_cast<const float2*>(A.xhr + (size_t)f * 768);
    const int t = u < 12 ? u : 0;
    const int sb = t < 10 ? kBorder[t] : t - 6, bk = t < 10 ? group_bk(t) : 0;
    const bool rot = bk < nr;
    PsHWalk W;
    W.begin();
    chunks(
        [&](MixBuf& b, int s0) {
#pragma unroll
            for (int i = 0; i < kMixChunk; i++) {
                b.x[i] = hl[(s0 + i) * 12 + sb];
                b.r[i] = hr[(s0 + i) * 12 + sb];
                b.G[i] = pg[(s0 + i) * 20 + bk];
            }
        },
        [&](const MixBuf& b, int s0) {
            if (u < 10) {
#pragma unroll
                for (int i = 0; i < kMixChunk; i++) {
                    W.step(hbf, bw, t, rot, s0 + i);
                    float2 ol, orr;
                    ps_mix_slot(W.H, rot, b.x[i], b.r[i], b.G[i], ol, orr);
                    L.ml[i][sb] = ol;
                    L.mr[i][sb] = orr;
                }
            } else if (u < 12) {
#pragma unroll
                for (int i = 0; i < kMixChunk; i++) {
                    L.ml[i][sb] = b.x[i];
                    L.mr[i][sb] = make_float2(0.0f, 0.0f);
                }
            }
            wave_sync();
            if (u < 2 * kMixChunk) {
                const int i = u & (kMixChunk - 1), n = s0 + i;
                const float2* m = u < kMixChunk ? L.ml[i] : L.mr[i];
                float2* x = u < kMixChunk ? xl : xr;
                constexpr int res[3] = {8, 2, 2};
#pragma unroll
                for (int band = 0, off = 0; band < 3; band++) {
                    float re = 0.0f, im = 0.0f;  // (0 + the first term: -0 becomes +0, as in the Java)
#pragma unroll
                    for (int k = 0; k < res[band]; k++) {
                        re += m[off + k].x;
                        im += m[off + k].y;
                    }
                    x[n * 64 + band] = make_float2(re, im);
                    off += res[band];
                }
            }
            wave_sync();  // (the next chunk rewrites ml / mr)
        });
}

// ---------------------------------------------------------------------------------------------
// per-run state after its last frame: filterbank history (the recurrences' and the mixing
// parameters' state is written by ps_decor_kernel)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ps_state_kernel(SbrArgs A)
{
    const uint32_t run = blockIdx.x;
    const uint32_t nfr = A.runs[2 * run + 1];
    if (nfr == 0) return;  // no PS frame in this call: the slot's PS state stays
    const uint32_t fl = A.ps_list[A.runs[2 * run] + nfr - 1];
    const int u = lane_id();
    PsState& S = A.pss[A.recs[fl].slot];
    if (u < 36) {
        const float2 h = hyb_history_after(A, fl, u / 12, u % 12);
        S.hyb[u / 12][u % 12][0] = h.x;
        S.hyb[u / 12][u % 12][1] = h.y;
    }
    wave_sync();
    if (u == 0) S.init = 1;
}

}  // namespace

hipError_t launch_ps(const SbrArgs& a, hipStream_t stream)
{
    if (!a.n_runs) return hipSuccess;
    const dim3 g((a.n_cf + kPsWaves - 1) / kPsWaves);
    hipLaunchKernelGGL(ps_analysis_kernel, g, dim3(64 * kPsWaves), 0, stream, a);
    hipLaunchKernelGGL(ps_decor_kernel, dim3(a.n_runs), dim3(64 * kDecorWaves), 0, stream, a);
    // (before the mixing: the state's hybrid history is X_left, which the mixing overwrites)
    hipLaunchKernelGGL(ps_state_kernel, dim3(a.n_runs), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(ps_mix_kernel, g, dim3(64 * kPsWaves), 0, stream, a);
    return hipGetLastError();
}

}  // namespace jaad
