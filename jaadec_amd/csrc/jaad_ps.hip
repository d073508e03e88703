// Parametric stereo (HE-AAC v2) for gfx950, A/ = aac/src/main/java/net/sourceforge/jaad/aac/ of the
// reference: PSImpl.process (A/ps/PSImpl.java:685-707) = hybrid analysis (A/ps/Filterbank.java:
// 18-68, T20), decorrelation (:202-400), mixing without IPD/OPD (:406-681), hybrid synthesis
// (A/ps/Filterbank.java:70-86).  Same binary32 evaluation order as the Java (-ffp-contract=off).
//
// PS state (all-pass / delay lines, transient detector, h_prev) is carried frame to frame, so one
// wave walks the frames of one run in order; lane = QMF band for the all-pass and mixing stages,
// lane = time slot for the hybrid filterbank and the energy sums, lane = parameter band for the
// transient detector.  The working set of a frame (X_left/right [38|32][64], hybrid [32][12],
// delay lines) lives in one wave's LDS (~57 KB); input is the mono SBR synthesis matrix in HBM
// (sbr_hf_kernel output, rows l < t_E[0] patched from the carry of frame f-1), output is
// (X_left', X_right) in xps for the two-channel synthesis.
#include <hip/hip_runtime.h>

#include "jaad_sbr.h"
#include "jaad_wave.h"

namespace jaad {
namespace {

constexpr int kBorder[23] = {6, 7, 0, 1, 2, 3, 9, 8, 10, 11, 3, 4, 5, 6, 7, 8, 9, 11, 14, 18, 23, 35, 64};
constexpr int kSerLen[3] = {3, 4, 5};   // PSTables.delay_length_d
constexpr int kSerOff[3] = {4, 10, 18}; // float offsets of the all-pass links in a delay column
constexpr float kAlphaDecay = 0.76592833836465f, kAlphaSmooth = 0.25f, kDecaySlope = 0.05f;
constexpr float kCoefSqrt2 = 1.4142135623731f;

__device__ __forceinline__ int group_bk(int gr) { return gr == 0 ? 1 : (gr == 1 ? 0 : gr - 2); }

struct PsLds {
    float2 xl[38][65];  // X_left (rows 32..37: bands 0..4 of Xsbr rows 34..39), padded rows
    float2 xr[32][65];
    float2 hl[32][12], hr[32][12];
    float g[32][20];        // P, then G_TransientRatio
    float h[22][5][8];      // per group/envelope: H start (4) + delta (4)
    float dq[28][64];       // QMF delay lines (PsState::dq)
    float dh[28][16];       // hybrid delay lines (PsState::dh)
    float2 hyb[3][12];      // hybrid filterbank history
};

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
// 3+4 and 2+5 merged (A/ps/Filterbank.java:55-67)
__device__ void filter8(const float2 b[13], const float* c, float2 out[8])
{
    float r1[4], i1[4], r2[4], i2[4], x[4];
    r1[0] = (c[6] * b[6].x);
    r1[1] = (c[5] * (b[5].x + b[7].x));
    r1[2] = -(c[0] * (b[0].x + b[12].x)) + (c[4] * (b[4].x + b[8].x));
    r1[3] = -(c[1] * (b[1].x + b[11].x)) + (c[3] * (b[3].x + b[9].x));
    i1[0] = (c[5] * (b[7].y - b[5].y));
    i1[1] = (c[0] * (b[12].y - b[0].y)) + (c[4] * (b[8].y - b[4].y));
    i1[2] = (c[1] * (b[11].y - b[1].y)) + (c[3] * (b[9].y - b[3].y));
    i1[3] = (c[2] * (b[10].y - b[2].y));
    float re[8], im[8];
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
__device__ void filter2(const float2 b[13], const float* c, float2 out[2])
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

// one all-pass step of PSImpl.ps_decorrelate (:286-336) on delay column d (stride ds floats)
__device__ __forceinline__ float2 allpass(float* d, int ds, float2 x, int td, const int ts[3], const float phi[2],
                                          const float q[3][2], const float gdf[3])
{
    const float t0r = d[(2 * td) * ds], t0i = d[(2 * td + 1) * ds];
    d[(2 * td) * ds] = x.x;
    d[(2 * td + 1) * ds] = x.y;
    float r0r = (t0r * phi[0]) + (t0i * phi[1]);
    float r0i = (t0i * phi[0]) - (t0r * phi[1]);
#pragma unroll
    for (int m = 0; m < 3; m++) {
        float* dl = d + (kSerOff[m] + 2 * ts[m]) * ds;
        const float a = dl[0], b = dl[ds];
        float tr = (a * q[m][0]) + (b * q[m][1]);
        float ti = (b * q[m][0]) - (a * q[m][1]);
        tr -= gdf[m] * r0r;
        ti -= gdf[m] * r0i;
        dl[0] = r0r + (gdf[m] * tr);
        dl[ds] = r0i + (gdf[m] * ti);
        r0r = tr;
        r0i = ti;
    }
    return make_float2(r0r, r0i);
}

__global__ __launch_bounds__(64) void ps_kernel(SbrArgs A)
{
    __shared__ PsLds L;
    const uint32_t run = blockIdx.x;
    if (run >= A.n_runs) return;
    const uint32_t f0 = A.runs[2 * run], nfr = A.runs[2 * run + 1];
    const int u = lane_id();
    const uint32_t slot = A.recs[f0].slot;
    PsState& S = A.pss[slot];
    const PsConst& K = *A.psc;
    const bool fresh = S.init == 0;

    for (int i = u; i < 28 * 64; i += 64) (&L.dq[0][0])[i] = fresh ? 0.0f : (&S.dq[0][0])[i];
    for (int i = u; i < 28 * 16; i += 64) (&L.dh[0][0])[i] = fresh ? 0.0f : (&S.dh[0][0])[i];
    if (u < 36) L.hyb[u / 12][u % 12] = fresh ? make_float2(0.0f, 0.0f) : make_float2(S.hyb[u / 12][u % 12][0], S.hyb[u / 12][u % 12][1]);
    float peak = 0.0f, smooth = 0.0f, pprev = 0.0f;
    if (!fresh && u < 20) {
        peak = S.peak[u];
        smooth = S.smooth[u];
        pprev = S.pprev[u];
    }
    float hp[4] = {1.0f, 0.0f, 0.0f, 0.0f};  // PSImpl constructor (:87-92)
    if (!fresh && u < 22)
        for (int k = 0; k < 4; k++) hp[k] = S.h_prev[u][k];
    int sdelay = fresh ? 0 : S.saved_delay, dD = fresh ? 0 : S.dD;
    int ser[3];
    for (int m = 0; m < 3; m++) ser[m] = fresh ? 0 : S.ser[m];

    // lane constants: QMF band u (decorrelation / mixing of groups 10..21)
    int grq = 10;
    for (int gr = 10; gr < 22; gr++)
        if (u >= kBorder[gr]) grq = gr;
    const int bkq = grq - 2;
    float phq[2] = {K.phi_qmf[u][0], K.phi_qmf[u][1]}, qq[3][2], gdq[3];
    {
        float slope = 1.0f;
        if (u > 3) {
            const int decay = 3 - u;
            slope = decay <= -20 ? 0.0f : 1.0f + kDecaySlope * (float)decay;
        }
        for (int m = 0; m < 3; m++) {
            qq[m][0] = K.q_qmf[u][m][0];
            qq[m][1] = K.q_qmf[u][m][1];
            gdq[m] = slope * K.filter_a[m];
        }
    }
    // lane constants: hybrid group u < 10 (sub-band kBorder[u])
    const int grh = u < 10 ? u : 0, sbh = kBorder[grh], bkh = group_bk(grh);
    float phh[2] = {K.phi_sub[sbh][0], K.phi_sub[sbh][1]}, qh[3][2], gdh[3];
    for (int m = 0; m < 3; m++) {
        qh[m][0] = K.q_sub[sbh][m][0];
        qh[m][1] = K.q_sub[sbh][m][1];
        gdh[m] = 1.0f * K.filter_a[m];
    }
    wave_sync();

    for (uint32_t j = 0; j < nfr; j++) {
        const uint32_t f = f0 + j;
        const SbrRec& R = A.recs[f];
        const jaad_ps_frame& P = A.psf[f];
        const int num_env = P.num_env;
        const int n0 = P.border[0], n1 = P.border[num_env];

        // ---- X_left (SBR1.processPS :102-120) ----
        {
            const int t0 = R.t_E[0], kprev = R.kx_prev + R.M_prev;
            const float2* xs = reinterpret_cast<const float2*>(A.xsyn + (size_t)f * 4096);
            const float2* xc = R.first ? reinterpret_cast<const float2*>(&A.state[(size_t)slot * 2].xcarry[0][0][0])
                                       : reinterpret_cast<const float2*>(A.xcarry + (size_t)(f - 1) * 768);
            const float2* xn = reinterpret_cast<const float2*>(A.xcarry + (size_t)f * 768);
            for (int l = 0; l < 32; l++) {
                float2 v;
                if (l < t0) v = u < kprev ? xc[l * 64 + u] : make_float2(0.0f, 0.0f);
                else v = xs[l * 64 + u];
                L.xl[l][u] = v;
                L.xr[l][u] = make_float2(0.0f, 0.0f);
            }
            for (int l = 32; l < 38; l++) L.xl[l][u] = u < 5 ? xn[(l - 32) * 64 + u] : make_float2(0.0f, 0.0f);
            for (int i = u; i < 32 * 12; i += 64) (&L.hr[0][0])[i] = make_float2(0.0f, 0.0f);
        }
        wave_sync();

        // ---- hybrid analysis: lane = time slot; band 0 (Filter8) | band 1, then band 2 (Filter2) ----
        for (int pass = 0; pass < 2; pass++) {
            const int band = pass == 0 ? (u < 32 ? 0 : 1) : 2;
            const int n = u & 31;
            if (pass == 1 && u >= 32) break;
            float2 b[13];
#pragma unroll
            for (int i = 0; i < 13; i++) {
                const int w = n + i;  // work[w]: history (w < 12) or X_left[w - 6]
                b[i] = w < 12 ? L.hyb[band][w] : L.xl[w - 6][band];
            }
            if (band == 0) {
                float2 o[8];
                filter8(b, K.p8, o);
#pragma unroll
                for (int k = 0; k < 8; k++) L.hl[n][k] = o[k];
            } else {
                float2 o[2];
                filter2(b, K.p2, o);
                L.hl[n][6 + 2 * band] = o[0];
                L.hl[n][7 + 2 * band] = o[1];
            }
        }
        wave_sync();
        if (u < 36) L.hyb[u / 12][u % 12] = L.xl[26 + u % 12][u / 12];  // buffer = work[32..43]

        // ---- P[n][bk] (:213-236), lane = time slot ----
        if (u < 32) {
            float Pb[20];
#pragma unroll
            for (int k = 0; k < 20; k++) Pb[k] = 0.0f;
            if (u >= n0 && u < n1) {
#pragma unroll
                for (int gr = 0; gr < 22; gr++) {
                    const int bk = group_bk(gr);
                    if (gr < 10) {
                        const float2 v = L.hl[u][kBorder[gr]];
                        Pb[bk] += (v.x * v.x) + (v.y * v.y);
                    } else {
#pragma unroll
                        for (int sb = kBorder[gr]; sb < kBorder[gr + 1]; sb++) {
                            const float2 v = L.xl[u][sb];
                            Pb[bk] += (v.x * v.x) + (v.y * v.y);
                        }
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 20; k++) L.g[u][k] = Pb[k];
        }
        wave_sync();

        // ---- transient detection (:238-270), lane = parameter band ----
        if (u < 20) {
            for (int n = n0; n < n1; n++) {
                const float Pn = L.g[n][u];
                const float gamma = 1.5f;
                peak = (peak * kAlphaDecay);
                if (peak < Pn) peak = Pn;
                float sm = smooth;
                sm += ((peak - Pn - smooth) * kAlphaSmooth);
                smooth = sm;
                float nrg = pprev;
                nrg += ((Pn - pprev) * kAlphaSmooth);
                pprev = nrg;
                L.g[n][u] = (sm * gamma) <= nrg ? 1.0f : __fdiv_rn(nrg, (sm * gamma));
            }
        }
        wave_sync();

        // ---- decorrelation (:272-400): QMF bands 3..63, then hybrid groups 0..9 ----
        if (u >= 3) {
            int td = sdelay, dd = dD, ts[3] = {ser[0], ser[1], ser[2]};
            float* col = &L.dq[0][u];
            for (int n = n0; n < n1; n++) {
                const float2 x = L.xl[n][u];
                float2 r0;
                if (u > 22) {
                    const int idx = u < 35 ? dd : 0;  // delay_D = 14 below SHORT_DELAY_BAND, else 1
                    r0 = make_float2(col[(2 * idx) * 64], col[(2 * idx + 1) * 64]);
                    col[(2 * idx) * 64] = x.x;
                    col[(2 * idx + 1) * 64] = x.y;
                } else {
                    r0 = allpass(col, 64, x, td, ts, phq, qq, gdq);
                }
                const float G = L.g[n][bkq];
                L.xr[n][u] = make_float2((G * r0.x), (G * r0.y));
                td = td + 1 >= 2 ? 0 : td + 1;
                dd = dd + 1 >= 14 ? 0 : dd + 1;
                for (int m = 0; m < 3; m++) ts[m] = ts[m] + 1 >= kSerLen[m] ? 0 : ts[m] + 1;
            }
        }
        if (u < 10) {
            int td = sdelay, ts[3] = {ser[0], ser[1], ser[2]};
            float* col = &L.dh[0][u];
            for (int n = n0; n < n1; n++) {
                const float2 r0 = allpass(col, 16, L.hl[n][sbh], td, ts, phh, qh, gdh);
                const float G = L.g[n][bkh];
                L.hr[n][sbh] = make_float2((G * r0.x), (G * r0.y));
                td = td + 1 >= 2 ? 0 : td + 1;
                for (int m = 0; m < 3; m++) ts[m] = ts[m] + 1 >= kSerLen[m] ? 0 : ts[m] + 1;
            }
        }
        {
            const int cnt = n1 > n0 ? n1 - n0 : 0;
            sdelay = (sdelay + cnt) % 2;
            dD = (dD + cnt) % 14;
            for (int m = 0; m < 3; m++) ser[m] = (ser[m] + cnt) % kSerLen[m];
        }

        // ---- mixing matrices per group / envelope (:419-520), lane = group ----
        if (u < 22) {
            const int bk = group_bk(u);
            const int fine = P.iid_mode >= 3;
            const int steps = fine ? 15 : 7;
            const float* sf_iid = K.sf_iid[fine];
            for (int env = 0; env < num_env; env++) {
                int iid = P.iid[env][bk];
                const int sign = iid < 0 ? -1 : 1;
                iid = iid < 0 ? -iid : iid;
                const int icc = P.icc[env][bk];
                float h[4];
                if (P.icc_mode < 3) {
                    const float c1 = sf_iid[steps + iid], c2 = sf_iid[steps - iid];
                    const float cosa = K.cos_alphas[icc], sina = K.sin_alphas[icc];
                    const float cosb = K.cos_betas[fine][iid][icc];
                    const float sinb = K.sin_betas[fine][iid][icc] * (float)sign;
                    const float ab1 = (cosb * cosa), ab2 = (sinb * sina), ab3 = (sinb * cosa), ab4 = (cosb * sina);
                    h[0] = (c2 * (ab1 - ab2));
                    h[1] = (c1 * (ab1 + ab2));
                    h[2] = (c2 * (ab3 + ab4));
                    h[3] = (c1 * (ab3 - ab4));
                } else {
                    const float cosa = K.sincos_b[fine][steps + iid][icc];
                    const float sina = K.sincos_b[fine][2 * steps - (steps + iid)][icc];
                    const float cosg = K.cos_gammas[fine][iid][icc], sing = K.sin_gammas[fine][iid][icc];
                    h[0] = (kCoefSqrt2 * (cosa * cosg));
                    h[1] = (kCoefSqrt2 * (sina * cosg));
                    h[2] = (kCoefSqrt2 * (-cosa * sing));
                    h[3] = (kCoefSqrt2 * (sina * sing));
                }
                const float Lf = (float)(P.border[env + 1] - P.border[env]);
                for (int k = 0; k < 4; k++) {
                    L.h[u][env][k] = hp[k];
                    L.h[u][env][4 + k] = __fdiv_rn(h[k] - hp[k], Lf);
                    hp[k] = h[k];
                }
            }
        }
        wave_sync();

        // ---- mixing (:600-660): QMF bands 3..63, then hybrid groups 0..9 ----
        auto mix = [&](int gr, float2* lrow, float2* rrow, int stride) {
            for (int env = 0; env < num_env; env++) {
                const float* hv = L.h[gr][env];
                float H11 = hv[0], H12 = hv[1], H21 = hv[2], H22 = hv[3];
                const float d11 = hv[4], d12 = hv[5], d21 = hv[6], d22 = hv[7];
                for (int n = P.border[env]; n < P.border[env + 1]; n++) {
                    H11 += d11;
                    H12 += d12;
                    H21 += d21;
                    H22 += d22;
                    const float2 l = lrow[n * stride], r = rrow[n * stride];
                    lrow[n * stride] = make_float2((H11 * l.x) + (H21 * r.x), (H11 * l.y) + (H21 * r.y));
                    rrow[n * stride] = make_float2((H12 * l.x) + (H22 * r.x), (H12 * l.y) + (H22 * r.y));
                }
            }
        };
        if (u >= 3) mix(grq, &L.xl[0][u], &L.xr[0][u], 65);
        if (u < 10) mix(grh, &L.hl[0][sbh], &L.hr[0][sbh], 12);
        wave_sync();

        // ---- hybrid synthesis (A/ps/Filterbank.java:70-86): lanes 0..31 left, 32..63 right ----
        {
            const int n = u & 31;
            const float2* hrow = u < 32 ? L.hl[n] : L.hr[n];
            float2* xrow = u < 32 ? L.xl[n] : L.xr[n];
            const int res[3] = {8, 2, 2};
            for (int band = 0, off = 0; band < 3; band++) {
                float re = 0.0f, im = 0.0f;
                for (int k = 0; k < res[band]; k++) {
                    re += hrow[off + k].x;
                    im += hrow[off + k].y;
                }
                xrow[band] = make_float2(re, im);
                off += res[band];
            }
        }
        wave_sync();

        // ---- (X_left', X_right) -> xps for the two-channel synthesis ----
        {
            float2* ol = reinterpret_cast<float2*>(A.xps + (size_t)f * 8192);
            float2* orr = ol + 2048;
            for (int l = 0; l < 32; l++) {
                ol[l * 64 + u] = L.xl[l][u];
                orr[l * 64 + u] = L.xr[l][u];
            }
        }
        wave_sync();
    }

    // ---- state after the run's last frame ----
    for (int i = u; i < 28 * 64; i += 64) (&S.dq[0][0])[i] = (&L.dq[0][0])[i];
    for (int i = u; i < 28 * 16; i += 64) (&S.dh[0][0])[i] = (&L.dh[0][0])[i];
    if (u < 36) {
        S.hyb[u / 12][u % 12][0] = L.hyb[u / 12][u % 12].x;
        S.hyb[u / 12][u % 12][1] = L.hyb[u / 12][u % 12].y;
    }
    if (u < 20) {
        S.peak[u] = peak;
        S.smooth[u] = smooth;
        S.pprev[u] = pprev;
    }
    if (u < 22)
        for (int k = 0; k < 4; k++) S.h_prev[u][k] = hp[k];
    if (u == 0) {
        S.saved_delay = sdelay;
        S.dD = dD;
        for (int m = 0; m < 3; m++) S.ser[m] = ser[m];
        S.init = 1;
    }
}

}  // namespace

hipError_t launch_ps(const SbrArgs& a, hipStream_t stream)
{
    if (a.n_runs) hipLaunchKernelGGL(ps_kernel, dim3(a.n_runs), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace jaad
