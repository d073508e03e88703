/*
 * jaad_oracle_ps.c -- TEST INFRASTRUCTURE ONLY (see jaad_oracle.h for the parity status).
 *
 * Plain-C restatement of the reference's parametric stereo (HE-AAC v2) path, A/ = aac/src/main/
 * java/net/sourceforge/jaad/aac/: PSImpl (decorrelation, mixing), ps/Filterbank + Filter8 +
 * Filter2 (hybrid analysis/synthesis, T20 -- FBType.max always yields T20, A/ps/FBType.java:17-19).
 * Inputs are the values ps_data_decode leaves behind (jaad_ps_frame), including the IPD/OPD
 * indices of the PS extension and Extension.nr_par() (A/ps/Extension.java:81-86).
 */
#include "jaad_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../jaadec_amd/csrc/tables/jaad_ps_tables.inc"

#if defined(__FP_FAST_FMAF) || defined(__FAST_MATH__)
#error "the oracle must be compiled without fast-math / FMA contraction"
#endif

enum { NO_ALLPASS_LINKS = 3, NR_ALLPASS_BANDS = 22, SHORT_DELAY_BAND = 35, NEGATE_IPD_MASK = 0x1000 };
static const float ALPHA_DECAY = 0.76592833836465f, ALPHA_SMOOTH = 0.25f, DECAY_SLOPE = 0.05f;
static const float COEF_SQRT2 = 1.4142135623731f;

/* FBType.T20 (A/ps/FBType.java:29-32) */
enum { T20_NUM_GROUPS = 22, T20_NUM_HYBRID_GROUPS = 10, T20_NR_PAR_BANDS = 20, T20_DECAY_CUTOFF = 3 };
static const int MAP_GROUP2BK20[22] = {NEGATE_IPD_MASK | 1, NEGATE_IPD_MASK | 0, 0, 1, 2, 3, 4, 5, 6, 7, 8,
                                       9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19};
static int t20_bk(int gr) { return MAP_GROUP2BK20[gr] & ~NEGATE_IPD_MASK; }
static int t20_maxsb(int gr) { return gr < T20_NUM_HYBRID_GROUPS ? JAAD_PS_GROUP_BORDER20[gr] + 1 : JAAD_PS_GROUP_BORDER20[gr + 1]; }

struct orc_ps {
    int len;
    float hyb_buffer[3][12][2]; /* Filterbank.buffer[band][0..11] (A/ps/Filterbank.java:8,36-39) */
    int saved_delay, delay_buf_index_ser[NO_ALLPASS_LINKS], num_sample_delay_ser[NO_ALLPASS_LINKS];
    int delay_D[64], delay_buf_index_delay[64];
    float delay_Qmf[14][64][2], delay_SubQmf[2][32][2];
    float delay_Qmf_ser[NO_ALLPASS_LINKS][5][64][2], delay_SubQmf_ser[NO_ALLPASS_LINKS][5][32][2];
    float P_PeakDecayNrg[34], P_prev[34], P_SmoothPeakDecayDiffNrg_prev[34];
    float h11_prev[50][2], h12_prev[50][2], h21_prev[50][2], h22_prev[50][2];
    float ipd_prev[20][2][2], opd_prev[20][2][2]; /* PDData.prev (A/ps/PDData.java:13) */
    int phase_hist;
    /* parameters of the current frame */
    int num_env, border_position[6], iid_mode, icc_mode, nr_ipdopd_par;
    int iid_index[5][34], icc_index[5][34], ipd_index[5][17];
};

size_t orc_ps_bytes(void) { return sizeof(orc_ps); }

void orc_ps_init(orc_ps* ps) /* PSImpl constructor (A/ps/PSImpl.java:63-95) */
{
    memset(ps, 0, sizeof *ps);
    ps->len = 32;
    for (int i = 0; i < NO_ALLPASS_LINKS; i++) ps->num_sample_delay_ser[i] = JAAD_PS_DELAY_LENGTH_D[i];
    for (int i = 0; i < 64; i++) ps->delay_D[i] = i < SHORT_DELAY_BAND ? 14 : 1;
    for (int i = 0; i < 50; i++) {
        ps->h11_prev[i][0] = 1; /* h12_prev[i][1] = 1 twice; h21/h22 stay 0 (A/ps/PSImpl.java:87-92) */
        ps->h12_prev[i][1] = 1;
    }
}

void orc_ps_set_frame(orc_ps* ps, const jaad_ps_frame* f)
{
    ps->num_env = f->num_env;
    ps->iid_mode = f->iid_mode;
    ps->icc_mode = f->icc_mode;
    ps->nr_ipdopd_par = f->nr_ipdopd_par;
    for (int e = 0; e <= f->num_env && e < 6; e++) ps->border_position[e] = f->border[e];
    for (int e = 0; e < 5; e++)
        for (int b = 0; b < 34; b++) {
            ps->iid_index[e][b] = f->iid[e][b];
            ps->icc_index[e][b] = f->icc[e][b];
        }
    for (int e = 0; e < 5; e++)
        for (int b = 0; b < 17; b++) ps->ipd_index[e][b] = f->ipd[e][b];
}

/* Filter8.DCT3_4_unscaled (A/ps/Filter8.java:122-137), y may alias x */
static void dct3_4_unscaled(float* y, const float* x)
{
    float f0 = (x[2] * 0.7071067811865476f);
    float f1 = x[0] - f0;
    float f2 = x[0] + f0;
    float f3 = x[1] + x[3];
    float f4 = (x[1] * 1.3065629648763766f);
    float f5 = (f3 * (-0.9238795325112866f));
    float f6 = (x[3] * (-0.5411961001461967f));
    float f7 = f4 + f5;
    float f8 = f6 - f5;
    y[3] = f2 - f8;
    y[0] = f2 + f8;
    y[2] = f1 - f7;
    y[1] = f1 + f7;
}

/* Filter8.filter, p8_13_20 (A/ps/Filter8.java:54-119) */
static void filter8(int frame_len, float (*buffer)[2], float (*result)[12][2])
{
    const float* filter = JAAD_PS_P8_13_20;
    float input_re1[4], input_re2[4], input_im1[4], input_im2[4], x[4];
    for (int i = 0; i < frame_len; i++) {
        float(*b)[2] = buffer + i;
        input_re1[0] = (filter[6] * b[6][0]);
        input_re1[1] = (filter[5] * (b[5][0] + b[7][0]));
        input_re1[2] = -(filter[0] * (b[0][0] + b[12][0])) + (filter[4] * (b[4][0] + b[8][0]));
        input_re1[3] = -(filter[1] * (b[1][0] + b[11][0])) + (filter[3] * (b[3][0] + b[9][0]));
        input_im1[0] = (filter[5] * (b[7][1] - b[5][1]));
        input_im1[1] = (filter[0] * (b[12][1] - b[0][1])) + (filter[4] * (b[8][1] - b[4][1]));
        input_im1[2] = (filter[1] * (b[11][1] - b[1][1])) + (filter[3] * (b[9][1] - b[3][1]));
        input_im1[3] = (filter[2] * (b[10][1] - b[2][1]));
        for (int n = 0; n < 4; n++) x[n] = input_re1[n] - input_im1[3 - n];
        dct3_4_unscaled(x, x);
        result[i][7][0] = x[0];
        result[i][5][0] = x[2];
        result[i][3][0] = x[3];
        result[i][1][0] = x[1];
        for (int n = 0; n < 4; n++) x[n] = input_re1[n] + input_im1[3 - n];
        dct3_4_unscaled(x, x);
        result[i][6][0] = x[1];
        result[i][4][0] = x[3];
        result[i][2][0] = x[2];
        result[i][0][0] = x[0];
        input_im2[0] = (filter[6] * b[6][1]);
        input_im2[1] = (filter[5] * (b[5][1] + b[7][1]));
        input_im2[2] = -(filter[0] * (b[0][1] + b[12][1])) + (filter[4] * (b[4][1] + b[8][1]));
        input_im2[3] = -(filter[1] * (b[1][1] + b[11][1])) + (filter[3] * (b[3][1] + b[9][1]));
        input_re2[0] = (filter[5] * (b[7][0] - b[5][0]));
        input_re2[1] = (filter[0] * (b[12][0] - b[0][0])) + (filter[4] * (b[8][0] - b[4][0]));
        input_re2[2] = (filter[1] * (b[11][0] - b[1][0])) + (filter[3] * (b[9][0] - b[3][0]));
        input_re2[3] = (filter[2] * (b[10][0] - b[2][0]));
        for (int n = 0; n < 4; n++) x[n] = input_im2[n] + input_re2[3 - n];
        dct3_4_unscaled(x, x);
        result[i][7][1] = x[0];
        result[i][5][1] = x[2];
        result[i][3][1] = x[3];
        result[i][1][1] = x[1];
        for (int n = 0; n < 4; n++) x[n] = input_im2[n] - input_re2[3 - n];
        dct3_4_unscaled(x, x);
        result[i][6][1] = x[1];
        result[i][4][1] = x[3];
        result[i][2][1] = x[2];
        result[i][0][1] = x[0];
    }
}

/* Filter2.filter, p2_13_20 (A/ps/Filter2.java:40-67) */
static void filter2(int frame_len, float (*buffer)[2], float (*result)[12][2])
{
    const float* filter = JAAD_PS_P2_13_20;
    for (int i = 0; i < frame_len; i++) {
        float(*b)[2] = buffer + i;
        float r0 = (filter[0] * (b[0][0] + b[12][0]));
        float r1 = (filter[1] * (b[1][0] + b[11][0]));
        float r2 = (filter[2] * (b[2][0] + b[10][0]));
        float r3 = (filter[3] * (b[3][0] + b[9][0]));
        float r4 = (filter[4] * (b[4][0] + b[8][0]));
        float r5 = (filter[5] * (b[5][0] + b[7][0]));
        float r6 = (filter[6] * b[6][0]);
        float i0 = (filter[0] * (b[0][1] + b[12][1]));
        float i1 = (filter[1] * (b[1][1] + b[11][1]));
        float i2 = (filter[2] * (b[2][1] + b[10][1]));
        float i3 = (filter[3] * (b[3][1] + b[9][1]));
        float i4 = (filter[4] * (b[4][1] + b[8][1]));
        float i5 = (filter[5] * (b[5][1] + b[7][1]));
        float i6 = (filter[6] * b[6][1]);
        result[i][0][0] = r0 + r1 + r2 + r3 + r4 + r5 + r6;
        result[i][0][1] = i0 + i1 + i2 + i3 + i4 + i5 + i6;
        result[i][1][0] = r0 - r1 + r2 - r3 + r4 - r5 + r6;
        result[i][1][1] = i0 - i1 + i2 - i3 + i4 - i5 + i6;
    }
}

/* Filterbank.hybrid_analysis (A/ps/Filterbank.java:18-68), T20 */
static void hybrid_analysis(orc_ps* ps, float (*X)[64][2], float (*X_hybrid)[32][2])
{
    float work[32 + 12][2];
    float temp[32][12][2];
    static const int res[3] = {8, 2, 2};
    for (int band = 0, offset = 0; band < T20_DECAY_CUTOFF; band++) {
        for (int i = 0; i < 12; i++) {
            work[i][0] = ps->hyb_buffer[band][i][0];
            work[i][1] = ps->hyb_buffer[band][i][1];
        }
        for (int n = 0; n < ps->len; n++) {
            work[12 + n][0] = X[n + 6][band][0];
            work[12 + n][1] = X[n + 6][band][1];
        }
        for (int i = 0; i < 12; i++) {
            ps->hyb_buffer[band][i][0] = work[ps->len + i][0];
            ps->hyb_buffer[band][i][1] = work[ps->len + i][1];
        }
        if (band == 0) filter8(ps->len, work, temp);
        else filter2(ps->len, work, temp);
        for (int n = 0; n < ps->len; n++)
            for (int k = 0; k < res[band]; k++) {
                X_hybrid[n][offset + k][0] = temp[n][k][0];
                X_hybrid[n][offset + k][1] = temp[n][k][1];
            }
        offset += res[band];
    }
    for (int n = 0; n < ps->len; n++) { /* group hybrid channels (:55-67) */
        X_hybrid[n][3][0] += X_hybrid[n][4][0];
        X_hybrid[n][3][1] += X_hybrid[n][4][1];
        X_hybrid[n][4][0] = 0;
        X_hybrid[n][4][1] = 0;
        X_hybrid[n][2][0] += X_hybrid[n][5][0];
        X_hybrid[n][2][1] += X_hybrid[n][5][1];
        X_hybrid[n][5][0] = 0;
        X_hybrid[n][5][1] = 0;
    }
}

/* Filterbank.hybrid_synthesis (A/ps/Filterbank.java:70-86), T20 */
static void hybrid_synthesis(const orc_ps* ps, float (*X)[64][2], float (*X_hybrid)[32][2])
{
    static const int res[3] = {8, 2, 2};
    for (int band = 0, offset = 0; band < T20_DECAY_CUTOFF; band++) {
        for (int n = 0; n < ps->len; n++) {
            X[n][band][0] = 0;
            X[n][band][1] = 0;
            for (int k = 0; k < res[band]; k++) {
                X[n][band][0] += X_hybrid[n][offset + k][0];
                X[n][band][1] += X_hybrid[n][offset + k][1];
            }
        }
        offset += res[band];
    }
}

/* PSImpl.ps_decorrelate (A/ps/PSImpl.java:202-400) */
static void ps_decorrelate(orc_ps* ps, float (*X_left)[64][2], float (*X_right)[64][2], float (*X_hybrid_left)[32][2],
                           float (*X_hybrid_right)[32][2])
{
    float P[32][34], G_TransientRatio[32][34];
    memset(P, 0, sizeof P);
    memset(G_TransientRatio, 0, sizeof G_TransientRatio);
    const int n0 = ps->border_position[0], n1 = ps->border_position[ps->num_env];
    for (int gr = 0; gr < T20_NUM_GROUPS; gr++) {
        const int bk = t20_bk(gr), maxsb = t20_maxsb(gr);
        for (int n = n0; n < n1; n++)
            for (int sb = JAAD_PS_GROUP_BORDER20[gr]; sb < maxsb; sb++) {
                const float* xl = gr < T20_NUM_HYBRID_GROUPS ? X_hybrid_left[n][sb] : X_left[n][sb];
                float re = xl[0], im = xl[1];
                P[n][bk] += (re * re) + (im * im);
            }
    }
    for (int bk = 0; bk < T20_NR_PAR_BANDS; bk++) {
        for (int n = n0; n < n1; n++) {
            float gamma = 1.5f;
            ps->P_PeakDecayNrg[bk] = (ps->P_PeakDecayNrg[bk] * ALPHA_DECAY);
            if (ps->P_PeakDecayNrg[bk] < P[n][bk]) ps->P_PeakDecayNrg[bk] = P[n][bk];
            float sm = ps->P_SmoothPeakDecayDiffNrg_prev[bk];
            sm += ((ps->P_PeakDecayNrg[bk] - P[n][bk] - ps->P_SmoothPeakDecayDiffNrg_prev[bk]) * ALPHA_SMOOTH);
            ps->P_SmoothPeakDecayDiffNrg_prev[bk] = sm;
            float nrg = ps->P_prev[bk];
            nrg += ((P[n][bk] - ps->P_prev[bk]) * ALPHA_SMOOTH);
            ps->P_prev[bk] = nrg;
            if ((sm * gamma) <= nrg) G_TransientRatio[n][bk] = 1.0f;
            else G_TransientRatio[n][bk] = (nrg / (sm * gamma));
        }
    }
    int temp_delay = 0, temp_delay_ser[NO_ALLPASS_LINKS];
    float g_DecaySlope_filt[NO_ALLPASS_LINKS];
    for (int gr = 0; gr < T20_NUM_GROUPS; gr++) {
        const int maxsb = t20_maxsb(gr);
        const int hyb = gr < T20_NUM_HYBRID_GROUPS;
        for (int sb = JAAD_PS_GROUP_BORDER20[gr]; sb < maxsb; sb++) {
            float g_DecaySlope;
            if (hyb || sb <= T20_DECAY_CUTOFF) g_DecaySlope = 1.0f;
            else {
                int decay = T20_DECAY_CUTOFF - sb;
                if (decay <= -20) g_DecaySlope = 0;
                else g_DecaySlope = 1.0f + DECAY_SLOPE * (float)decay;
            }
            for (int m = 0; m < NO_ALLPASS_LINKS; m++) g_DecaySlope_filt[m] = g_DecaySlope * JAAD_PS_FILTER_A[m];
            temp_delay = ps->saved_delay;
            for (int n = 0; n < NO_ALLPASS_LINKS; n++) temp_delay_ser[n] = ps->delay_buf_index_ser[n];
            for (int n = n0; n < n1; n++) {
                float r0Re, r0Im;
                float re = hyb ? X_hybrid_left[n][sb][0] : X_left[n][sb][0];
                float im = hyb ? X_hybrid_left[n][sb][1] : X_left[n][sb][1];
                if (sb > NR_ALLPASS_BANDS && !hyb) {
                    float* delay = ps->delay_Qmf[ps->delay_buf_index_delay[sb]][sb];
                    r0Re = delay[0];
                    r0Im = delay[1];
                    delay[0] = re;
                    delay[1] = im;
                } else {
                    float* delayQmf = hyb ? ps->delay_SubQmf[temp_delay][sb] : ps->delay_Qmf[temp_delay][sb];
                    const float* Phi_Fract = hyb ? JAAD_PS_PHI_FRACT_SUBQMF20[sb] : JAAD_PS_PHI_FRACT_QMF[sb];
                    float tmp0Re = delayQmf[0], tmp0Im = delayQmf[1];
                    delayQmf[0] = re;
                    delayQmf[1] = im;
                    r0Re = (tmp0Re * Phi_Fract[0]) + (tmp0Im * Phi_Fract[1]);
                    r0Im = (tmp0Im * Phi_Fract[0]) - (tmp0Re * Phi_Fract[1]);
                    for (int m = 0; m < NO_ALLPASS_LINKS; m++) {
                        const float* q = hyb ? &JAAD_PS_Q_FRACT_ALLPASS_SUBQMF20[(sb * 3 + m) * 2]
                                             : &JAAD_PS_Q_FRACT_ALLPASS_QMF[(sb * 3 + m) * 2];
                        float* delay = hyb ? ps->delay_SubQmf_ser[m][temp_delay_ser[m]][sb]
                                           : ps->delay_Qmf_ser[m][temp_delay_ser[m]][sb];
                        tmp0Re = delay[0];
                        tmp0Im = delay[1];
                        float tmpRe = (tmp0Re * q[0]) + (tmp0Im * q[1]);
                        float tmpIm = (tmp0Im * q[0]) - (tmp0Re * q[1]);
                        tmpRe -= g_DecaySlope_filt[m] * r0Re;
                        tmpIm -= g_DecaySlope_filt[m] * r0Im;
                        delay[0] = r0Re + (g_DecaySlope_filt[m] * tmpRe);
                        delay[1] = r0Im + (g_DecaySlope_filt[m] * tmpIm);
                        r0Re = tmpRe;
                        r0Im = tmpIm;
                    }
                }
                const int bk = t20_bk(gr);
                float* xr = hyb ? X_hybrid_right[n][sb] : X_right[n][sb];
                xr[0] = (G_TransientRatio[n][bk] * r0Re);
                xr[1] = (G_TransientRatio[n][bk] * r0Im);
                if (++temp_delay >= 2) temp_delay = 0;
                if (sb > NR_ALLPASS_BANDS && !hyb)
                    if (++ps->delay_buf_index_delay[sb] >= ps->delay_D[sb]) ps->delay_buf_index_delay[sb] = 0;
                for (int m = 0; m < NO_ALLPASS_LINKS; m++)
                    if (++temp_delay_ser[m] >= ps->num_sample_delay_ser[m]) temp_delay_ser[m] = 0;
            }
        }
    }
    ps->saved_delay = temp_delay;
    memcpy(ps->delay_buf_index_ser, temp_delay_ser, sizeof temp_delay_ser);
}

/* PSImpl.magnitude_c (A/ps/PSImpl.java:402-404) */
static float magnitude_c(const float* c) { return (float)sqrt((double)((c[0] * c[0]) + (c[1] * c[1]))); }

/* PSImpl.ps_mix_phase (A/ps/PSImpl.java:406-681) */
static void ps_mix_phase(orc_ps* ps, float (*X_left)[64][2], float (*X_right)[64][2], float (*X_hybrid_left)[32][2],
                         float (*X_hybrid_right)[32][2])
{
    const int fine = ps->iid_mode >= 3;
    const int num_steps = fine ? 15 : 7;
    const float* sf_iid = fine ? JAAD_PS_SF_IID_FINE : JAAD_PS_SF_IID_NORMAL;
    const float* cos_betas = fine ? JAAD_PS_COS_BETAS_FINE : JAAD_PS_COS_BETAS_NORMAL;
    const float* sin_betas = fine ? JAAD_PS_SIN_BETAS_FINE : JAAD_PS_SIN_BETAS_NORMAL;
    /* IIDMode passes (sin_gammas_*, cos_gammas_*) into IIDTables(cos_gammas, sin_gammas): swapped
       (A/ps/IIDMode.java:16-28 vs A/ps/IIDTables.java:17-21) */
    const float* cos_gammas = fine ? JAAD_PS_SIN_GAMMAS_FINE : JAAD_PS_SIN_GAMMAS_NORMAL;
    const float* sin_gammas = fine ? JAAD_PS_COS_GAMMAS_FINE : JAAD_PS_COS_GAMMAS_NORMAL;
    const float* sincos_alphas_b = fine ? JAAD_PS_SINCOS_ALPHAS_B_FINE : JAAD_PS_SINCOS_ALPHAS_B_NORMAL;
    float h11[2] = {0, 0}, h12[2] = {0, 0}, h21[2] = {0, 0}, h22[2] = {0, 0};
    float H11[2] = {0, 0}, H12[2] = {0, 0}, H21[2] = {0, 0}, H22[2] = {0, 0};
    float deltaH11[2] = {0, 0}, deltaH12[2] = {0, 0}, deltaH21[2] = {0, 0}, deltaH22[2] = {0, 0};
    float tempLeft[2], tempRight[2], phaseLeft[2], phaseRight[2];
    const int nr_ipdopd_par = ps->nr_ipdopd_par;
    for (int gr = 0; gr < T20_NUM_GROUPS; gr++) {
        const int bk = t20_bk(gr);
        const int maxsb = gr < T20_NUM_HYBRID_GROUPS ? JAAD_PS_GROUP_BORDER20[gr] + 1 : JAAD_PS_GROUP_BORDER20[gr + 1];
        for (int env = 0; env < ps->num_env; env++) {
            int iid_index = ps->iid_index[env][bk];
            int iid_sign = iid_index < 0 ? -1 : 1;
            iid_index = abs(iid_index);
            int icc_index = ps->icc_index[env][bk];
            if (ps->icc_mode < 3) { /* type 'A' (:433-467) */
                float c_1 = sf_iid[num_steps + iid_index];
                float c_2 = sf_iid[num_steps - iid_index];
                float cosa = JAAD_PS_COS_ALPHAS[icc_index];
                float sina = JAAD_PS_SIN_ALPHAS[icc_index];
                float cosb = cos_betas[iid_index * 8 + icc_index];
                float sinb = sin_betas[iid_index * 8 + icc_index] * (float)iid_sign;
                float ab1 = (cosb * cosa), ab2 = (sinb * sina), ab3 = (sinb * cosa), ab4 = (cosb * sina);
                h11[0] = (c_2 * (ab1 - ab2));
                h12[0] = (c_1 * (ab1 + ab2));
                h21[0] = (c_2 * (ab3 + ab4));
                h22[0] = (c_1 * (ab3 - ab4));
            } else { /* type 'B' (:468-482) */
                float cosa = sincos_alphas_b[(num_steps + iid_index) * 8 + icc_index];
                float sina = sincos_alphas_b[(2 * num_steps - (num_steps + iid_index)) * 8 + icc_index];
                float cosg = cos_gammas[iid_index * 8 + icc_index];
                float sing = sin_gammas[iid_index * 8 + icc_index];
                h11[0] = (COEF_SQRT2 * (cosa * cosg));
                h12[0] = (COEF_SQRT2 * (sina * cosg));
                h21[0] = (COEF_SQRT2 * (-cosa * sing));
                h22[0] = (COEF_SQRT2 * (sina * sing));
            }
            if (bk < nr_ipdopd_par) { /* phase rotation (:484-567) */
                float* ipd_prev = ps->ipd_prev[bk][ps->phase_hist];
                float* opd_prev = ps->opd_prev[bk][ps->phase_hist];
                tempLeft[0] = (ipd_prev[0] * 0.25f);
                tempLeft[1] = (ipd_prev[1] * 0.25f);
                tempRight[0] = (opd_prev[0] * 0.25f);
                tempRight[1] = (opd_prev[1] * 0.25f);
                /* both indices are read from the IPD data (:502-503) */
                const int ipd_index = abs(ps->ipd_index[env][bk]);
                const int opd_index = abs(ps->ipd_index[env][bk]);
                ipd_prev[0] = JAAD_PS_IPDOPD_COS[ipd_index];
                ipd_prev[1] = JAAD_PS_IPDOPD_SIN[ipd_index];
                opd_prev[0] = JAAD_PS_IPDOPD_COS[opd_index];
                opd_prev[1] = JAAD_PS_IPDOPD_SIN[opd_index];
                tempLeft[0] += ipd_prev[0];
                tempLeft[1] += ipd_prev[1];
                tempRight[0] += opd_prev[0];
                tempRight[1] += opd_prev[1];
                ps->phase_hist = (ps->phase_hist + 1) % 2;
                /* the value before previous comes from opd.prev for both (:519-520) */
                ipd_prev = ps->opd_prev[bk][ps->phase_hist];
                opd_prev = ps->opd_prev[bk][ps->phase_hist];
                tempLeft[0] += (ipd_prev[0] * 0.5f);
                tempLeft[1] += (ipd_prev[1] * 0.5f);
                tempRight[0] += (opd_prev[0] * 0.5f);
                tempRight[1] += (opd_prev[1] * 0.5f);
                const float xy = magnitude_c(tempRight);
                const float pq = magnitude_c(tempLeft);
                if (xy != 0) {
                    phaseLeft[0] = (tempRight[0] / xy);
                    phaseLeft[1] = (tempRight[1] / xy);
                } else {
                    phaseLeft[0] = 0;
                    phaseLeft[1] = 0;
                }
                const float xypq = (xy * pq);
                if (xypq != 0) {
                    const float tmp1 = (tempRight[0] * tempLeft[0]) + (tempRight[1] * tempLeft[1]);
                    const float tmp2 = (tempRight[1] * tempLeft[0]) - (tempRight[0] * tempLeft[1]);
                    phaseRight[0] = (tmp1 / xypq);
                    phaseRight[1] = (tmp2 / xypq);
                } else {
                    phaseRight[0] = 0;
                    phaseRight[1] = 0;
                }
                h11[1] = (h11[0] * phaseLeft[1]);
                h12[1] = (h12[0] * phaseRight[1]);
                h21[1] = (h21[0] * phaseLeft[1]);
                h22[1] = (h22[0] * phaseRight[1]);
                h11[0] = (h11[0] * phaseLeft[0]);
                h12[0] = (h12[0] * phaseRight[0]);
                h21[0] = (h21[0] * phaseLeft[0]);
                h22[0] = (h22[0] * phaseRight[0]);
            }
            const float L = (float)(ps->border_position[env + 1] - ps->border_position[env]);
            deltaH11[0] = (h11[0] - ps->h11_prev[gr][0]) / L;
            deltaH12[0] = (h12[0] - ps->h12_prev[gr][0]) / L;
            deltaH21[0] = (h21[0] - ps->h21_prev[gr][0]) / L;
            deltaH22[0] = (h22[0] - ps->h22_prev[gr][0]) / L;
            H11[0] = ps->h11_prev[gr][0];
            H12[0] = ps->h12_prev[gr][0];
            H21[0] = ps->h21_prev[gr][0];
            H22[0] = ps->h22_prev[gr][0];
            ps->h11_prev[gr][0] = h11[0];
            ps->h12_prev[gr][0] = h12[0];
            ps->h21_prev[gr][0] = h21[0];
            ps->h22_prev[gr][0] = h22[0];
            if (bk < nr_ipdopd_par) {
                deltaH11[1] = (h11[1] - ps->h11_prev[gr][1]) / L;
                deltaH12[1] = (h12[1] - ps->h12_prev[gr][1]) / L;
                deltaH21[1] = (h21[1] - ps->h21_prev[gr][1]) / L;
                deltaH22[1] = (h22[1] - ps->h22_prev[gr][1]) / L;
                H11[1] = ps->h11_prev[gr][1];
                H12[1] = ps->h12_prev[gr][1];
                H21[1] = ps->h21_prev[gr][1];
                H22[1] = ps->h22_prev[gr][1];
                if (bk != 0) { /* FBType.bkm tests the band bits, not NEGATE_IPD_MASK (A/ps/FBType.java:71-73) */
                    deltaH11[1] = -deltaH11[1];
                    deltaH12[1] = -deltaH12[1];
                    deltaH21[1] = -deltaH21[1];
                    deltaH22[1] = -deltaH22[1];
                    H11[1] = -H11[1];
                    H12[1] = -H12[1];
                    H21[1] = -H21[1];
                    H22[1] = -H22[1];
                }
                ps->h11_prev[gr][1] = h11[1];
                ps->h12_prev[gr][1] = h12[1];
                ps->h21_prev[gr][1] = h21[1];
                ps->h22_prev[gr][1] = h22[1];
            }
            for (int n = ps->border_position[env]; n < ps->border_position[env + 1]; n++) {
                H11[0] += deltaH11[0];
                H12[0] += deltaH12[0];
                H21[0] += deltaH21[0];
                H22[0] += deltaH22[0];
                if (bk < nr_ipdopd_par) {
                    H11[1] += deltaH11[1];
                    H12[1] += deltaH12[1];
                    H21[1] += deltaH21[1];
                    H22[1] += deltaH22[1];
                }
                for (int sb = JAAD_PS_GROUP_BORDER20[gr]; sb < maxsb; sb++) {
                    float inLeft[2], inRight[2], tl[2], tr[2];
                    const int hyb = gr < T20_NUM_HYBRID_GROUPS;
                    inLeft[0] = hyb ? X_hybrid_left[n][sb][0] : X_left[n][sb][0];
                    inLeft[1] = hyb ? X_hybrid_left[n][sb][1] : X_left[n][sb][1];
                    inRight[0] = hyb ? X_hybrid_right[n][sb][0] : X_right[n][sb][0];
                    inRight[1] = hyb ? X_hybrid_right[n][sb][1] : X_right[n][sb][1];
                    tl[0] = (H11[0] * inLeft[0]) + (H21[0] * inRight[0]);
                    tl[1] = (H11[0] * inLeft[1]) + (H21[0] * inRight[1]);
                    tr[0] = (H12[0] * inLeft[0]) + (H22[0] * inRight[0]);
                    tr[1] = (H12[0] * inLeft[1]) + (H22[0] * inRight[1]);
                    if (bk < nr_ipdopd_par) {
                        tl[0] -= (H11[1] * inLeft[1]) + (H21[1] * inRight[1]);
                        tl[1] += (H11[1] * inLeft[0]) + (H21[1] * inRight[0]);
                        tr[0] -= (H12[1] * inLeft[1]) + (H22[1] * inRight[1]);
                        tr[1] += (H12[1] * inLeft[0]) + (H22[1] * inRight[0]);
                    }
                    float* ol = hyb ? X_hybrid_left[n][sb] : X_left[n][sb];
                    float* orr = hyb ? X_hybrid_right[n][sb] : X_right[n][sb];
                    ol[0] = tl[0];
                    ol[1] = tl[1];
                    orr[0] = tr[0];
                    orr[1] = tr[1];
                }
            }
        }
    }
}

/* PSImpl.process (A/ps/PSImpl.java:685-707); X_left [38][64], X_right [38][64] */
void orc_ps_process(orc_ps* ps, float (*X_left)[64][2], float (*X_right)[64][2])
{
    float X_hybrid_left[32][32][2], X_hybrid_right[32][32][2];
    memset(X_hybrid_left, 0, sizeof X_hybrid_left);
    memset(X_hybrid_right, 0, sizeof X_hybrid_right);
    hybrid_analysis(ps, X_left, X_hybrid_left);
    ps_decorrelate(ps, X_left, X_right, X_hybrid_left, X_hybrid_right);
    ps_mix_phase(ps, X_left, X_right, X_hybrid_left, X_hybrid_right);
    hybrid_synthesis(ps, X_left, X_hybrid_left);
    hybrid_synthesis(ps, X_right, X_hybrid_right);
}

/* tests: hybrid analysis of X [38][64][2] with a fresh filterbank -> X_hybrid [32][32][2] */
void orc_ps_hybrid_analysis(const float* X, float* X_hybrid)
{
    orc_ps* ps = (orc_ps*)calloc(1, sizeof(orc_ps));
    if (!ps) return;
    orc_ps_init(ps);
    float Xl[38][64][2];
    memcpy(Xl, X, sizeof Xl);
    memset(X_hybrid, 0, 32 * 32 * 2 * sizeof(float));
    hybrid_analysis(ps, Xl, (float(*)[32][2])X_hybrid);
    free(ps);
}
