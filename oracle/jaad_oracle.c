/*
 * jaad_oracle.c -- TEST INFRASTRUCTURE ONLY (see jaad_oracle.h for the parity status).
 *
 * Restates, operation for operation and in the same binary32 evaluation order, the Java DSP of
 * pucgenie/JAADec.  Paths below are relative to aac/src/main/java/net/sourceforge/jaad/aac/
 * ("A/") and src/main/java/net/sourceforge/jaad/ ("S/").  Build: gcc -O2 -ffp-contract=off.
 */
#include "jaad_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../jaadec_amd/csrc/tables/jaad_tables.inc"

#if defined(__FP_FAST_FMAF) || defined(__FAST_MATH__)
#error "the oracle must be compiled without fast-math / FMA contraction"
#endif

/* SampleFrequency maxTNS_SFB {long, short} (A/SampleFrequency.java:15-26) */
static const unsigned char MAX_TNS_SFB[12][2] = {
    {31, 9}, {31, 9}, {34, 10}, {40, 14}, {42, 14}, {51, 14},
    {46, 14}, {46, 14}, {42, 14}, {42, 14}, {42, 14}, {39, 14}};

/* ------------------------------------------------------------------------------------------ */
/* FFT.process (A/filterbank/FFT.java:48-135)                                                  */
/* ------------------------------------------------------------------------------------------ */
void orc_fft(float (*in)[2], int length, int forward)
{
    float rev[512][2];
    const float(*roots)[2] = NULL;
    const float(*roots3)[3] = NULL;
    if (length == 512) roots3 = JAAD_FFT_TABLE_512;
    else roots = JAAD_FFT_TABLE_64;

    /* bit-reversal (FFT.java:51-66) */
    int ii = 0;
    for (int i = 0; i < length; i++) {
        rev[i][0] = in[ii][0];
        rev[i][1] = in[ii][1];
        int k = length >> 1;
        while (ii >= k && k > 0) {
            ii -= k;
            k >>= 1;
        }
        ii += k;
    }
    for (int i = 0; i < length; i++) {
        in[i][0] = rev[i][0];
        in[i][1] = rev[i][1];
    }
    /* bottom radix-4 round (FFT.java:69-108) */
    for (int i = 0; i < length; i += 4) {
        float aRe = in[i][0] + in[i + 1][0];
        float aIm = in[i][1] + in[i + 1][1];
        float bRe = in[i + 2][0] + in[i + 3][0];
        float bIm = in[i + 2][1] + in[i + 3][1];
        float cRe = in[i][0] - in[i + 1][0];
        float cIm = in[i][1] - in[i + 1][1];
        float dRe = in[i + 2][0] - in[i + 3][0];
        float dIm = in[i + 2][1] - in[i + 3][1];
        in[i][0] = aRe + bRe;
        in[i][1] = aIm + bIm;
        in[i + 2][0] = aRe - bRe;
        in[i + 2][1] = aIm - bIm;
        float e1Re = cRe - dIm, e1Im = cIm + dRe;
        float e2Re = cRe + dIm, e2Im = cIm - dRe;
        if (forward) {
            in[i + 1][0] = e2Re; in[i + 1][1] = e2Im;
            in[i + 3][0] = e1Re; in[i + 3][1] = e1Im;
        } else {
            in[i + 1][0] = e1Re; in[i + 1][1] = e1Im;
            in[i + 3][0] = e2Re; in[i + 3][1] = e2Im;
        }
    }
    /* radix-2 stages (FFT.java:110-134); inverse uses column 1 (+sin), forward column 2 */
    for (int i = 4; i < length; i <<= 1) {
        int shift = i << 1;
        int m = length / shift;
        for (int j = 0; j < length; j += shift) {
            for (int k = 0; k < i; k++) {
                int km = k * m;
                float rootRe, rootIm;
                if (roots3) {
                    rootRe = roots3[km][0];
                    rootIm = roots3[km][forward ? 2 : 1];
                } else {
                    rootRe = roots[km][0];
                    rootIm = roots[km][1]; /* 64-point table has no forward column (LTP only) */
                }
                float* v0 = in[j + k];
                float* v1 = in[i + k + j];
                float zRe = v1[0] * rootRe - v1[1] * rootIm;
                float zIm = v1[0] * rootIm + v1[1] * rootRe;
                v1[0] = v0[0] - zRe;
                v1[1] = v0[1] - zIm;
                v0[0] = v0[0] + zRe;
                v0[1] = v0[1] + zIm;
            }
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* MDCT.process (A/filterbank/MDCT.java:36-81)                                                 */
/* ------------------------------------------------------------------------------------------ */
void orc_imdct(const float* in, float* out, int N)
{
    const int N2 = N >> 1, N4 = N >> 2, N8 = N >> 3;
    const float(*sincos)[2] = (N == 2048) ? JAAD_MDCT_TABLE_2048 : JAAD_MDCT_TABLE_128;
    float buf[512][2];
    for (int k = 0; k < N4; k++) {
        buf[k][1] = (in[2 * k] * sincos[k][0]) + (in[N2 - 1 - 2 * k] * sincos[k][1]);
        buf[k][0] = (in[N2 - 1 - 2 * k] * sincos[k][0]) - (in[2 * k] * sincos[k][1]);
    }
    orc_fft(buf, N4, 0);
    for (int k = 0; k < N4; k++) {
        float t0 = buf[k][0];
        float t1 = buf[k][1];
        buf[k][1] = (t1 * sincos[k][0]) + (t0 * sincos[k][1]);
        buf[k][0] = (t0 * sincos[k][0]) - (t1 * sincos[k][1]);
    }
    for (int k = 0; k < N8; k += 2) {
        out[2 * k] = buf[N8 + k][1];
        out[2 + 2 * k] = buf[N8 + 1 + k][1];
        out[1 + 2 * k] = -buf[N8 - 1 - k][0];
        out[3 + 2 * k] = -buf[N8 - 2 - k][0];
        out[N4 + 2 * k] = buf[k][0];
        out[N4 + 2 + 2 * k] = buf[1 + k][0];
        out[N4 + 1 + 2 * k] = -buf[N4 - 1 - k][1];
        out[N4 + 3 + 2 * k] = -buf[N4 - 2 - k][1];
        out[N2 + 2 * k] = buf[N8 + k][0];
        out[N2 + 2 + 2 * k] = buf[N8 + 1 + k][0];
        out[N2 + 1 + 2 * k] = -buf[N8 - 1 - k][1];
        out[N2 + 3 + 2 * k] = -buf[N8 - 2 - k][1];
        out[N2 + N4 + 2 * k] = -buf[k][1];
        out[N2 + N4 + 2 + 2 * k] = -buf[1 + k][1];
        out[N2 + N4 + 1 + 2 * k] = buf[N4 - 1 - k][0];
        out[N2 + N4 + 3 + 2 * k] = buf[N4 - 2 - k][0];
    }
}

/* ------------------------------------------------------------------------------------------ */
/* FilterBank.process (A/filterbank/FilterBank.java:39-123), 1024-sample frames                */
/* ------------------------------------------------------------------------------------------ */
void orc_filterbank(int seq, int shape, int shape_prev, const float* in, float* out, float* overlap)
{
    const float* LW[2] = {JAAD_SINE_1024, JAAD_KBD_1024};
    const float* SW[2] = {JAAD_SINE_128, JAAD_KBD_128};
    const int length = 1024, shortLen = 128, mid = 448, trans = 64;
    float buf[2048];
    int i;
    switch (seq) {
    case JAAD_ONLY_LONG_SEQUENCE:
        orc_imdct(in, buf, 2048);
        for (i = 0; i < length; i++) out[i] = overlap[i] + (buf[i] * LW[shape_prev][i]);
        for (i = 0; i < length; i++) overlap[i] = buf[length + i] * LW[shape][length - 1 - i];
        break;
    case JAAD_LONG_START_SEQUENCE:
        orc_imdct(in, buf, 2048);
        for (i = 0; i < length; i++) out[i] = overlap[i] + (buf[i] * LW[shape_prev][i]);
        for (i = 0; i < mid; i++) overlap[i] = buf[length + i];
        for (i = 0; i < shortLen; i++) overlap[mid + i] = buf[length + mid + i] * SW[shape][shortLen - i - 1];
        for (i = 0; i < mid; i++) overlap[mid + shortLen + i] = 0;
        break;
    case JAAD_EIGHT_SHORT_SEQUENCE: {
        const float* S = SW[shape];
        for (i = 0; i < 8; i++) orc_imdct(in + i * shortLen, buf + 2 * i * shortLen, 256);
        for (i = 0; i < mid; i++) out[i] = overlap[i];
        for (i = 0; i < shortLen; i++) {
            out[mid + i] = overlap[mid + i] + (buf[i] * SW[shape_prev][i]);
            out[mid + 1 * shortLen + i] = overlap[mid + shortLen * 1 + i] + (buf[shortLen * 1 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 2 + i] * S[i]);
            out[mid + 2 * shortLen + i] = overlap[mid + shortLen * 2 + i] + (buf[shortLen * 3 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 4 + i] * S[i]);
            out[mid + 3 * shortLen + i] = overlap[mid + shortLen * 3 + i] + (buf[shortLen * 5 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 6 + i] * S[i]);
            if (i < trans)
                out[mid + 4 * shortLen + i] = overlap[mid + shortLen * 4 + i] + (buf[shortLen * 7 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 8 + i] * S[i]);
        }
        for (i = 0; i < shortLen; i++) {
            if (i >= trans)
                overlap[mid + 4 * shortLen + i - length] = (buf[shortLen * 7 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 8 + i] * S[i]);
            overlap[mid + 5 * shortLen + i - length] = (buf[shortLen * 9 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 10 + i] * S[i]);
            overlap[mid + 6 * shortLen + i - length] = (buf[shortLen * 11 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 12 + i] * S[i]);
            overlap[mid + 7 * shortLen + i - length] = (buf[shortLen * 13 + i] * S[shortLen - 1 - i]) + (buf[shortLen * 14 + i] * S[i]);
            overlap[mid + 8 * shortLen + i - length] = (buf[shortLen * 15 + i] * S[shortLen - 1 - i]);
        }
        for (i = 0; i < mid; i++) overlap[mid + shortLen + i] = 0;
        break;
    }
    case JAAD_LONG_STOP_SEQUENCE:
        orc_imdct(in, buf, 2048);
        for (i = 0; i < mid; i++) out[i] = overlap[i];
        for (i = 0; i < shortLen; i++) out[mid + i] = overlap[mid + i] + (buf[mid + i] * SW[shape_prev][i]);
        for (i = 0; i < mid; i++) out[mid + shortLen + i] = overlap[mid + shortLen + i] + buf[mid + shortLen + i];
        for (i = 0; i < length; i++) overlap[i] = buf[length + i] * LW[shape][length - 1 - i];
        break;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* ICSInfo window grouping (A/syntax/ICSInfo.java:93-107)                                      */
/* ------------------------------------------------------------------------------------------ */
static int group_lengths(const jaad_ics_info* info, int* glen)
{
    int n = 1;
    glen[0] = 1;
    if (info->window_sequence != JAAD_EIGHT_SHORT_SEQUENCE) return 1;
    for (int i = 0; i < 7; i++) {
        if (info->grouping & (1u << i)) glen[n - 1]++;
        else glen[n++] = 1;
    }
    return n;
}

static const short* swb_offsets(const jaad_ics_info* info, int sf_index, int* count)
{
    if (info->window_sequence == JAAD_EIGHT_SHORT_SEQUENCE) {
        *count = JAAD_SWB_SHORT_WINDOW_COUNT[sf_index];
        return JAAD_SWB_OFFSET_SHORT_WINDOW[sf_index];
    }
    *count = JAAD_SWB_LONG_WINDOW_COUNT[sf_index];
    return JAAD_SWB_OFFSET_LONG_WINDOW[sf_index];
}

/* ------------------------------------------------------------------------------------------ */
/* ICStream.decodeSpectralData, IQ + PNS half (A/syntax/ICStream.java:222-275)                 */
/* ------------------------------------------------------------------------------------------ */
int orc_dequant(const jaad_ics_info* info, int sf_index, const int16_t* q, const uint8_t* sf,
                const uint8_t* cb, uint32_t* rand_state, float* iqData)
{
    int glen[8], nswb;
    const int windowGroups = group_lengths(info, glen);
    const short* offsets = swb_offsets(info, sf_index, &nswb);
    const int maxSFB = info->max_sfb;
    if (maxSFB > nswb) return JAAD_ERR_BITSTREAM;
    int32_t randomState = (int32_t)*rand_state;

    memset(iqData, 0, 1024 * sizeof(float));
    for (int g = 0, idx = 0, groupOff = 0; g < windowGroups; g++) {
        int groupLen = glen[g];
        for (int sfb = 0; sfb < maxSFB; sfb++, idx++) {
            int hcb = cb[idx];
            int off = groupOff + offsets[sfb];
            int width = offsets[sfb + 1] - offsets[sfb];
            /* scaleFactors[idx] as decodeScaleFactors left it (ICStream.java:172-220) */
            float sfv = JAAD_SCALEFACTOR_TABLE[sf[idx] + 100];
            if (hcb == JAAD_ZERO_HCB || hcb == JAAD_INTENSITY_HCB || hcb == JAAD_INTENSITY_HCB2) {
                /* stays zero */
            } else if (hcb == JAAD_NOISE_HCB) {
                float scalefactor = -sfv;
                for (int w = 0; w < groupLen; w++, off += 128) {
                    float energy = 0;
                    for (int k = 0; k < width; k++) {
                        randomState = (int32_t)(1664525u * (uint32_t)randomState + 1013904223u);
                        iqData[off + k] = (float)randomState;
                        energy += iqData[off + k] * iqData[off + k];
                    }
                    float scale = (float)((double)scalefactor / sqrt((double)energy));
                    for (int k = 0; k < width; k++) iqData[off + k] *= scale;
                }
            } else {
                for (int w = 0; w < groupLen; w++, off += 128) {
                    for (int k = 0; k < width; k++) {
                        int v = q[off + k];
                        iqData[off + k] = (v > 0) ? JAAD_IQ_TABLE[v] : -JAAD_IQ_TABLE[-v];
                        iqData[off + k] *= sfv;
                    }
                }
            }
        }
        groupOff += groupLen << 7;
    }
    *rand_state = (uint32_t)randomState;
    return JAAD_OK;
}

static int ms_bit(const uint64_t* ms_used, int idx) { return (int)((ms_used[idx >> 6] >> (idx & 63)) & 1u); }

/* MS.process (A/tools/MS.java:17-41) */
void orc_ms(const jaad_ics_info* info, int sf_index, const uint8_t* cbL, const uint8_t* cbR,
            const uint64_t* ms_used, float* specL, float* specR)
{
    int glen[8], nswb;
    const int windowGroups = group_lengths(info, glen);
    const short* offsets = swb_offsets(info, sf_index, &nswb);
    const int maxSFB = info->max_sfb;
    for (int g = 0, idx = 0, groupOff = 0; g < windowGroups; g++) {
        for (int i = 0; i < maxSFB; i++, idx++) {
            if (ms_bit(ms_used, idx) && cbL[idx] < JAAD_NOISE_HCB && cbR[idx] < JAAD_NOISE_HCB) {
                for (int w = 0; w < glen[g]; w++) {
                    int off = groupOff + w * 128 + offsets[i];
                    for (int j = 0; j < offsets[i + 1] - offsets[i]; j++) {
                        float t = specL[off + j] - specR[off + j];
                        specL[off + j] += specR[off + j];
                        specR[off + j] = t;
                    }
                }
            }
        }
        groupOff += glen[g] * 128;
    }
}

/* IS.process (A/tools/IS.java:17-53); infoL carries the CPE's ms-mask-present flag */
void orc_is(const jaad_ics_info* infoL, const jaad_ics_info* info, int sf_index, const uint8_t* sfbCB,
            const uint8_t* sfR, const uint64_t* ms_used, float* specL, float* specR)
{
    int glen[8], nswb;
    const int windowGroups = group_lengths(info, glen);
    const short* offsets = swb_offsets(info, sf_index, &nswb);
    const int maxSFB = info->max_sfb;
    const int msMaskPresent = (infoL->flags & JAAD_ICS_MS_PRESENT) != 0;
    for (int g = 0, idx = 0, groupOff = 0; g < windowGroups; g++) {
        for (int i = 0; i < maxSFB; i++, idx++) {
            if (sfbCB[idx] == JAAD_INTENSITY_HCB || sfbCB[idx] == JAAD_INTENSITY_HCB2) {
                int c = sfbCB[idx] == JAAD_INTENSITY_HCB ? 1 : -1;
                if (msMaskPresent) c *= ms_bit(ms_used, idx) ? -1 : 1;
                float scale = (float)c * JAAD_SCALEFACTOR_TABLE[sfR[idx] + 100];
                for (int w = 0; w < glen[g]; w++) {
                    int off = groupOff + w * 128 + offsets[i];
                    for (int j = 0; j < offsets[i + 1] - offsets[i]; j++) specR[off + j] = specL[off + j] * scale;
                }
            }
        }
        groupOff += glen[g] * 128;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* TNS, spec mode: ISO/IEC 14496-3 4.6.9.3 (tns_decode_coef + all-pole tns_ar_filter).         */
/* The reference only parses TNS (A/tools/TNS.java:35-61) and its process() is a no-op.       */
/* Coefficient values: the reference tables (A/tools/TNSTables.java) hold -sin(...) of the    */
/* ISO inverse quantiser, so the ISO value is the negated table entry.                         */
/* ------------------------------------------------------------------------------------------ */
static const float* tns_table(int compress, int res)
{
    switch (2 * compress + res) {
    case 0: return JAAD_TNS_COEF_0_3;
    case 1: return JAAD_TNS_COEF_0_4;
    case 2: return JAAD_TNS_COEF_1_3;
    default: return JAAD_TNS_COEF_1_4;
    }
}

void orc_tns_spec(const jaad_ics_info* info, int sf_index, const jaad_tns* tns, float* spec)
{
    const int is_short = info->window_sequence == JAAD_EIGHT_SHORT_SEQUENCE;
    int nswb;
    const short* offsets = swb_offsets(info, sf_index, &nswb);
    const int tns_max = MAX_TNS_SFB[sf_index][is_short];
    int bottom_w[8];
    for (int w = 0; w < 8; w++) bottom_w[w] = nswb;
    for (int f = 0; f < tns->n_filters; f++) {
        const jaad_tns_filter* F = &tns->filt[f];
        int w = F->window;
        int top = bottom_w[w];
        int bottom = top - F->length;
        if (bottom < 0) bottom = 0;
        bottom_w[w] = bottom;
        int order = F->order;
        if (!order) continue;
        const float* tab = tns_table((F->flags >> 2) & 1, (F->flags >> 1) & 1);
        float tmp2[20], a[21], b[21];
        for (int i = 0; i < order; i++) tmp2[i] = -tab[F->coef[i]];
        a[0] = 1.0f;
        for (int m = 1; m <= order; m++) {
            for (int i = 1; i < m; i++) b[i] = a[i] + tmp2[m - 1] * a[m - i];
            for (int i = 1; i < m; i++) a[i] = b[i];
            a[m] = tmp2[m - 1];
        }
        int s = bottom < tns_max ? bottom : tns_max;
        if (s > info->max_sfb) s = info->max_sfb;
        int e = top < tns_max ? top : tns_max;
        if (e > info->max_sfb) e = info->max_sfb;
        int start = offsets[s], end = offsets[e];
        int size = end - start;
        if (size <= 0) continue;
        int inc = 1;
        if (F->flags & 1) {
            inc = -1;
            start = end - 1;
        }
        float state[20] = {0};
        float* x = spec + (is_short ? w * 128 : 0) + start;
        for (int n = 0; n < size; n++, x += inc) {
            float y = *x;
            for (int j = 0; j < order; j++) y -= state[j] * a[j + 1];
            for (int j = order - 1; j > 0; j--) state[j] = state[j - 1];
            state[0] = y;
            *x = y;
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* SampleBuffer.accept (S/SampleBuffer.java:168-209)                                           */
/* ------------------------------------------------------------------------------------------ */
static int java_round_clamp16(float s, int* clipped)
{
    /* Math.round(float): floor(s + 1/2) evaluated exactly (ties toward +inf); NaN -> 0;
       saturating to int, then clamped to the short range. */
    int pulse;
    if (s != s) pulse = 0;
    else {
        double r = floor((double)s + 0.5);
        pulse = r >= 2147483647.0 ? 2147483647 : r <= -2147483648.0 ? (int)-2147483647 - 1 : (int)r;
    }
    if (pulse > 32767 || pulse < -32768) (*clipped)++;
    return pulse > 32767 ? 32767 : pulse < -32768 ? -32768 : pulse;
}

int orc_pcm_pack(const float* const* ch, int n_ch, int len, uint32_t flags, void* out)
{
    int clipped = 0;
    unsigned char* o = (unsigned char*)out;
    for (int is = 0; is < len; ++is) {
        for (int c = 0; c < n_ch; c++) {
            float s = ch[c][is]; /* k = sample.length*is/sampleLength == is: equal lengths here */
            if (flags & JAAD_PCM_FLOAT32) {
                memcpy(o, &s, 4);
                o += 4;
                continue;
            }
            int v = java_round_clamp16(s, &clipped);
            uint16_t u = (uint16_t)(int16_t)v;
            if (flags & JAAD_PCM_LITTLE_ENDIAN) { o[0] = (unsigned char)(u & 0xff); o[1] = (unsigned char)(u >> 8); }
            else { o[0] = (unsigned char)(u >> 8); o[1] = (unsigned char)(u & 0xff); }
            o += 2;
        }
    }
    return clipped;
}

/* ------------------------------------------------------------------------------------------ */
/* Frame driver: SCE.process (A/syntax/SCE.java:90-133) / CPE.process (A/syntax/CPE.java:149-208)
 * + SyntacticElements.process mono->stereo duplication (A/syntax/SyntacticElements.java:235-248) */
/* ------------------------------------------------------------------------------------------ */
size_t orc_stream_bytes(void) { return sizeof(orc_stream); }

void orc_streams_free(orc_stream* streams, int n)
{
    for (int i = 0; i < n; i++) {
        orc_sbr_free(streams[i].sbr);
        free(streams[i].sbr);
        streams[i].sbr = NULL;
    }
}

/* SBR doubles the output rate unless it runs downsampled (extension rate = core rate) */
static int sbr_down(const jaad_stream_cfg* cfg) { return cfg->sbr && cfg->ext_sf_index == cfg->sf_index; }
static int frame_samples(const jaad_stream_cfg* cfg) { return cfg->sbr && !sbr_down(cfg) ? 2048 : 1024; }

/* ChannelElement.processDependentCoupling (A/syntax/ChannelElement.java:105-130) at `point` for
 * the frame's channels: every term of frame f (jaad_gpu.h jaad_cce_term, in the reference's order)
 * runs CCE.applyDependentCoupling (A/syntax/CCE.java:188-215) on its target's spectrum, with the
 * CCE's ICStream spectrum from decodeSpectralData (its own LCG state: cce_ics.pns_state). */
static int orc_couple(const jaad_stream_cfg* cfg, const jaad_batch* b, uint32_t f, int point, int nch,
                      float (*spec)[1024])
{
    uint32_t lo = 0, hi = b->n_cce_terms;
    while (lo < hi) { /* first term of frame f (terms are sorted by frame) */
        const uint32_t m = (lo + hi) / 2;
        if (b->cce_terms[m].frame < f) lo = m + 1;
        else hi = m;
    }
    for (uint32_t t = lo; t < b->n_cce_terms && b->cce_terms[t].frame == f; t++) {
        const jaad_cce_term* T = &b->cce_terms[t];
        if (T->point != point) continue;
        if (T->channel >= nch || T->cce >= b->n_cce) return JAAD_ERR_INVALID_ARG;
        const jaad_ics_info* info = &b->cce_ics[T->cce];
        const uint8_t* sfbCB = b->cce_cb + (size_t)T->cce * 128;
        float iqData[1024];
        uint32_t rs = info->pns_state;
        int rc = orc_dequant(info, cfg->sf_index, b->cce_q + (size_t)T->cce * 1024, b->cce_sf + (size_t)T->cce * 128,
                             sfbCB, &rs, iqData);
        if (rc) return rc;
        int glen[8], nswb;
        const int windowGroupCount = group_lengths(info, glen);
        const short* swbOffsets = swb_offsets(info, cfg->sf_index, &nswb);
        const int maxSFB = info->max_sfb;
        float* data = spec[T->channel];
        int srcOff = 0, dstOff = 0, idx = 0;
        for (int g = 0; g < windowGroupCount; g++) {
            const int len = glen[g];
            for (int sfb = 0; sfb < maxSFB; sfb++, idx++) {
                if (sfbCB[idx] != JAAD_ZERO_HCB) {
                    const float x = T->gain[idx];
                    for (int group = 0; group < len; group++)
                        for (int k = swbOffsets[sfb]; k < swbOffsets[sfb + 1]; k++)
                            data[dstOff + group * 128 + k] += x * iqData[srcOff + group * 128 + k];
                }
            }
            dstOff += len * 128;
            srcOff += len * 128;
        }
    }
    return JAAD_OK;
}

static int decode_frame(const jaad_stream_cfg* cfg, orc_stream* st, const jaad_batch* b, uint32_t f,
                        uint32_t* rand_state, unsigned char* pcm, uint32_t flags)
{
    const int nch = cfg->channel_config == 2 ? 2 : 1;
    float iq[2][1024], data[2][2048];
    int rc;
    for (int c = 0; c < nch; c++) {
        size_t cf = (size_t)f * nch + c;
        const jaad_ics_info* info = &b->ics[cf];
        uint32_t rs = info->pns_state; /* host-recorded static LCG state for this ICStream */
        rc = orc_dequant(info, cfg->sf_index, b->q + cf * 1024, b->sf + cf * 128, b->cb + cf * 128, &rs, iq[c]);
        if (rc) return rc;
        *rand_state = rs;
    }
    if (nch == 2) {
        size_t cL = (size_t)f * 2, cR = cL + 1;
        const jaad_ics_info* iL = &b->ics[cL];
        const uint64_t* ms = b->ms_used ? b->ms_used + (size_t)f * 2 : NULL;
        if ((iL->flags & JAAD_ICS_COMMON_WINDOW) && (iL->flags & JAAD_ICS_MS_PRESENT) && ms)
            orc_ms(iL, cfg->sf_index, b->cb + cL * 128, b->cb + cR * 128, ms, iq[0], iq[1]);
        static const uint64_t zero_ms[2] = {0, 0};
        orc_is(iL, &b->ics[cR], cfg->sf_index, b->cb + cR * 128, b->sf + cR * 128, ms ? ms : zero_ms, iq[0], iq[1]);
    }
    /* CPE.process / SCE.process: dependent coupling before TNS, TNS, dependent coupling after
       TNS (A/syntax/CPE.java:172-179, A/syntax/SCE.java:100-108) */
    if (b->n_cce_terms && (rc = orc_couple(cfg, b, f, 0, nch, iq))) return rc;
    for (int c = 0; c < nch; c++) {
        size_t cf = (size_t)f * nch + c;
        const jaad_ics_info* info = &b->ics[cf];
        if (cfg->tns_mode == JAAD_TNS_SPEC && (info->flags & JAAD_ICS_TNS) && b->tns)
            orc_tns_spec(info, cfg->sf_index, &b->tns[cf], iq[c]);
    }
    if (b->n_cce_terms && (rc = orc_couple(cfg, b, f, 1, nch, iq))) return rc;
    for (int c = 0; c < nch; c++) {
        size_t cf = (size_t)f * nch + c;
        const jaad_ics_info* info = &b->ics[cf];
        orc_filterbank(info->window_sequence, info->window_shape, info->window_shape_prev, iq[c], data[c],
                       st->overlap[c]);
    }
    if (cfg->sbr && b->sbr[f].status == JAAD_SBR_UPSAMPLE) {
        if (b->sbr[f].header_present) { /* SBR.decode still took the header (orc_sbr_take_header) */
            if (!st->sbr) return JAAD_ERR_UNSUPPORTED;  /* no SBR object has seen a header yet */
            rc = orc_sbr_take_header(st->sbr, &b->sbr[f].hdr);
            if (rc) return rc;
        }
        /* SBR invalid (ChannelElement.isSBRPresent false, A/syntax/ChannelElement.java:76-78):
         * CPE.process / SCE.process upsample the core instead (A/syntax/CPE.java:201-204,
         * A/syntax/SCE.java:129-131) when the buffer is longer than a frame; the SBR object is
         * not touched.  SBR.upsample (A/sbr/SBR.java:302-309) runs i = len/2-1 down to 1, so
         * data[0] and data[1] keep the core's first two samples. */
        if (frame_samples(cfg) != 1024)
            for (int c = 0; c < nch; c++)
                for (int i = 1024 - 1; i > 0; --i) {
                    const float v = data[c][i];
                    data[c][2 * i] = v;
                    data[c][2 * i + 1] = v;
                }
        /* one channel accepted for an SCE: SyntacticElements.process duplicates it */
        const float* chans[2] = {data[0], nch == 2 ? data[1] : data[0]};
        orc_pcm_pack(chans, 2, frame_samples(cfg), flags, pcm);
        return JAAD_OK;
    }
    if (cfg->sbr) {
        /* CPE.process / SCE.process -> SBR.process (A/syntax/CPE.java:195-204, SCE.java:122-133) */
        if (!st->sbr) {
            st->sbr = (orc_sbr*)calloc(1, orc_sbr_bytes());
            if (!st->sbr) return JAAD_ERR_NOMEM;
            orc_sbr_init(st->sbr, cfg->ext_sf_index);
            orc_sbr_set_downsampled(st->sbr, sbr_down(cfg));
        }
        rc = orc_sbr_decode(st->sbr, &b->sbr[f], nch);
        if (rc) return rc;
        orc_sbr_process(st->sbr, data[0], data[1], nch);
        const float* chans[2] = {data[0], data[1]};
        orc_pcm_pack(chans, 2, frame_samples(cfg), flags, pcm);
        return JAAD_OK;
    }
    const float* chans[2] = {data[0], nch == 2 ? data[1] : data[0]};
    orc_pcm_pack(chans, 2, 1024, flags, pcm);
    return JAAD_OK;
}

static int check_batch(const jaad_stream_cfg* cfg, const jaad_batch* b, size_t pcm_bytes, uint32_t flags)
{
    if (!cfg || !b || (!b->q && b->n_frames) || !b->sf || !b->cb || !b->ics || !b->frame_begin) return JAAD_ERR_INVALID_ARG;
    if (cfg->channel_config != 1 && cfg->channel_config != 2) return JAAD_ERR_UNSUPPORTED;
    if (cfg->sbr && (!b->sbr || (cfg->ext_sf_index + 3 != cfg->sf_index && !sbr_down(cfg)))) return JAAD_ERR_INVALID_ARG;
    if (cfg->ps && (!cfg->sbr || cfg->channel_config != 1)) return JAAD_ERR_UNSUPPORTED;
    size_t per = (size_t)frame_samples(cfg) * 2 * ((flags & JAAD_PCM_FLOAT32) ? 4 : 2);
    if (pcm_bytes < per * b->n_frames) return JAAD_ERR_INVALID_ARG;
    return JAAD_OK;
}

/* A frame dropped as Decoder.decodeFrame drops it (EOSException caught, process() and accept skipped,
 * A/Decoder.java:89-101): no DSP.  If its SBR payload was read whole before the bitstream ended,
 * SBR.decode had already swapped in its header and recomputed the frequency tables (A/sbr/SBR.java:
 * 162-184), as for a frame whose SBR data is invalid: orc_sbr_take_header. */
static int dropped_frame(const jaad_stream_cfg* cfg, orc_stream* st, const jaad_batch* b, uint32_t f)
{
    if (!cfg->sbr || !b->sbr || !b->sbr[f].header_present) return JAAD_OK;
    if (!st->sbr) return JAAD_ERR_UNSUPPORTED; /* no SBR frame has run: no patches to keep */
    return orc_sbr_take_header(st->sbr, &b->sbr[f].hdr);
}

int orc_decode_batch(const jaad_stream_cfg* cfg, orc_stream* streams, const jaad_batch* b, void* pcm_out,
                     size_t pcm_bytes, uint32_t flags)
{
    int rc = check_batch(cfg, b, pcm_bytes, flags);
    if (rc) return rc;
    size_t per = (size_t)frame_samples(cfg) * 2 * ((flags & JAAD_PCM_FLOAT32) ? 4 : 2);
    uint32_t rs = 0;
    for (uint32_t r = 0; r < b->n_runs; r++) {
        orc_stream* st = &streams[b->stream_slot[r]];
        for (uint32_t f = b->frame_begin[r]; f < b->frame_begin[r + 1]; f++) {
            if (b->frame_status && b->frame_status[f]) rc = dropped_frame(cfg, st, b, f);
            else rc = decode_frame(cfg, st, b, f, &rs, (unsigned char*)pcm_out + per * f, flags);
            if (rc) return rc;
        }
    }
    return JAAD_OK;
}

typedef struct {
    const jaad_stream_cfg* cfg;
    orc_stream* streams;
    const jaad_batch* b;
    unsigned char* pcm;
    uint32_t flags;
    size_t per;
    uint32_t r0, r1;
    int rc;
} mt_job;

static void* mt_worker(void* p)
{
    mt_job* j = (mt_job*)p;
    uint32_t rs = 0;
    for (uint32_t r = j->r0; r < j->r1 && !j->rc; r++) {
        orc_stream* st = &j->streams[j->b->stream_slot[r]];
        for (uint32_t f = j->b->frame_begin[r]; f < j->b->frame_begin[r + 1] && !j->rc; f++)
            j->rc = j->b->frame_status && j->b->frame_status[f]
                        ? dropped_frame(j->cfg, st, j->b, f)
                        : decode_frame(j->cfg, st, j->b, f, &rs, j->pcm + j->per * f, j->flags);
    }
    return NULL;
}

int orc_decode_batch_mt(const jaad_stream_cfg* cfg, orc_stream* streams, const jaad_batch* b, void* pcm_out,
                        size_t pcm_bytes, uint32_t flags, int threads)
{
    int rc = check_batch(cfg, b, pcm_bytes, flags);
    if (rc) return rc;
    if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (threads > 256) threads = 256;
    if ((uint32_t)threads > b->n_runs) threads = (int)(b->n_runs ? b->n_runs : 1);
    mt_job jobs[256];
    pthread_t tid[256];
    size_t per = (size_t)frame_samples(cfg) * 2 * ((flags & JAAD_PCM_FLOAT32) ? 4 : 2);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (mt_job){cfg, streams, b, (unsigned char*)pcm_out, flags, per,
                           (uint32_t)((uint64_t)b->n_runs * t / threads),
                           (uint32_t)((uint64_t)b->n_runs * (t + 1) / threads), 0};
        pthread_create(&tid[t], NULL, mt_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    return rc;
}
