/*
 * TEST INFRASTRUCTURE ONLY (never linked into the product): an AAC-LC raw_data_block WRITER.
 *
 * The reference has no bitstreams in its tests (PlayGoldDust needs an external
 * file), so the host parser (jaadec_amd/csrc/jaad_parse.cpp) is pinned by round trips: the
 * synthetic parsed-frame records of jaad_synth.h are written as ISO/IEC 14496-3 syntax with
 * the reference's own codebooks (A/huffman/Codebooks.java, carried as data in
 * jaad_huffman_tables.inc) and must parse back to exactly the same records.  The syntax written
 * is the one the reference reads:
 *   raw_data_block / FIL / DSE      A/syntax/SyntacticElements.java:57-203, DSE.java:37-48
 *   CPE / ics_info                  A/syntax/CPE.java:85-123, ICSInfo.java:86-119
 *   section data / scalefactors     A/syntax/ICStream.java:113-146, 172-220
 *   pulse / TNS / gain control      A/syntax/ICStream.java:76-98,148-170, A/tools/TNS.java:35-61
 *   spectral data + escapes         A/syntax/ICStream.java:222-275, A/huffman/Huffman.java:30-84
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/jaad_gpu.h"
#include "../jaadec_amd/csrc/tables/jaad_huffman_tables.inc"
#include "../jaadec_amd/csrc/tables/jaad_tables.inc"

typedef struct {
    uint8_t* d;
    size_t cap, pos; /* bits */
    int overflow;
} Bw;

static void put(Bw* w, uint32_t v, int n)
{
    for (int i = n - 1; i >= 0; i--) {
        if (w->pos >= 8 * w->cap) {
            w->overflow = 1;
            return;
        }
        const uint32_t b = (v >> i) & 1u;
        if (b) w->d[w->pos >> 3] |= (uint8_t)(0x80u >> (w->pos & 7));
        w->pos++;
    }
}
static void align(Bw* w)
{
    while (w->pos & 7) put(w, 0, 1);
}

/* row of codebook cb (1..11) holding value tuple v, or -1 */
static int find_row(int cb, const int* v)
{
    static const int n[11] = {81, 81, 81, 81, 81, 81, 64, 64, 169, 169, 289};
    const int* rows[11] = {&JAAD_HCB1[0][0], &JAAD_HCB2[0][0], &JAAD_HCB3[0][0], &JAAD_HCB4[0][0], &JAAD_HCB5[0][0],
                           &JAAD_HCB6[0][0], &JAAD_HCB7[0][0], &JAAD_HCB8[0][0], &JAAD_HCB9[0][0], &JAAD_HCB10[0][0],
                           &JAAD_HCB11[0][0]};
    const int stride = cb < 5 ? 6 : 4, num = cb < 5 ? 4 : 2;
    for (int r = 0; r < n[cb - 1]; r++) {
        const int* row = rows[cb - 1] + r * stride;
        int ok = 1;
        for (int j = 0; j < num; j++) ok &= row[2 + j] == v[j];
        if (ok) return r;
    }
    return -1;
}
static void put_row(Bw* w, int cb, int r)
{
    const int* rows[11] = {&JAAD_HCB1[0][0], &JAAD_HCB2[0][0], &JAAD_HCB3[0][0], &JAAD_HCB4[0][0], &JAAD_HCB5[0][0],
                           &JAAD_HCB6[0][0], &JAAD_HCB7[0][0], &JAAD_HCB8[0][0], &JAAD_HCB9[0][0], &JAAD_HCB10[0][0],
                           &JAAD_HCB11[0][0]};
    const int* row = rows[cb - 1] + r * (cb < 5 ? 6 : 4);
    put(w, (uint32_t)row[1], row[0]);
}
static int put_sf_delta(Bw* w, int d)
{
    if (d < -60 || d > 60) return -1;
    for (int r = 0; r < 121; r++)
        if (JAAD_HCB_SF[r][2] == d + 60) {
            put(w, (uint32_t)JAAD_HCB_SF[r][1], JAAD_HCB_SF[r][0]);
            return 0;
        }
    return -1;
}

typedef struct {
    int seq, shape, max_sfb, grouping, ngroups, glen[8];
} Info;

static void info_of(const jaad_ics_info* ic, Info* I)
{
    I->seq = ic->window_sequence;
    I->shape = ic->window_shape;
    I->max_sfb = ic->max_sfb;
    I->grouping = ic->grouping;
    I->ngroups = 1;
    I->glen[0] = 1;
    if (I->seq == JAAD_EIGHT_SHORT_SEQUENCE)
        for (int i = 0; i < 7; i++) {
            if (I->grouping & (1 << i)) I->glen[I->ngroups - 1]++;
            else I->glen[I->ngroups++] = 1;
        }
}

static void put_ics_info(Bw* w, const Info* I)
{
    put(w, 0, 1);
    put(w, (uint32_t)I->seq, 2);
    put(w, (uint32_t)I->shape, 1);
    if (I->seq == JAAD_EIGHT_SHORT_SEQUENCE) {
        put(w, (uint32_t)I->max_sfb, 4);
        for (int i = 0; i < 7; i++) put(w, (I->grouping >> i) & 1, 1);
    } else {
        put(w, (uint32_t)I->max_sfb, 6);
        put(w, 0, 1); /* predictor_data_present */
    }
}

/* individual_channel_stream; returns 0 or -1 (records not representable) */
static int put_ics(Bw* w, int sf_index, int common, const int16_t* q, const uint8_t* sf, const uint8_t* cb,
                   const jaad_ics_info* ic, const jaad_tns* tns, int pulse)
{
    Info I;
    info_of(ic, &I);
    const int is_short = I.seq == JAAD_EIGHT_SHORT_SEQUENCE;
    const short* swb = is_short ? JAAD_SWB_OFFSET_SHORT_WINDOW[sf_index] : JAAD_SWB_OFFSET_LONG_WINDOW[sf_index];
    const int nb = I.ngroups * I.max_sfb;
    /* global_gain: the first spectral band's scalefactor (100 when there is none) */
    int gg = 100;
    for (int i = 0; i < nb; i++)
        if (cb[i] && cb[i] < JAAD_NOISE_HCB) {
            gg = sf[i];
            break;
        }
    put(w, (uint32_t)gg, 8);
    if (!common) put_ics_info(w, &I);
    /* section data: maximal runs of one codebook inside a group */
    const int bits = is_short ? 3 : 5, esc = (1 << bits) - 1;
    for (int g = 0; g < I.ngroups; g++) {
        for (int k = 0; k < I.max_sfb;) {
            const int c = cb[g * I.max_sfb + k];
            int e = k;
            while (e < I.max_sfb && cb[g * I.max_sfb + e] == c) e++;
            put(w, (uint32_t)c, 4);
            int len = e - k;
            while (len >= esc) {
                put(w, (uint32_t)esc, bits);
                len -= esc;
            }
            put(w, (uint32_t)len, bits);
            k = e;
        }
    }
    /* scalefactors */
    int off0 = gg, off1 = gg - 90, off2 = 0, first_noise = 1;
    for (int i = 0; i < nb; i++) {
        const int c = cb[i];
        if (c == JAAD_ZERO_HCB) continue;
        if (c == JAAD_INTENSITY_HCB || c == JAAD_INTENSITY_HCB2) {
            const int t = 100 - sf[i];
            if (put_sf_delta(w, t - off2)) return -1;
            off2 = t;
        } else if (c == JAAD_NOISE_HCB) {
            const int t = sf[i] - 100;
            if (first_noise) {
                const int v = t - off1 + 256;
                if (v < 0 || v > 511) return -1;
                put(w, (uint32_t)v, 9);
                first_noise = 0;
            } else if (put_sf_delta(w, t - off1)) {
                return -1;
            }
            off1 = t;
        } else {
            if (put_sf_delta(w, sf[i] - off0)) return -1;
            off0 = sf[i];
        }
    }
    /* pulse data (parsed and dropped by the reference): optional, long windows only */
    if (pulse && !is_short && I.max_sfb > 0) {
        put(w, 1, 1);
        put(w, 1, 2);         /* 2 pulses */
        put(w, 0, 6);         /* start swb 0 */
        put(w, 3, 5);
        put(w, 5, 4);
        put(w, 7, 5);
        put(w, 2, 4);
    } else {
        put(w, 0, 1);
    }
    /* TNS */
    const int tp = (ic->flags & JAAD_ICS_TNS) && tns;
    put(w, (uint32_t)tp, 1);
    if (tp) {
        const int nwin = is_short ? 8 : 1;
        const int b0 = is_short ? 1 : 2, b1 = is_short ? 4 : 6, b2 = is_short ? 3 : 5;
        for (int win = 0; win < nwin; win++) {
            int nf = 0, first = -1;
            for (int f = 0; f < tns->n_filters; f++)
                if (tns->filt[f].window == win) {
                    if (first < 0) first = f;
                    nf++;
                }
            put(w, (uint32_t)nf, b0);
            if (!nf) continue;
            const int res = (tns->filt[first].flags >> 1) & 1;
            put(w, (uint32_t)res, 1);
            for (int f = 0; f < tns->n_filters; f++) {
                const jaad_tns_filter* F = &tns->filt[f];
                if (F->window != win) continue;
                put(w, F->length, b1);
                put(w, F->order, b2);
                if (F->order) {
                    const int comp = (F->flags >> 2) & 1;
                    put(w, F->flags & 1, 1);
                    put(w, (uint32_t)comp, 1);
                    for (int i = 0; i < F->order; i++) put(w, F->coef[i], res + 3 - comp);
                }
            }
        }
    }
    put(w, 0, 1); /* gain_control_data_present */
    /* spectral data */
    for (int g = 0, idx = 0, goff = 0; g < I.ngroups; g++) {
        for (int s = 0; s < I.max_sfb; s++, idx++) {
            const int c = cb[idx];
            if (c == JAAD_ZERO_HCB || c >= JAAD_NOISE_HCB) continue;
            const int width = swb[s + 1] - swb[s];
            const int num = c >= JAAD_FIRST_PAIR_HCB ? 2 : 4;
            const int uns = c == 3 || c == 4 || c >= 7;
            for (int win = 0; win < I.glen[g]; win++) {
                const int off = goff + win * 128 + swb[s];
                for (int k = 0; k < width; k += num) {
                    int v[4] = {0, 0, 0, 0}, key[4] = {0, 0, 0, 0};
                    for (int j = 0; j < num; j++) {
                        v[j] = q[off + k + j];
                        int a = uns ? abs(v[j]) : v[j];
                        if (c == JAAD_ESCAPE_HCB && a >= 16) a = 16;
                        key[j] = a;
                    }
                    const int r = find_row(c, key);
                    if (r < 0) return -1;
                    put_row(w, c, r);
                    if (uns)
                        for (int j = 0; j < num; j++)
                            if (v[j]) put(w, v[j] < 0, 1);
                    if (c == JAAD_ESCAPE_HCB)
                        for (int j = 0; j < 2; j++) {
                            const int a = abs(v[j]);
                            if (a < 16) continue;
                            int n = 4;
                            while ((a >> (n + 1)) != 0) n++;
                            for (int i = 4; i < n; i++) put(w, 1, 1);
                            put(w, 0, 1);
                            put(w, (uint32_t)(a & ((1 << n) - 1)), n);
                        }
                }
            }
        }
        goff += I.glen[g] << 7;
    }
    return 0;
}

long jaad_sbr_fil_bits(void* state, int nch, const jaad_sbr_frame* rec, uint8_t* out, size_t cap);

/* one channel element: id 0 SCE / 3 LFE (one ICS) or 1 CPE (A/syntax/CPE.java:85-123), instance tag */
static int put_element(Bw* w, int sf_index, int id, int tag, const int16_t* q, const uint8_t* sf, const uint8_t* cb,
                       const jaad_ics_info* ics, const uint64_t* ms_used, const jaad_tns* tns, int extras)
{
    put(w, (uint32_t)id, 3);
    put(w, (uint32_t)tag, 4);
    if (id != 1) return put_ics(w, sf_index, 0, q, sf, cb, ics, tns, extras & 2);
    const int common = (ics[0].flags & JAAD_ICS_COMMON_WINDOW) != 0;
    put(w, (uint32_t)common, 1);
    if (common) {
        Info I;
        info_of(&ics[0], &I);
        put_ics_info(w, &I);
        const int nb = I.ngroups * I.max_sfb;
        if (ics[0].flags & JAAD_ICS_MS_PRESENT) {
            int all = 1;
            for (int i = 0; i < nb; i++) all &= (int)((ms_used[i >> 6] >> (i & 63)) & 1);
            if (all && nb) {
                put(w, 2, 2);
            } else {
                put(w, 1, 2);
                for (int i = 0; i < nb; i++) put(w, (uint32_t)((ms_used[i >> 6] >> (i & 63)) & 1), 1);
            }
        } else {
            put(w, 0, 2);
        }
    }
    if (put_ics(w, sf_index, common, q, sf, cb, &ics[0], tns, extras & 2)) return -1;
    return put_ics(w, sf_index, common, q + 1024, sf + 128, cb + 128, &ics[1], tns ? tns + 1 : NULL, extras & 2);
}

/*
 * One raw_data_block of a multichannel frame: the elements ids[0..n_elem) (0 SCE, 1 CPE, 3 LFE)
 * in order over the frame's channel records (q/sf/cb/ics/tns: all channels, element k starting
 * at the channels before it; ms_used: one pair per CPE), then END.
 */
long jaad_write_frame_mc(int sf_index, int n_elem, const int* ids, const int16_t* q, const uint8_t* sf,
                         const uint8_t* cb, const jaad_ics_info* ics, const uint64_t* ms_used, const jaad_tns* tns,
                         uint8_t* out, size_t cap)
{
    Bw w = {out, cap, 0, 0};
    memset(out, 0, cap);
    int ch = 0, cpe = 0, tags[8] = {0};
    for (int k = 0; k < n_elem; k++) {
        const int id = ids[k];
        if (put_element(&w, sf_index, id, tags[id]++, q + (size_t)ch * 1024, sf + ch * 128, cb + ch * 128, ics + ch,
                        id == 1 ? ms_used + 2 * cpe : NULL, tns ? tns + ch : NULL, 0))
            return -1;
        ch += id == 1 ? 2 : 1;
        cpe += id == 1;
    }
    put(&w, 7, 3); /* END */
    align(&w);
    return w.overflow ? -1 : (long)(w.pos / 8);
}

/*
 * A raw_data_block of a multichannel HE-AAC frame: as jaad_write_frame_mc, with element k's SBR
 * record sbr[k] written as a FIL (EXT_SBR_DATA) right after the element when its status is
 * JAAD_SBR_OK and sbr_state[k] (that element's writer state) is set.
 */
long jaad_write_frame_mc_sbr(int sf_index, int n_elem, const int* ids, const int16_t* q, const uint8_t* sf,
                             const uint8_t* cb, const jaad_ics_info* ics, const uint64_t* ms_used, const jaad_tns* tns,
                             const jaad_sbr_frame* sbr, void* const* sbr_state, uint8_t* out, size_t cap)
{
    Bw w = {out, cap, 0, 0};
    memset(out, 0, cap);
    int ch = 0, cpe = 0, tags[8] = {0};
    for (int k = 0; k < n_elem; k++) {
        const int id = ids[k];
        if (put_element(&w, sf_index, id, tags[id]++, q + (size_t)ch * 1024, sf + ch * 128, cb + ch * 128, ics + ch,
                        id == 1 ? ms_used + 2 * cpe : NULL, tns ? tns + ch : NULL, 0))
            return -1;
        if (sbr && sbr_state && sbr_state[k] && sbr[k].status == JAAD_SBR_OK) {
            uint8_t fil[512];
            const long nbits = jaad_sbr_fil_bits(sbr_state[k], id == 1 ? 2 : 1, &sbr[k], fil, sizeof fil);
            if (nbits < 0) return -1;
            for (long i = 0; i < nbits; i++) put(&w, (fil[i >> 3] >> (7 - (i & 7))) & 1u, 1);
        }
        ch += id == 1 ? 2 : 1;
        cpe += id == 1;
    }
    put(&w, 7, 3); /* END */
    align(&w);
    return w.overflow ? -1 : (long)(w.pos / 8);
}

/*
 * coupling_channel_element (the syntax CCE.decode reads, A/syntax/CCE.java:112-175) of a test
 * description: targets, coupling domain, gain sign/scale, the CCE's ICStream records and its gain
 * element codes.  gain list i (i >= 1): cge[i] = common_gain_element_present; with it, code[i][0]
 * is the common gain (-60..60); without it code[i][idx] is the per-band dpcm value for every band
 * idx whose cb != ZERO_HCB.
 */
typedef struct jaad_cce_desc {
    uint8_t ind_sw, count, domain, sign, scale;  /* count = num_coupled_elements (0..7)          */
    uint8_t pair[8], id[8], chs[8];               /* chs[i] (cc_l/cc_r as 2 bits) when pair[i]  */
    uint8_t pos;                                  /* written before channel element `pos`        */
    uint8_t cge[16];
    int8_t code[16][120];
} jaad_cce_desc;

static int put_cce(Bw* w, int sf_index, int tag, const jaad_cce_desc* d, const int16_t* q, const uint8_t* sf,
                   const uint8_t* cb, const jaad_ics_info* ic)
{
    put(w, 2, 3);
    put(w, (uint32_t)tag, 4);
    put(w, d->ind_sw, 1);
    put(w, d->count, 3);
    int gain_count = 0;
    for (int i = 0; i <= d->count; i++) {
        gain_count++;
        put(w, d->pair[i], 1);
        put(w, d->id[i], 4);
        if (d->pair[i]) {
            put(w, d->chs[i], 2);
            if (d->chs[i] == 3) gain_count++;
        }
    }
    put(w, d->domain, 1);
    put(w, d->sign, 1);
    put(w, d->scale, 2);
    if (put_ics(w, sf_index, 0, q, sf, cb, ic, NULL, 0)) return -1;
    int point = 2 * d->ind_sw + d->domain;
    point |= point >> 1;
    Info I;
    info_of(ic, &I);
    for (int i = 1; i < gain_count; i++) {
        const int cge = point == 2 ? 1 : d->cge[i];
        if (point != 2) put(w, (uint32_t)cge, 1);
        if (cge) {
            if (put_sf_delta(w, d->code[i][0])) return -1;
            continue;
        }
        for (int idx = 0; idx < I.ngroups * I.max_sfb; idx++)
            if (cb[idx] != JAAD_ZERO_HCB && put_sf_delta(w, d->code[i][idx])) return -1;
    }
    return 0;
}

/*
 * A raw_data_block of channel elements ids[0..n_elem) (as jaad_write_frame_mc) with n_cce coupling
 * channel elements (records cq/csf/ccb/cics, descriptions d) inserted before their d[k].pos-th
 * channel element (pos = n_elem: after the last), then END.
 */
long jaad_write_frame_cce_sbr(int sf_index, int n_elem, const int* ids, const int16_t* q, const uint8_t* sf,
                              const uint8_t* cb, const jaad_ics_info* ics, const uint64_t* ms_used, int n_cce,
                              const jaad_cce_desc* d, const int16_t* cq, const uint8_t* csf, const uint8_t* ccb,
                              const jaad_ics_info* cics, const jaad_sbr_frame* sbr, void* const* sbr_state,
                              uint8_t* out, size_t cap);

long jaad_write_frame_cce(int sf_index, int n_elem, const int* ids, const int16_t* q, const uint8_t* sf,
                          const uint8_t* cb, const jaad_ics_info* ics, const uint64_t* ms_used, int n_cce,
                          const jaad_cce_desc* d, const int16_t* cq, const uint8_t* csf, const uint8_t* ccb,
                          const jaad_ics_info* cics, uint8_t* out, size_t cap)
{
    return jaad_write_frame_cce_sbr(sf_index, n_elem, ids, q, sf, cb, ics, ms_used, n_cce, d, cq, csf, ccb, cics, NULL,
                                    NULL, out, cap);
}

/* as jaad_write_frame_cce, with element k's SBR record sbr[k] as a FIL right after the element
 * (when sbr_state[k] is set and the record's status is JAAD_SBR_OK) */
long jaad_write_frame_cce_sbr(int sf_index, int n_elem, const int* ids, const int16_t* q, const uint8_t* sf,
                              const uint8_t* cb, const jaad_ics_info* ics, const uint64_t* ms_used, int n_cce,
                              const jaad_cce_desc* d, const int16_t* cq, const uint8_t* csf, const uint8_t* ccb,
                              const jaad_ics_info* cics, const jaad_sbr_frame* sbr, void* const* sbr_state,
                              uint8_t* out, size_t cap)
{
    Bw w = {out, cap, 0, 0};
    memset(out, 0, cap);
    int ch = 0, cpe = 0, tags[8] = {0};
    for (int k = 0; k <= n_elem; k++) {
        for (int j = 0; j < n_cce; j++)
            if (d[j].pos == k &&
                put_cce(&w, sf_index, j, &d[j], cq + (size_t)j * 1024, csf + j * 128, ccb + j * 128, cics + j))
                return -1;
        if (k == n_elem) break;
        const int id = ids[k];
        if (put_element(&w, sf_index, id, tags[id]++, q + (size_t)ch * 1024, sf + ch * 128, cb + ch * 128, ics + ch,
                        id == 1 ? ms_used + 2 * cpe : NULL, NULL, 0))
            return -1;
        if (sbr && sbr_state && sbr_state[k] && sbr[k].status == JAAD_SBR_OK) {
            uint8_t fil[512];
            const long nbits = jaad_sbr_fil_bits(sbr_state[k], id == 1 ? 2 : 1, &sbr[k], fil, sizeof fil);
            if (nbits < 0) return -1;
            for (long i = 0; i < nbits; i++) put(&w, (fil[i >> 3] >> (7 - (i & 7))) & 1u, 1);
        }
        ch += id == 1 ? 2 : 1;
        cpe += id == 1;
    }
    put(&w, 7, 3); /* END */
    align(&w);
    return w.overflow ? -1 : (long)(w.pos / 8);
}

/*
 * One raw_data_block of the frame's records (nch = 1: SCE, 2: CPE), optionally wrapped in
 * extra DSE / FIL(fill) elements (extras bit 0) and carrying pulse data (bit 1); with `sbr`
 * (and the stream's writer state, jaad_writer_sbr.c) the SBR record follows the channel
 * element as a FIL element.  Returns the byte count, or -1 when a record cannot be
 * represented / cap is too small.
 */
long jaad_write_frame_sbr(int sf_index, int nch, const int16_t* q, const uint8_t* sf, const uint8_t* cb,
                          const jaad_ics_info* ics, const uint64_t* ms_used, const jaad_tns* tns, int extras,
                          const jaad_sbr_frame* sbr, void* sbr_state, uint8_t* out, size_t cap)
{
    Bw w = {out, cap, 0, 0};
    memset(out, 0, cap);
    if (extras & 1) { /* DSE with 3 bytes, byte aligned */
        put(&w, 4, 3);
        put(&w, 5, 4);
        put(&w, 1, 1);
        put(&w, 3, 8);
        align(&w);
        put(&w, 0xABCDEF, 24);
    }
    if (put_element(&w, sf_index, nch == 1 ? 0 : 1, 0, q, sf, cb, ics, ms_used, tns, extras)) return -1;
    if (sbr) {
        uint8_t fil[512];
        const long nbits = jaad_sbr_fil_bits(sbr_state, nch, sbr, fil, sizeof fil);
        if (nbits < 0) return -1;
        for (long i = 0; i < nbits; i++) put(&w, (fil[i >> 3] >> (7 - (i & 7))) & 1u, 1);
    }
    if (extras & 1) { /* FIL element: 2 bytes of EXT_FILL_DATA */
        put(&w, 6, 3);
        put(&w, 2, 4);
        put(&w, 1, 4);
        put(&w, 0xA5A, 12);
    }
    put(&w, 7, 3); /* END */
    align(&w);
    return w.overflow ? -1 : (long)(w.pos / 8);
}

long jaad_write_frame(int sf_index, int nch, const int16_t* q, const uint8_t* sf, const uint8_t* cb,
                      const jaad_ics_info* ics, const uint64_t* ms_used, const jaad_tns* tns, int extras,
                      uint8_t* out, size_t cap)
{
    return jaad_write_frame_sbr(sf_index, nch, q, sf, cb, ics, ms_used, tns, extras, NULL, NULL, out, cap);
}

/* ADTS header (S/adts/ADTSFrame.java:48-111) for a payload of `payload` bytes, no CRC */
int jaad_write_adts_header(int sf_index, int channel_config, size_t payload, uint8_t* out)
{
    const size_t len = payload + 7;
    if (len >= (1u << 13)) return -1;
    out[0] = 0xFF;
    out[1] = 0xF1; /* sync low bits, MPEG-4, layer 0, protection_absent */
    out[2] = (uint8_t)((1 << 6) | (sf_index << 2) | ((channel_config >> 2) & 1)); /* profile LC (1) */
    out[3] = (uint8_t)(((channel_config & 3) << 6) | ((len >> 11) & 3));
    out[4] = (uint8_t)((len >> 3) & 0xFF);
    out[5] = (uint8_t)(((len & 7) << 5) | 0x1F); /* buffer fullness 0x7FF (VBR) */
    out[6] = 0xFC;                                /* fullness low bits, 1 raw data block */
    return 7;
}
