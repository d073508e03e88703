/*
 * TEST INFRASTRUCTURE ONLY (never linked into the product): the SBR / PS part of the test
 * bitstream WRITER (jaad_writer.c).  It writes a jaad_sbr_frame record as the
 * sbr_extension_data of a FIL element in the syntax the reference reads, so that the host
 * parser's SBR/PS path (jaadec_amd/csrc/jaad_parse_sbr.cpp) is pinned by round trips:
 *   FIL / EXT_SBR_DATA(_CRC)           A/syntax/SyntacticElements.java:169-214
 *   SBR.decode / Header.decode         A/sbr/SBR.java:161-245, A/sbr/Header.java:24-62
 *   sbr_data SCE / CPE                 A/sbr/SBR1.java:34-60, A/sbr/SBR2.java:35-135
 *   grid / dtdf / invf / envelope /    A/sbr/Channel.java:85-583
 *     noise (+ delta decoding)
 *   ps_data + its Huffman trees        A/ps/PSImpl.java:103-134, A/ps/Envelope.java, A/ps/Huffman.java
 * Which of the equivalent codings is used (frequency or time deltas, CRC, explicit header
 * defaults, header repetition of PS) is drawn from a seeded generator, so a stream exercises
 * all of them.  Band counts come from the oracle's restatement of calc_sbr_tables
 * (orc_sbr_res_tables in jaad_oracle_sbr.c).
 */
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include "../include/jaad_gpu.h"
#include "../jaadec_amd/csrc/tables/jaad_huffman_tables.inc"

int orc_sbr_res_tables(const jaad_sbr_header* h, int out_sf_index, int* info, int* ftr);

typedef struct {
    uint8_t* d;
    size_t cap, pos;
    int overflow;
} Sw;

static void sput(Sw* w, uint32_t v, int n)
{
    for (int i = n - 1; i >= 0; i--) {
        if (w->pos >= 8 * w->cap) {
            w->overflow = 1;
            return;
        }
        if ((v >> i) & 1u) w->d[w->pos >> 3] |= (uint8_t)(0x80u >> (w->pos & 7));
        w->pos++;
    }
}

/* codeword of value (leaf = value - bias) in a binary tree; 0 or -1 (not encodable) */
static int tree_find(const int (*t)[2], int nn, int node, int leaf, uint32_t acc, int depth, uint32_t* code, int* len)
{
    if (node >= nn || depth > 30) return -1;
    for (int b = 0; b < 2; b++) {
        const int nx = t[node][b];
        const uint32_t a = (acc << 1) | (uint32_t)b;
        if (nx < 0) {
            if (nx == leaf) {
                *code = a;
                *len = depth + 1;
                return 0;
            }
        } else if (!tree_find(t, nn, nx, leaf, a, depth + 1, code, len)) {
            return 0;
        }
    }
    return -1;
}
static int put_tree(Sw* w, const int (*t)[2], int nn, int bias, int value)
{
    uint32_t code;
    int len;
    if (tree_find(t, nn, 0, value - bias, 0, 0, &code, &len)) return -1;
    sput(w, code, len);
    return 0;
}
/* JAAD_WRITER_DEBUG=1: name the line a record is refused at */
static int fail_at(int line)
{
    if (getenv("JAAD_WRITER_DEBUG")) fprintf(stderr, "jaad_writer_sbr: record refused at line %d\n", line);
    return -1;
}
#define FAIL fail_at(__LINE__)
#define NN(tab) (int)(sizeof(tab) / sizeof((tab)[0]))

typedef struct {
    uint64_t rng;
    int out_sf;
    int have_hdr;
    jaad_sbr_header hdr;
    int n[2], N_Q, N_high, N_low, ftr[2][64];
    int tables_gen; /* bumped on each table reset */
    int prev_gen[2], have_prev[2];
    int E_prev[2][64], Q_prev[2][64], f_prev[2];
    /* what the reader's Channel keeps between frames: L_E / L_Q (a coupled channel 1 reads its
     * dtdf bits with the previous frame's counts, A/sbr/SBR2.java:48-50) and bs_df_env /
     * bs_df_noise (entries past those counts stay as an earlier frame left them) */
    int L_E_last[2], L_Q_last[2], df_env[2][9], df_noise[2][3];
    int ps_have_hdr, ps_iid_mode, ps_icc_mode;
    int ps_first_iid[34], ps_first_icc[34];
} jaad_sbr_wstate;

size_t jaad_sbr_wstate_size(void) { return sizeof(jaad_sbr_wstate); }
void jaad_sbr_wstate_init(void* p, int out_sf_index, uint64_t seed)
{
    jaad_sbr_wstate* s = (jaad_sbr_wstate*)p;
    memset(s, 0, sizeof *s);
    s->out_sf = out_sf_index;
    s->rng = seed * 0x9E3779B97F4A7C15ull + 0x1234567ull;
}
static uint32_t rnd(jaad_sbr_wstate* s, uint32_t n)
{
    s->rng ^= s->rng << 13;
    s->rng ^= s->rng >> 7;
    s->rng ^= s->rng << 17;
    return (uint32_t)(s->rng >> 11) % n;
}

static int hdr_differs(const jaad_sbr_header* a, const jaad_sbr_header* b)
{
    return a->start_freq != b->start_freq || a->stop_freq != b->stop_freq || a->freq_scale != b->freq_scale ||
           a->alter_scale != b->alter_scale || a->xover_band != b->xover_band || a->noise_bands != b->noise_bands;
}

static void put_header(Sw* w, jaad_sbr_wstate* s, const jaad_sbr_header* h)
{
    sput(w, h->amp_res, 1);
    sput(w, h->start_freq, 4);
    sput(w, h->stop_freq, 4);
    sput(w, h->xover_band, 3);
    sput(w, 0, 2);
    const int x1 = !(h->freq_scale == 2 && h->alter_scale == 1 && h->noise_bands == 2) || rnd(s, 2);
    const int x2 = !(h->limiter_bands == 2 && h->limiter_gains == 2 && h->interpol_freq == 1 && h->smoothing_mode == 1) ||
                   rnd(s, 2);
    sput(w, (uint32_t)x1, 1);
    sput(w, (uint32_t)x2, 1);
    if (x1) {
        sput(w, h->freq_scale, 2);
        sput(w, h->alter_scale, 1);
        sput(w, h->noise_bands, 2);
    }
    if (x2) {
        sput(w, h->limiter_bands, 2);
        sput(w, h->limiter_gains, 2);
        sput(w, h->interpol_freq, 1);
        sput(w, h->smoothing_mode, 1);
    }
}

/* sbr_grid from the record's class, borders and pointer (inverse of Channel.sbr_grid) */
static int put_grid(Sw* w, const jaad_sbr_channel* c)
{
    const int L_E = c->L_E;
    sput(w, c->frame_class, 2);
    switch (c->frame_class) {
    case 0: { /* FIXFIX: 1, 2 or 4 envelopes of one resolution */
        const int i = L_E == 1 ? 0 : (L_E == 2 ? 1 : (L_E == 4 ? 2 : -1));
        if (i < 0) return FAIL;
        sput(w, (uint32_t)i, 2);
        sput(w, c->f[0], 1);
        return 0;
    }
    case 1:   /* FIXVAR */
    case 2: { /* VARFIX */
        static const int lg[10] = {0, 0, 1, 2, 2, 3, 3, 3, 3, 4};
        if (L_E < 1 || L_E > 4) return FAIL;
        const int fixvar = c->frame_class == 1;
        const int ab = fixvar ? c->t_E[L_E] / 2 - 16 : c->t_E[0] / 2;
        if (ab < 0 || ab > 3) return FAIL;
        sput(w, (uint32_t)ab, 2);
        sput(w, (uint32_t)(L_E - 1), 2);
        for (int r = 0; r < L_E - 1; r++) {
            const int d = fixvar ? (c->t_E[L_E - r] - c->t_E[L_E - r - 1]) / 2 : (c->t_E[r + 1] - c->t_E[r]) / 2;
            if (d < 2 || d > 8 || (d & 1)) return FAIL;
            sput(w, (uint32_t)((d - 2) / 2), 2);
        }
        sput(w, c->bs_pointer, lg[L_E + 1]);
        for (int e = 0; e < L_E; e++) sput(w, fixvar ? c->f[L_E - e - 1] : c->f[e], 1);
        return 0;
    }
    default: { /* VARVAR, all relative borders from the leading side */
        static const int lg[10] = {0, 0, 1, 2, 2, 3, 3, 3, 3, 4};
        if (L_E < 1 || L_E > 4) return FAIL;
        const int lead = c->t_E[0] / 2, trail = c->t_E[L_E] / 2 - 16;
        if (lead < 0 || lead > 3 || trail < 0 || trail > 3) return FAIL;
        sput(w, (uint32_t)lead, 2);
        sput(w, (uint32_t)trail, 2);
        sput(w, (uint32_t)(L_E - 1), 2);
        sput(w, 0, 2);
        for (int r = 0; r < L_E - 1; r++) {
            const int d = (c->t_E[r + 1] - c->t_E[r]) / 2;
            if (d < 2 || d > 8 || (d & 1)) return FAIL;
            sput(w, (uint32_t)((d - 2) / 2), 2);
        }
        sput(w, c->bs_pointer, lg[L_E + 1]);
        for (int e = 0; e < L_E; e++) sput(w, c->f[e], 1);
        return 0;
    }
    }
}

/* previous-envelope value the time-delta decoding adds to band k of envelope l
 * (Channel.extract_envelope_data, A/sbr/Channel.java:203-240) */
static int env_prev_value(const jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, int l, int k)
{
    const int g = l == 0 ? s->f_prev[ch] : c->f[l - 1], f = c->f[l];
    const int16_t* pe = l == 0 ? NULL : c->E[l - 1];
    int i = k;
    if (g == 1 && f == 0) {
        for (i = 0; i < s->N_high; i++)
            if (s->ftr[1][i] == s->ftr[0][k]) break;
    } else if (g == 0 && f == 1) {
        for (i = 0; i < s->N_low; i++)
            if (s->ftr[0][i] <= s->ftr[1][k] && s->ftr[1][k] < s->ftr[0][i + 1]) break;
    }
    return pe ? pe[i] : s->E_prev[ch][i];
}

static int put_envelope(Sw* w, jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, const int* df)
{
    const int amp_res = (c->L_E == 1 && c->frame_class == 0) ? 0 : s->hdr.amp_res;
    const int(*th)[2] = amp_res ? JAAD_SBR_T_HUFFMAN_ENV_3_0DB : JAAD_SBR_T_HUFFMAN_ENV_1_5DB;
    const int(*fh)[2] = amp_res ? JAAD_SBR_F_HUFFMAN_ENV_3_0DB : JAAD_SBR_F_HUFFMAN_ENV_1_5DB;
    const int tn = amp_res ? NN(JAAD_SBR_T_HUFFMAN_ENV_3_0DB) : NN(JAAD_SBR_T_HUFFMAN_ENV_1_5DB);
    const int fn = amp_res ? NN(JAAD_SBR_F_HUFFMAN_ENV_3_0DB) : NN(JAAD_SBR_F_HUFFMAN_ENV_1_5DB);
    for (int l = 0; l < c->L_E; l++) {
        const int nb = s->n[c->f[l] & 1];
        if (!df[l]) {
            const int bits = amp_res ? 6 : 7;
            if (c->E[l][0] < 0 || c->E[l][0] >= (1 << bits)) return FAIL;
            sput(w, (uint32_t)c->E[l][0], bits);
            for (int k = 1; k < nb; k++)
                if (put_tree(w, fh, fn, 64, c->E[l][k] - c->E[l][k - 1])) return FAIL;
        } else {
            for (int k = 0; k < nb; k++)
                if (put_tree(w, th, tn, 64, c->E[l][k] - env_prev_value(s, ch, c, l, k))) return FAIL;
        }
    }
    return 0;
}

static int put_noise(Sw* w, jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, const int* df)
{
    for (int l = 0; l < c->L_Q; l++) {
        if (!df[l]) {
            if (c->Q[l][0] < 0 || c->Q[l][0] > 31) return FAIL;
            sput(w, (uint32_t)c->Q[l][0], 5);
            for (int k = 1; k < s->N_Q; k++)
                if (put_tree(w, JAAD_SBR_F_HUFFMAN_ENV_3_0DB, NN(JAAD_SBR_F_HUFFMAN_ENV_3_0DB), 64, c->Q[l][k] - c->Q[l][k - 1]))
                    return FAIL;
        } else {
            for (int k = 0; k < s->N_Q; k++) {
                const int p = l == 0 ? s->Q_prev[ch][k] : c->Q[l - 1][k];
                if (put_tree(w, JAAD_SBR_T_HUFFMAN_NOISE_3_0DB, NN(JAAD_SBR_T_HUFFMAN_NOISE_3_0DB), 64, c->Q[l][k] - p))
                    return FAIL;
            }
        }
    }
    return 0;
}

/* can envelope l (noise envelope l) of an uncoupled channel be time-delta coded: every delta in
 * the time tree (T_HUFFMAN_ENV_*, T_HUFFMAN_NOISE_3_0DB) */
static int env_time_ok(const jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, int l)
{
    const int amp_res = (c->L_E == 1 && c->frame_class == 0) ? 0 : s->hdr.amp_res;
    const int(*th)[2] = amp_res ? JAAD_SBR_T_HUFFMAN_ENV_3_0DB : JAAD_SBR_T_HUFFMAN_ENV_1_5DB;
    const int tn = amp_res ? NN(JAAD_SBR_T_HUFFMAN_ENV_3_0DB) : NN(JAAD_SBR_T_HUFFMAN_ENV_1_5DB);
    uint32_t code;
    int len;
    for (int k = 0; k < s->n[c->f[l] & 1]; k++)
        if (tree_find(th, tn, 0, c->E[l][k] - env_prev_value(s, ch, c, l, k) - 64, 0, 0, &code, &len)) return 0;
    return 1;
}
static int noise_time_ok(const jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, int l)
{
    uint32_t code;
    int len;
    for (int k = 0; k < s->N_Q; k++) {
        const int p = l == 0 ? s->Q_prev[ch][k] : c->Q[l - 1][k];
        if (tree_find(JAAD_SBR_T_HUFFMAN_NOISE_3_0DB, NN(JAAD_SBR_T_HUFFMAN_NOISE_3_0DB), 0, c->Q[l][k] - p - 64, 0, 0,
                      &code, &len))
            return 0;
    }
    return 1;
}

/* coded value of band k of envelope l of a coupled channel 1 (sbr_envelope with coupled = true:
 * BAL tables, values transmitted >> 1, A/sbr/Channel.java:125-198); -1 when not codable */
static int bal_env_ok(const jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, int l, int df)
{
    const int amp_res = (c->L_E == 1 && c->frame_class == 0) ? 0 : s->hdr.amp_res;
    const int nb = s->n[c->f[l] & 1], range = amp_res ? 12 : 24;
    for (int k = 0; k < nb; k++) {
        const int v = c->E[l][k];
        const int base = df ? env_prev_value(s, ch, c, l, k) : (k ? c->E[l][k - 1] : 0);
        const int d = v - base;
        if (v < 0 || (d & 1)) return 0;
        if (!df && k == 0) {
            if ((v >> 1) >= (1 << (amp_res ? 5 : 6))) return 0;
        } else if (d / 2 < -range || d / 2 > range) {
            return 0;
        }
    }
    return 1;
}
static int put_bal_envelope(Sw* w, jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, const int* df)
{
    const int amp_res = (c->L_E == 1 && c->frame_class == 0) ? 0 : s->hdr.amp_res;
    const int(*th)[2] = amp_res ? JAAD_SBR_T_HUFFMAN_ENV_BAL_3_0DB : JAAD_SBR_T_HUFFMAN_ENV_BAL_1_5DB;
    const int(*fh)[2] = amp_res ? JAAD_SBR_F_HUFFMAN_ENV_BAL_3_0DB : JAAD_SBR_F_HUFFMAN_ENV_BAL_1_5DB;
    const int tn = amp_res ? NN(JAAD_SBR_T_HUFFMAN_ENV_BAL_3_0DB) : NN(JAAD_SBR_T_HUFFMAN_ENV_BAL_1_5DB);
    const int fn = amp_res ? NN(JAAD_SBR_F_HUFFMAN_ENV_BAL_3_0DB) : NN(JAAD_SBR_F_HUFFMAN_ENV_BAL_1_5DB);
    for (int l = 0; l < c->L_E; l++) {
        if (!bal_env_ok(s, ch, c, l, df[l])) return FAIL;
        const int nb = s->n[c->f[l] & 1];
        if (!df[l]) {
            sput(w, (uint32_t)(c->E[l][0] >> 1), amp_res ? 5 : 6);
            for (int k = 1; k < nb; k++)
                if (put_tree(w, fh, fn, 64, (c->E[l][k] - c->E[l][k - 1]) / 2)) return FAIL;
        } else {
            for (int k = 0; k < nb; k++)
                if (put_tree(w, th, tn, 64, (c->E[l][k] - env_prev_value(s, ch, c, l, k)) / 2)) return FAIL;
        }
    }
    return 0;
}
static int bal_noise_ok(const jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, int l, int df)
{
    for (int k = 0; k < s->N_Q; k++) {
        const int v = c->Q[l][k];
        const int base = df ? (l == 0 ? s->Q_prev[ch][k] : c->Q[l - 1][k]) : (k ? c->Q[l][k - 1] : 0);
        const int d = v - base;
        if (v < 0 || (d & 1)) return 0;
        if (!df && k == 0) {
            if ((v >> 1) > 31) return 0;
        } else if (d / 2 < -12 || d / 2 > 12) {
            return 0;
        }
    }
    return 1;
}
static int put_bal_noise(Sw* w, jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* c, const int* df)
{
    for (int l = 0; l < c->L_Q; l++) {
        if (!bal_noise_ok(s, ch, c, l, df[l])) return FAIL;
        if (!df[l]) {
            sput(w, (uint32_t)(c->Q[l][0] >> 1), 5);
            for (int k = 1; k < s->N_Q; k++)
                if (put_tree(w, JAAD_SBR_F_HUFFMAN_ENV_BAL_3_0DB, NN(JAAD_SBR_F_HUFFMAN_ENV_BAL_3_0DB), 64,
                             (c->Q[l][k] - c->Q[l][k - 1]) / 2))
                    return FAIL;
        } else {
            for (int k = 0; k < s->N_Q; k++) {
                const int p = l == 0 ? s->Q_prev[ch][k] : c->Q[l - 1][k];
                if (put_tree(w, JAAD_SBR_T_HUFFMAN_NOISE_BAL_3_0DB, NN(JAAD_SBR_T_HUFFMAN_NOISE_BAL_3_0DB), 64,
                             (c->Q[l][k] - p) / 2))
                    return FAIL;
            }
        }
    }
    return 0;
}

/* ps_data for records with IID / ICC enabled, fixed borders and no IPD/OPD extension */
static int put_ps(Sw* w, jaad_sbr_wstate* s, const jaad_ps_frame* p)
{
    static const int nr_par[6] = {10, 20, 34, 10, 20, 34};
    if (p->nr_ipdopd_par || p->iid_mode > 5 || p->icc_mode > 5) return FAIL;
    const int ne = p->num_env, tmp = ne == 1 ? 1 : (ne == 2 ? 2 : (ne == 4 ? 3 : -1));
    if (tmp < 0) return FAIL;
    for (int e = 0; e <= ne; e++)
        if (p->border[e] != e * 32 / ne) return FAIL;
    const int hdr = !s->ps_have_hdr || s->ps_iid_mode != p->iid_mode || s->ps_icc_mode != p->icc_mode || rnd(s, 3) == 0;
    sput(w, (uint32_t)hdr, 1);
    if (hdr) {
        sput(w, 1, 1);
        sput(w, p->iid_mode, 3);
        sput(w, 1, 1);
        sput(w, p->icc_mode, 3);
        sput(w, 0, 1); /* no extension */
        s->ps_have_hdr = 1;
        s->ps_iid_mode = p->iid_mode;
        s->ps_icc_mode = p->icc_mode;
    }
    sput(w, 0, 1); /* var_borders */
    sput(w, (uint32_t)tmp, 2);
    for (int which = 0; which < 2; which++) {
        const int id = which ? p->icc_mode : p->iid_mode;
        const int stride = id % 3 == 0 ? 2 : 0, np = nr_par[id];
        const int fine = !which && id >= 3;
        const int(*ft)[2] = which ? JAAD_PS_F_HUFF_ICC : (fine ? JAAD_PS_F_HUFF_IID_FINE : JAAD_PS_F_HUFF_IID_DEF);
        const int(*tt)[2] = which ? JAAD_PS_T_HUFF_ICC : (fine ? JAAD_PS_T_HUFF_IID_FINE : JAAD_PS_T_HUFF_IID_DEF);
        const int fnn = which ? NN(JAAD_PS_F_HUFF_ICC) : (fine ? NN(JAAD_PS_F_HUFF_IID_FINE) : NN(JAAD_PS_F_HUFF_IID_DEF));
        const int tnn = which ? NN(JAAD_PS_T_HUFF_ICC) : (fine ? NN(JAAD_PS_T_HUFF_IID_FINE) : NN(JAAD_PS_T_HUFF_IID_DEF));
        int* first = which ? s->ps_first_icc : s->ps_first_iid;
        for (int e = 0; e < ne; e++) {
            const int8_t* v = which ? p->icc[e] : p->iid[e];
            const int8_t* pv = e ? (which ? p->icc[e - 1] : p->iid[e - 1]) : NULL;
            /* coded value i is the decoded index[i * max(stride, 1)] (Envelope.decode) */
            const int st = stride ? stride : 1;
            /* time or frequency deltas: the shorter one, or a random one when they cost about
             * the same (time deltas out of the table's range cannot be coded) */
            int cost[2] = {0, 0};
            for (int i = 0; i < np; i++) {
                uint32_t code;
                int len;
                const int dd = v[i * st] - (pv ? pv[i * stride] : first[i * stride]);
                const int df = i == 0 ? v[0] : v[i * st] - v[(i - 1) * st];
                cost[1] = (cost[1] < 0 || tree_find(tt, tnn, 0, dd - 31, 0, 0, &code, &len)) ? -1 : cost[1] + len;
                cost[0] = (cost[0] < 0 || tree_find(ft, fnn, 0, df - 31, 0, 0, &code, &len)) ? -1 : cost[0] + len;
            }
            int dt;
            if (cost[1] < 0) dt = 0;
            else if (cost[0] < 0) dt = 1;
            else if (abs(cost[0] - cost[1]) < 24) dt = (int)rnd(s, 2);
            else dt = cost[1] < cost[0];
            sput(w, (uint32_t)dt, 1);
            for (int i = 0; i < np; i++) {
                const int target = v[i * st];
                int d;
                if (dt) d = target - (pv ? pv[i * stride] : first[i * stride]);
                else d = i == 0 ? target : target - v[(i - 1) * st];
                if (put_tree(w, dt ? tt : ft, dt ? tnn : fnn, 31, d)) return FAIL;
            }
        }
        const int8_t* last = which ? p->icc[ne - 1] : p->iid[ne - 1];
        for (int b = 0; b < 34; b++) first[b] = last[b];
    }
    return 0;
}

/* the FIL element (SyntacticElements.decodeFIL, A/syntax/SyntacticElements.java:169-203) around an
 * extension payload of `bits` bits in buf: count bytes (escape: count = 15 + esc - 1), payload
 * padded to whole bytes */
static long emit_fil(Sw* outw, const uint8_t* buf, size_t bits)
{
    const int count = (int)((bits + 7) / 8);
    if (count > 15 + 255 - 1) return FAIL;
    sput(outw, 6, 3);
    if (count >= 15) {
        sput(outw, 15, 4);
        sput(outw, (uint32_t)(count - 14), 8);
    } else {
        sput(outw, (uint32_t)count, 4);
    }
    for (int i = 0; i < count; i++) sput(outw, buf[i], 8);
    return outw->overflow ? -1 : (long)outw->pos;
}

/* a grid whose borders do not fit: VARFIX, lead border 3, relative borders 8, 8, 8 -> the third
 * border 27 puts 2 * 27 + tHFAdj past numTimeSlotsRate + tHFGen (A/sbr/Channel.java:497-503) */
static void put_bad_grid(Sw* w, jaad_sbr_wstate* s)
{
    sput(w, 2, 2);          /* VARFIX */
    sput(w, 3, 2);          /* bs_abs_bord */
    sput(w, 3, 2);          /* bs_num_env - 1 */
    for (int r = 0; r < 3; r++) sput(w, 3, 2); /* rel = 2 * 3 + 2 */
    sput(w, rnd(s, 5), 3);  /* bs_pointer (sbr_log2(5) = 3 bits) */
    for (int e = 0; e < 4; e++) sput(w, rnd(s, 2), 1);
    for (int i = 0; i < 16; i++) sput(w, rnd(s, 2), 1); /* whatever followed: never read */
}

/* bs_df_env / bs_df_noise of one channel: the reader reads n_env / n_noise flags (the channel's
 * L_E / L_Q when it reads them) and keeps older entries; an envelope past them takes the entry an
 * earlier frame left */
static void choose_df(jaad_sbr_wstate* s, int ch, const jaad_sbr_channel* C, int n_env, int n_noise, int bal,
                      int* dfe, int* dfq)
{
    const int prev_ok = s->have_prev[ch] && s->prev_gen[ch] == s->tables_gen;
    for (int l = 0; l < C->L_E; l++) {
        if (l >= n_env) {
            dfe[l] = s->df_env[ch][l];
            continue;
        }
        dfe[l] = (l > 0 || prev_ok) ? (int)rnd(s, 2) : 0;
        if (dfe[l] && !(bal ? bal_env_ok(s, ch, C, l, 1) : env_time_ok(s, ch, C, l))) dfe[l] = 0;
    }
    for (int l = 0; l < C->L_Q; l++) {
        if (l >= n_noise) {
            dfq[l] = s->df_noise[ch][l];
            continue;
        }
        dfq[l] = (l > 0 || prev_ok) ? (int)rnd(s, 2) : 0;
        if (dfq[l] && !(bal ? bal_noise_ok(s, ch, C, l, 1) : noise_time_ok(s, ch, C, l))) dfq[l] = 0;
    }
}

/*
 * The FIL element carrying `rec` for the channel element just written (nch 1: SCE, 2: CPE),
 * MSB-first into out[cap].  Returns its length in bits (0: no FIL element, for a frame whose SBR
 * payload is missing), or -1 when the record is not representable by this writer.
 *   status JAAD_SBR_UPSAMPLE: no payload, or a payload whose grid does not fit (sbr_data fails);
 *   no header seen yet: a payload of bs_header_flag = 0 only (the reader skips sbr_data);
 *   coupling: SBR2.sbr_data's coupled branch (A/sbr/SBR2.java:44-72), channel 1 balance coded.
 */
long jaad_sbr_fil_bits(void* state, int nch, const jaad_sbr_frame* rec, uint8_t* out, size_t cap)
{
    jaad_sbr_wstate* s = (jaad_sbr_wstate*)state;
    memset(out, 0, cap);
    Sw fil = {out, cap, 0, 0};
    Sw* outw = &fil;
    uint8_t buf[1024];
    memset(buf, 0, sizeof buf);
    Sw w = {buf, sizeof buf, 0, 0};
    if (rec->status == JAAD_SBR_UPSAMPLE) {
        if (rec->header_present) return FAIL;
        if (!s->have_hdr || rnd(s, 2)) return 0; /* no SBR payload after the element */
    }
    const int crc = (int)rnd(s, 4) == 0;
    sput(&w, crc ? 14 : 13, 4);
    if (crc) sput(&w, rnd(s, 1024), 10);
    if (rec->status == JAAD_SBR_UPSAMPLE) { /* a header-less payload whose grid fails */
        sput(&w, 0, 1);
        if (nch == 1) {
            sput(&w, 0, 1);
            put_bad_grid(&w, s);
        } else {
            sput(&w, 0, 1);
            const int coupled = (int)rnd(s, 2);
            sput(&w, (uint32_t)coupled, 1);
            if (!coupled && rnd(s, 2)) { /* channel 0's grid fits, channel 1's does not */
                sput(&w, 0, 2);
                sput(&w, rnd(s, 3), 2);
                sput(&w, rnd(s, 2), 1);
            }
            put_bad_grid(&w, s);
        }
        if (w.overflow) return FAIL;
        return emit_fil(outw, buf, w.pos);
    }
    if (!rec->header_present && !s->have_hdr) { /* before the first header: nothing is read */
        sput(&w, 0, 1);
        for (int i = 0; i < 8; i++) sput(&w, rnd(s, 2), 1);
        return emit_fil(outw, buf, w.pos);
    }
    /* header */
    sput(&w, rec->header_present, 1);
    if (rec->header_present) {
        put_header(&w, s, &rec->hdr);
        if (!s->have_hdr || hdr_differs(&rec->hdr, &s->hdr)) {
            int info[5];
            if (orc_sbr_res_tables(&rec->hdr, s->out_sf, info, &s->ftr[0][0])) return FAIL;
            s->n[0] = info[0];
            s->n[1] = info[1];
            s->N_Q = info[2];
            s->N_high = info[3];
            s->N_low = info[4];
            s->tables_gen++;
        }
        s->hdr = rec->hdr;
        s->have_hdr = 1;
    } else if (memcmp(&rec->hdr, &s->hdr, sizeof rec->hdr)) {
        return FAIL; /* a header-less frame carries the current header */
    }
    const int coupled = nch == 2 && rec->coupling;
    int dfe[2][9], dfq[2][3];
    if (coupled) {
        const jaad_sbr_channel *C0 = &rec->ch[0], *C1 = &rec->ch[1];
        if (C1->frame_class != C0->frame_class || C1->L_E != C0->L_E || C1->L_Q != C0->L_Q ||
            C1->bs_pointer != C0->bs_pointer || memcmp(C1->t_E, C0->t_E, C0->L_E + 1) ||
            memcmp(C1->f, C0->f, C0->L_E) || memcmp(C1->t_Q, C0->t_Q, C0->L_Q + 1) ||
            memcmp(C1->invf_mode, C0->invf_mode, (size_t)s->N_Q))
            return FAIL; /* not what Channel.couple leaves */
        choose_df(s, 0, C0, C0->L_E, C0->L_Q, 0, dfe[0], dfq[0]);
        /* channel 1 reads its flags before couple(): with the previous frame's L_E / L_Q */
        choose_df(s, 1, C1, s->L_E_last[1], s->L_Q_last[1], 1, dfe[1], dfq[1]);
        sput(&w, 0, 1); /* bs_data_extra */
        sput(&w, 1, 1); /* bs_coupling */
        if (put_grid(&w, C0)) return FAIL;
        for (int l = 0; l < C0->L_E; l++) sput(&w, (uint32_t)dfe[0][l], 1);
        for (int l = 0; l < C0->L_Q; l++) sput(&w, (uint32_t)dfq[0][l], 1);
        for (int l = 0; l < s->L_E_last[1]; l++) sput(&w, (uint32_t)(l < C1->L_E ? dfe[1][l] : s->df_env[1][l]), 1);
        for (int l = 0; l < s->L_Q_last[1]; l++) sput(&w, (uint32_t)(l < C1->L_Q ? dfq[1][l] : s->df_noise[1][l]), 1);
        for (int k = 0; k < s->N_Q; k++) sput(&w, C0->invf_mode[k] & 3, 2);
        if (put_envelope(&w, s, 0, C0, dfe[0]) || put_noise(&w, s, 0, C0, dfq[0]) ||
            put_bal_envelope(&w, s, 1, C1, dfe[1]) || put_bal_noise(&w, s, 1, C1, dfq[1]))
            return FAIL;
        /* flags the reader now holds */
        for (int l = 0; l < C0->L_E; l++) s->df_env[0][l] = dfe[0][l];
        for (int l = 0; l < C0->L_Q; l++) s->df_noise[0][l] = dfq[0][l];
        for (int l = 0; l < s->L_E_last[1] && l < C1->L_E; l++) s->df_env[1][l] = dfe[1][l];
        for (int l = 0; l < s->L_Q_last[1] && l < C1->L_Q; l++) s->df_noise[1][l] = dfq[1][l];
    } else {
        for (int c = 0; c < nch; c++) choose_df(s, c, &rec->ch[c], rec->ch[c].L_E, rec->ch[c].L_Q, 0, dfe[c], dfq[c]);
        if (nch == 1) {
            sput(&w, 0, 1); /* bs_data_extra */
        } else {
            sput(&w, 1, 1); /* bs_data_extra: 8 reserved bits */
            sput(&w, 0x5A, 8);
            sput(&w, 0, 1); /* bs_coupling */
        }
        for (int c = 0; c < nch; c++)
            if (put_grid(&w, &rec->ch[c])) return FAIL;
        for (int c = 0; c < nch; c++) {
            for (int l = 0; l < rec->ch[c].L_E; l++) sput(&w, (uint32_t)dfe[c][l], 1);
            for (int l = 0; l < rec->ch[c].L_Q; l++) sput(&w, (uint32_t)dfq[c][l], 1);
        }
        for (int c = 0; c < nch; c++)
            for (int k = 0; k < s->N_Q; k++) sput(&w, rec->ch[c].invf_mode[k] & 3, 2);
        if (nch == 1) {
            if (put_envelope(&w, s, 0, &rec->ch[0], dfe[0]) || put_noise(&w, s, 0, &rec->ch[0], dfq[0])) return FAIL;
        } else {
            if (put_envelope(&w, s, 0, &rec->ch[0], dfe[0]) || put_envelope(&w, s, 1, &rec->ch[1], dfe[1]) ||
                put_noise(&w, s, 0, &rec->ch[0], dfq[0]) || put_noise(&w, s, 1, &rec->ch[1], dfq[1]))
                return FAIL;
        }
        for (int c = 0; c < nch; c++) {
            for (int l = 0; l < rec->ch[c].L_E; l++) s->df_env[c][l] = dfe[c][l];
            for (int l = 0; l < rec->ch[c].L_Q; l++) s->df_noise[c][l] = dfq[c][l];
        }
    }
    for (int c = 0; c < nch; c++) {
        const jaad_sbr_channel* C = &rec->ch[c];
        sput(&w, C->add_harmonic_flag, 1);
        if (C->add_harmonic_flag)
            for (int k = 0; k < s->N_high; k++) sput(&w, (uint32_t)((C->add_harmonic >> k) & 1u), 1);
    }
    /* extended data: PS of an SCE */
    if (nch == 1 && rec->ps_present) {
        uint8_t pb[512];
        memset(pb, 0, sizeof pb);
        Sw pw = {pb, sizeof pb, 0, 0};
        sput(&pw, 2, 2); /* EXTENSION_ID_PS */
        if (put_ps(&pw, s, &rec->ps) || pw.overflow) return FAIL;
        const int cnt = (int)((pw.pos + 7) / 8);
        sput(&w, 1, 1);
        if (cnt >= 15) {
            sput(&w, 15, 4);
            sput(&w, (uint32_t)(cnt - 15), 8);
        } else {
            sput(&w, (uint32_t)cnt, 4);
        }
        for (int i = 0; i < cnt; i++) sput(&w, pb[i], 8);
    } else {
        sput(&w, 0, 1);
    }
    if (w.overflow) return FAIL;
    if ((w.pos + 7) / 8 > 15 + 255 - 1) return FAIL;
    /* state the next frame's delta coding starts from (sbr_save_prev_data) */
    for (int c = 0; c < nch; c++) {
        const jaad_sbr_channel* C = &rec->ch[c];
        s->f_prev[c] = C->f[C->L_E - 1];
        for (int k = 0; k < 64; k++) {
            s->E_prev[c][k] = C->E[C->L_E - 1][k];
            s->Q_prev[c][k] = k < 8 ? C->Q[C->L_Q - 1][k] : 0;
        }
        s->have_prev[c] = 1;
        s->prev_gen[c] = s->tables_gen;
        s->L_E_last[c] = C->L_E;
        s->L_Q_last[c] = C->L_Q;
    }
    return emit_fil(outw, buf, w.pos);
}
