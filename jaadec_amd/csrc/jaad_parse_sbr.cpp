// SBR / PS extension payloads of the host bitstream front end (include/jaad_parse.h): one
// sbr_extension_data element (FIL type EXT_SBR_DATA / _CRC) -> one jaad_sbr_frame record, as
// the reference's parse leaves its state (A/ = aac/src/main/java/net/sourceforge/jaad/aac/):
//
//   SBR.decode / readHeader / readExtendedData   A/sbr/SBR.java:161-245
//   Header.decode / differs                      A/sbr/Header.java:24-79
//   SBR1.sbr_data (SCE), SBR2.sbr_data (CPE)     A/sbr/SBR1.java:34-60, A/sbr/SBR2.java:35-135
//   Channel grid / dtdf / invf / envelope /      A/sbr/Channel.java:85-583
//     noise + extract_*_data, couple
//   sinusoidal_coding                            A/sbr/SBR.java:248-254
//   sbr_save_prev_data (E/Q/f of frame f-1)      A/sbr/SBR.java:256-284
//   PSImpl.decode + ps_data_decode               A/ps/PSImpl.java:103-199
//   EnvData / Envelope / modes / Extension       A/ps/EnvData.java, Envelope.java, IIDMode.java,
//                                                ICCMode.java, PDMode.java, Extension.java, ExtData.java
#include <cstring>

#include "jaad_parse_internal.h"
#include "jaad_sbr.h"
#include "tables/jaad_huffman_tables.inc"

namespace jaad {
namespace parse {
namespace {

enum { FIXFIX = 0, FIXVAR = 1, VARFIX = 2, VARVAR = 3 };

// binary-tree Huffman (Channel.decodeHuffman / ps Huffman.table): leaf < 0; value = leaf + bias
int tree_decode(BitReader& br, const int (*t)[2], int nnodes, int bias, int& v)
{
    int index = 0;
    for (int steps = 0; index >= 0; steps++) {
        if (br.left() < 1) return JAAD_ERR_EOS;
        if (index >= nnodes || steps > 64) return JAAD_ERR_BITSTREAM;
        index = t[index][br.read(1)];
    }
    v = index + bias;
    return JAAD_OK;
}
#define TREE(tab) (tab), (int)(sizeof(tab) / sizeof((tab)[0]))

// Header.decode (A/sbr/Header.java:24-62), defaults of the optional parts applied
int read_header(BitReader& br, jaad_sbr_header& h)
{
    if (br.left() < 16) return JAAD_ERR_EOS;
    std::memset(&h, 0, sizeof h);
    h.amp_res = (uint8_t)br.read(1);
    h.start_freq = (uint8_t)br.read(4);
    h.stop_freq = (uint8_t)br.read(4);
    h.xover_band = (uint8_t)br.read(3);
    br.skip(2);
    const bool x1 = br.read(1), x2 = br.read(1);
    if (x1) {
        if (br.left() < 5) return JAAD_ERR_EOS;
        h.freq_scale = (uint8_t)br.read(2);
        h.alter_scale = (uint8_t)br.read(1);
        h.noise_bands = (uint8_t)br.read(2);
    } else {
        h.freq_scale = 2;
        h.alter_scale = 1;
        h.noise_bands = 2;
    }
    if (x2) {
        if (br.left() < 6) return JAAD_ERR_EOS;
        h.limiter_bands = (uint8_t)br.read(2);
        h.limiter_gains = (uint8_t)br.read(2);
        h.interpol_freq = (uint8_t)br.read(1);
        h.smoothing_mode = (uint8_t)br.read(1);
    } else {
        h.limiter_bands = 2;
        h.limiter_gains = 2;
        h.interpol_freq = 1;
        h.smoothing_mode = 1;
    }
    return JAAD_OK;
}

bool header_differs(const jaad_sbr_header& a, const jaad_sbr_header& b)  // Header.differs
{
    return a.start_freq != b.start_freq || a.stop_freq != b.stop_freq || a.freq_scale != b.freq_scale ||
           a.alter_scale != b.alter_scale || a.xover_band != b.xover_band || a.noise_bands != b.noise_bands;
}

// the channel state is parsed in place (on the parser's uncommitted copy of its state)
using ChWork = SbrParseState::Ch;

int sbr_log2(int v)
{
    static const int tab[10] = {0, 0, 1, 2, 2, 3, 3, 3, 3, 4};
    return v >= 0 && v < 10 ? tab[v] : 0;
}

// Channel.sbr_grid + envelope_time_border_vector + noise_floor_time_border_vector (:324-583);
// numTimeSlots 16, rate 2, tHFAdj 2, tHFGen 8 (1024-sample frames)
// Channel.sbr_grid returning 1 (A/sbr/Channel.java:418-432): the grid's borders do not fit.  The
// reference then marks the frame's SBR data invalid (SBR.decode, A/sbr/SBR.java:179-182).
constexpr int kGridInvalid = 1;

int read_grid(BitReader& br, ChWork& w)
{
    const int NTS = 16, RATE = 2;
    if (br.left() < 2) return JAAD_ERR_EOS;
    w.frame_class = (int)br.read(2);
    int abs_lead = 0, abs_trail = NTS, n_rel_lead = 0, n_rel_trail = 0, num_env = 0;
    int rel[9] = {0}, rel0[9] = {0}, rel1[9] = {0}, nrel0 = 0, nrel1 = 0;
    switch (w.frame_class) {
    case FIXFIX: {
        if (br.left() < 3) return JAAD_ERR_EOS;
        const int i = (int)br.read(2);
        num_env = (1 << i) < 5 ? (1 << i) : 5;
        const int fr = (int)br.read(1);
        for (int e = 0; e < num_env && e < 6; e++) w.f[e] = fr;
        w.L_E = num_env < 4 ? num_env : 4;
        abs_lead = 0;
        abs_trail = NTS;
        n_rel_lead = num_env - 1;
        break;
    }
    case FIXVAR:
    case VARFIX: {
        if (br.left() < 4) return JAAD_ERR_EOS;
        const int ab = (int)br.read(2);
        num_env = (int)br.read(2) + 1;
        for (int r = 0; r < num_env - 1; r++) {
            if (br.left() < 2) return JAAD_ERR_EOS;
            rel[r] = 2 * (int)br.read(2) + 2;
        }
        const int pb = sbr_log2(num_env + 1);
        if (br.left() < pb + num_env) return JAAD_ERR_EOS;
        w.bs_pointer = (int)br.read(pb);
        for (int e = 0; e < num_env; e++) {
            if (w.frame_class == FIXVAR) w.f[num_env - e - 1] = (int)br.read(1);
            else w.f[e] = (int)br.read(1);
        }
        w.L_E = num_env < 4 ? num_env : 4;
        if (w.frame_class == FIXVAR) {
            abs_lead = 0;
            abs_trail = ab + NTS;
            n_rel_trail = num_env - 1;
        } else {
            abs_lead = ab;
            abs_trail = NTS;
            n_rel_lead = num_env - 1;
        }
        break;
    }
    default: {  // VARVAR
        if (br.left() < 8) return JAAD_ERR_EOS;
        abs_lead = (int)br.read(2);
        abs_trail = (int)br.read(2) + NTS;
        nrel0 = (int)br.read(2);
        nrel1 = (int)br.read(2);
        num_env = nrel0 + nrel1 + 1 < 5 ? nrel0 + nrel1 + 1 : 5;
        for (int r = 0; r < nrel0; r++) {
            if (br.left() < 2) return JAAD_ERR_EOS;
            rel0[r] = 2 * (int)br.read(2) + 2;
        }
        for (int r = 0; r < nrel1; r++) {
            if (br.left() < 2) return JAAD_ERR_EOS;
            rel1[r] = 2 * (int)br.read(2) + 2;
        }
        const int pb = sbr_log2(nrel0 + nrel1 + 2);
        if (br.left() < pb + num_env) return JAAD_ERR_EOS;
        w.bs_pointer = (int)br.read(pb);
        for (int e = 0; e < num_env; e++) w.f[e] = (int)br.read(1);
        w.L_E = num_env;
        n_rel_lead = nrel0;
        n_rel_trail = nrel1;
        break;
    }
    }
    (void)n_rel_lead;
    (void)n_rel_trail;
    if (w.L_E <= 0) return kGridInvalid;
    w.L_Q = w.L_E > 1 ? 2 : 1;
    // envelope_time_border_vector (:455-542)
    // eTmp persists in the reference; t_E is a full copy of it, so entries past L_E are stale
    int e[6];
    for (int i = 0; i < 6; i++) e[i] = w.t_E[i];
    e[0] = RATE * abs_lead;
    e[w.L_E] = RATE * abs_trail;
    switch (w.frame_class) {
    case FIXFIX:
        if (w.L_E == 4) {
            const int t = NTS / 4;
            e[3] = RATE * 3 * t;
            e[2] = RATE * 2 * t;
            e[1] = RATE * t;
        } else if (w.L_E == 2) {
            e[1] = RATE * (NTS / 2);
        }
        break;
    case FIXVAR:
        if (w.L_E > 1) {
            int i = w.L_E, border = abs_trail;
            for (int l = 0; l < w.L_E - 1; l++) {
                if (border < rel[l]) return kGridInvalid;
                border -= rel[l];
                e[--i] = RATE * border;
            }
        }
        break;
    case VARFIX:
        if (w.L_E > 1) {
            int i = 1, border = abs_lead;
            for (int l = 0; l < w.L_E - 1; l++) {
                border += rel[l];
                if (RATE * border + 2 > 2 * NTS + 8) return kGridInvalid;
                e[i++] = RATE * border;
            }
        }
        break;
    default:
        if (nrel0) {
            int i = 1, border = abs_lead;
            for (int l = 0; l < nrel0; l++) {
                border += rel0[l];
                if (RATE * border + 2 > 2 * NTS + 8) return kGridInvalid;
                e[i++] = RATE * border;
            }
        }
        if (nrel1) {
            int i = w.L_E, border = abs_trail;
            for (int l = 0; l < nrel1; l++) {
                if (border < rel1[l]) return kGridInvalid;
                border -= rel1[l];
                e[--i] = RATE * border;
            }
        }
        break;
    }
    for (int i = 0; i < 6; i++) w.t_E[i] = e[i];
    // noise_floor_time_border_vector + middleBorder (:544-582)
    w.t_Q[0] = w.t_E[0];
    if (w.L_E == 1) {
        w.t_Q[1] = w.t_E[1];
        w.t_Q[2] = 0;
    } else {
        int mid = 0;
        switch (w.frame_class) {
        case FIXFIX: mid = w.L_E / 2; break;
        case VARFIX: mid = w.bs_pointer == 0 ? 1 : (w.bs_pointer == 1 ? w.L_E - 1 : w.bs_pointer - 1); break;
        default: mid = w.bs_pointer > 1 ? w.L_E + 1 - w.bs_pointer : w.L_E - 1; break;
        }
        if (mid < 0) mid = 0;
        if (mid > 5) return JAAD_ERR_BITSTREAM;  // t_E[6]: out of bounds in the reference (throws)
        w.t_Q[1] = w.t_E[mid];
        w.t_Q[2] = w.t_E[w.L_E];
    }
    return JAAD_OK;
}

int read_dtdf(BitReader& br, ChWork& w)  // Channel.sbr_dtdf (:85-94)
{
    if (br.left() < w.L_E + w.L_Q) return JAAD_ERR_EOS;
    for (int i = 0; i < w.L_E; i++) w.df_env[i] = (int)br.read(1);
    for (int i = 0; i < w.L_Q; i++) w.df_noise[i] = (int)br.read(1);
    return JAAD_OK;
}

int read_invf(BitReader& br, ChWork& w, int N_Q)  // Channel.invf_mode (:97-101)
{
    if (br.left() < 2 * N_Q) return JAAD_ERR_EOS;
    for (int n = 0; n < N_Q; n++) w.invf[n] = (int)br.read(2);
    return JAAD_OK;
}

// Channel.sbr_envelope + extract_envelope_data (:125-250)
int read_envelope(BitReader& br, ChWork& w, const SbrParseState& S, bool coupled)
{
    const bool amp_res = (w.L_E == 1 && w.frame_class == FIXFIX) ? false : S.hdr.amp_res != 0;
    const int delta = coupled ? 1 : 0;
    const int(*th)[2];
    const int(*fh)[2];
    int tn, fn;
    if (coupled) {
        if (amp_res) {
            th = JAAD_SBR_T_HUFFMAN_ENV_BAL_3_0DB, tn = 24;
            fh = JAAD_SBR_F_HUFFMAN_ENV_BAL_3_0DB, fn = 24;
        } else {
            th = JAAD_SBR_T_HUFFMAN_ENV_BAL_1_5DB, tn = 48;
            fh = JAAD_SBR_F_HUFFMAN_ENV_BAL_1_5DB, fn = 48;
        }
    } else {
        if (amp_res) {
            th = JAAD_SBR_T_HUFFMAN_ENV_3_0DB, tn = 62;
            fh = JAAD_SBR_F_HUFFMAN_ENV_3_0DB, fn = 62;
        } else {
            th = JAAD_SBR_T_HUFFMAN_ENV_1_5DB, tn = 120;
            fh = JAAD_SBR_F_HUFFMAN_ENV_1_5DB, fn = 120;
        }
    }
    for (int env = 0; env < w.L_E; env++) {
        const int nb = S.n[w.f[env] & 1];
        if (w.df_env[env] == 0) {
            const int bits = coupled ? (amp_res ? 5 : 6) : (amp_res ? 6 : 7);
            if (br.left() < bits) return JAAD_ERR_EOS;
            w.E[0][env] = (int)br.read(bits) * (1 << delta);  // Java << on an int (negative deltas too)
            for (int band = 1; band < nb; band++) {
                int v;
                const int st = tree_decode(br, fh, fn, 64, v);
                if (st) return st;
                w.E[band][env] = v * (1 << delta);  // Java << on an int (negative deltas too)
            }
        } else {
            for (int band = 0; band < nb; band++) {
                int v;
                const int st = tree_decode(br, th, tn, 64, v);
                if (st) return st;
                w.E[band][env] = v * (1 << delta);  // Java << on an int (negative deltas too)
            }
        }
    }
    // extract_envelope_data (:203-250)
    for (int l = 0; l < w.L_E; l++) {
        const int nb = S.n[w.f[l] & 1];
        if (w.df_env[l] == 0) {
            for (int k = 1; k < nb; k++) {
                w.E[k][l] = w.E[k - 1][l] + w.E[k][l];
                if (w.E[k][l] < 0) w.E[k][l] = 0;
            }
        } else {
            const int g = l == 0 ? w.f_prev : w.f[l - 1];
            if (w.f[l] == g) {
                for (int k = 0; k < nb; k++) w.E[k][l] = (l == 0 ? w.E_prev[k] : w.E[k][l - 1]) + w.E[k][l];
            } else if (g == 1 && w.f[l] == 0) {
                for (int k = 0; k < nb; k++)
                    for (int i = 0; i < S.N_high; i++)
                        if (S.f_table_res[1][i] == S.f_table_res[0][k])
                            w.E[k][l] = (l == 0 ? w.E_prev[i] : w.E[i][l - 1]) + w.E[k][l];
            } else if (g == 0 && w.f[l] == 1) {
                for (int k = 0; k < nb; k++)
                    for (int i = 0; i < S.N_low; i++)
                        if (S.f_table_res[0][i] <= S.f_table_res[1][k] && S.f_table_res[1][k] < S.f_table_res[0][i + 1])
                            w.E[k][l] = (l == 0 ? w.E_prev[i] : w.E[i][l - 1]) + w.E[k][l];
            }
        }
    }
    return JAAD_OK;
}

// Channel.sbr_noise + extract_noise_floor_data (:253-321)
int read_noise(BitReader& br, ChWork& w, const SbrParseState& S, bool coupled)
{
    const int delta = coupled ? 1 : 0;
    const int(*th)[2] = coupled ? JAAD_SBR_T_HUFFMAN_NOISE_BAL_3_0DB : JAAD_SBR_T_HUFFMAN_NOISE_3_0DB;
    const int tn = coupled ? 24 : 62;
    const int(*fh)[2] = coupled ? JAAD_SBR_F_HUFFMAN_ENV_BAL_3_0DB : JAAD_SBR_F_HUFFMAN_ENV_3_0DB;
    const int fn = coupled ? 24 : 62;
    for (int noise = 0; noise < w.L_Q; noise++) {
        if (w.df_noise[noise] == 0) {
            if (br.left() < 5) return JAAD_ERR_EOS;
            w.Q[0][noise] = (int)br.read(5) * (1 << delta);  // Java << on an int (negative deltas too)
            for (int band = 1; band < S.N_Q; band++) {
                int v;
                const int st = tree_decode(br, fh, fn, 64, v);
                if (st) return st;
                w.Q[band][noise] = v * (1 << delta);  // Java << on an int (negative deltas too)
            }
        } else {
            for (int band = 0; band < S.N_Q; band++) {
                int v;
                const int st = tree_decode(br, th, tn, 64, v);
                if (st) return st;
                w.Q[band][noise] = v * (1 << delta);  // Java << on an int (negative deltas too)
            }
        }
    }
    for (int l = 0; l < w.L_Q; l++) {
        if (w.df_noise[l] == 0) {
            for (int k = 1; k < S.N_Q; k++) w.Q[k][l] = w.Q[k][l] + w.Q[k - 1][l];
        } else {
            for (int k = 0; k < S.N_Q; k++) w.Q[k][l] = (l == 0 ? w.Q_prev[k] : w.Q[k][l - 1]) + w.Q[k][l];
        }
    }
    return JAAD_OK;
}

int read_harmonics(BitReader& br, ChWork& w, int N_high)  // SBR.sinusoidal_coding (:248-254)
{
    if (br.left() < 1) return JAAD_ERR_EOS;
    w.add_harmonic_flag = (int)br.read(1);
    w.add_harmonic = 0;
    if (w.add_harmonic_flag) {
        if (br.left() < N_high) return JAAD_ERR_EOS;
        for (int n = 0; n < N_high; n++)
            if (br.read(1)) w.add_harmonic |= 1ull << n;
    }
    return JAAD_OK;
}

// ---------------------------------------------------------------------------------------------
// Parametric stereo (PSImpl.decode, A/ps/PSImpl.java:103-134, and ps_data_decode :137-199)
// ---------------------------------------------------------------------------------------------
const int kIccNrPar[6] = {10, 20, 34, 10, 20, 34};
const int kPdNrPar[6] = {5, 11, 17, 5, 11, 17};

struct PsKind {
    int nr_par, stride, len;
    int lo, hi;  // clip range (PD: modulo 8)
    bool modulo;
    const int (*f)[2];
    int fn;
    const int (*t)[2];
    int tn;
};

PsKind iid_kind(int id)
{
    const bool fine = id >= 3;
    const int steps = fine ? 15 : 7;
    return PsKind{kIccNrPar[id], id % 3 == 0 ? 2 : 0, 34, -steps, steps, false,
                  fine ? JAAD_PS_F_HUFF_IID_FINE : JAAD_PS_F_HUFF_IID_DEF, fine ? 60 : 28,
                  fine ? JAAD_PS_T_HUFF_IID_FINE : JAAD_PS_T_HUFF_IID_DEF, fine ? 60 : 28};
}
PsKind icc_kind(int id)
{
    return PsKind{kIccNrPar[id], id % 3 == 0 ? 2 : 0, 34, 0, 7, false, JAAD_PS_F_HUFF_ICC, 14, JAAD_PS_T_HUFF_ICC, 14};
}
PsKind pd_kind(int id, bool opd)  // id < 0 (null mode): a placeholder, never read or decoded with
{
    id = id < 0 ? 0 : id;
    return PsKind{kPdNrPar[id], 1, 17, 0, 7, true, opd ? JAAD_PS_F_HUFF_OPD : JAAD_PS_F_HUFF_IPD, 7,
                  opd ? JAAD_PS_T_HUFF_OPD : JAAD_PS_T_HUFF_IPD, 7};
}
int clipv(const PsKind& k, int v)
{
    if (k.modulo) return v & 7;
    return v < k.lo ? k.lo : (v > k.hi ? k.hi : v);
}
// EnvData.readData / Envelope.read
int env_read(BitReader& br, PsEnvData& d, const PsKind& k, int num_env)
{
    if (d.mode < 0) return JAAD_OK;
    for (int n = 0; n < num_env; n++) {
        if (br.left() < 1) return JAAD_ERR_EOS;
        d.dt[n] = br.read(1) != 0;
        for (int i = 0; i < k.nr_par; i++) {
            int v;
            const int st = d.dt[n] ? tree_decode(br, k.t, k.tn, 31, v) : tree_decode(br, k.f, k.fn, 31, v);
            if (st) return st;
            d.index[n][i] = v;
        }
    }
    return JAAD_OK;
}
const int* env_prev(const PsEnvData& d, int l) { return l == 0 ? d.first : d.index[l - 1]; }
// EnvData.decode / Envelope.decode (stride quirk: stride() is 0 for modes 1, 2, 4, 5)
void env_decode(PsEnvData& d, const PsKind* k, int num_env)
{
    if (num_env == 0) {
        if (d.mode >= 0) std::memcpy(d.index[0], d.first, sizeof d.first);
        else {
            d.dt[0] = false;
            std::memset(d.index[0], 0, sizeof d.index[0]);
        }
        return;
    }
    for (int env = 0; env < num_env; env++) {
        int* ix = d.index[env];
        if (d.mode < 0 || !k) {
            d.dt[env] = false;
            std::memset(ix, 0, sizeof d.index[env]);
            continue;
        }
        const int* prev = env_prev(d, env);
        if (d.dt[env]) {
            for (int i = 0; i < k->nr_par; i++) ix[i] = clipv(*k, prev[i * k->stride] + ix[i]);
        } else {
            int p = ix[0];
            for (int i = 1; i < k->nr_par; i++) {
                p = clipv(*k, p + ix[i]);
                ix[i] = p;
            }
        }
        if (k->stride > 1)
            for (int i = k->stride * k->nr_par - 1; i > 0; --i) ix[i] = ix[i / k->stride];
    }
}
void env_update(PsEnvData& d, int num_env)  // EnvData.update
{
    if (num_env == 0) std::memset(d.first, 0, sizeof d.first);
    else std::memcpy(d.first, d.index[num_env - 1], sizeof d.first);
}
void env_restore(PsEnvData& d, int num_env)  // EnvData.restore: envs[num_env] = its predecessor
{
    std::memcpy(d.index[num_env], env_prev(d, num_env), sizeof d.index[num_env]);
}

int ps_decode(BitReader& br, SbrParseState::Ps& P, jaad_ps_frame& out)
{
    static const int num_env_tab[2][4] = {{0, 1, 2, 4}, {1, 2, 3, 4}};
    if (br.left() < 1) return JAAD_ERR_EOS;
    if (br.read(1)) {  // PS header: iid / icc / ext modes
        for (int which = 0; which < 2; which++) {
            PsEnvData& d = which ? P.icc : P.iid;
            if (br.left() < 1) return JAAD_ERR_EOS;
            if (br.read(1)) {
                if (br.left() < 3) return JAAD_ERR_EOS;
                const int id = (int)br.read(3);
                if (id > 5) return JAAD_ERR_BITSTREAM;  // IID_MODES / ICC_MODES have 6 entries
                d.mode = id;
            } else {
                d.mode = -1;
            }
        }
        if (br.left() < 1) return JAAD_ERR_EOS;
        P.ext_enabled = br.read(1) != 0;  // Extension.readMode
        if (P.ext_enabled) P.ext_data = true;
        if (P.ext_data) P.ipd.mode = P.opd.mode = P.ext_enabled ? P.iid.mode : -1;
    }
    if (br.left() < 3) return JAAD_ERR_EOS;
    P.var_borders = br.read(1) != 0;
    int num_env = num_env_tab[P.var_borders ? 1 : 0][br.read(2)];
    if (P.var_borders)
        for (int n = 1; n < num_env + 1; n++) {
            if (br.left() < 5) return JAAD_ERR_EOS;
            P.border[n] = (int)br.read(5) + 1;
        }
    const PsKind ki = iid_kind(P.iid.mode < 0 ? 0 : P.iid.mode);
    const PsKind kc = icc_kind(P.icc.mode < 0 ? 1 : P.icc.mode);
    int st = env_read(br, P.iid, ki, num_env);
    if (st) return st;
    st = env_read(br, P.icc, kc, num_env);
    if (st) return st;
    if (P.ext_enabled) {  // Extension.readData: ps_extension sub-stream
        if (br.left() < 4) return JAAD_ERR_EOS;
        int cnt = (int)br.read(4);
        if (cnt == 15) {
            if (br.left() < 8) return JAAD_ERR_EOS;
            cnt += (int)br.read(8);
        }
        if (br.left() < 8 * cnt) return JAAD_ERR_EOS;
        BitReader sub = br.sub(8 * cnt);
        br.skip(8 * cnt);
        while (sub.left() > 7) {
            const int id = (int)sub.read(2);
            if (id != 0 || !P.ext_data) continue;
            if (sub.left() < 1) return JAAD_ERR_EOS;
            P.ext_data_enabled = sub.read(1) != 0;  // ExtData.readData
            if (P.ext_data_enabled) {
                st = env_read(sub, P.ipd, pd_kind(P.ipd.mode, false), num_env);
                if (st) return st;
                st = env_read(sub, P.opd, pd_kind(P.opd.mode, true), num_env);
                if (st) return st;
            }
            if (sub.left() < 1) return JAAD_ERR_EOS;
            sub.skip(1);
        }
    }
    // an enabled extension with IID off has no PD mode: Extension.nr_par() dereferences the null
    // mode (A/ps/ExtData.java:54-58) for every PS frame the reference processes
    if (P.ext_enabled && P.ext_data && P.ipd.mode < 0) return JAAD_ERR_BITSTREAM;
    // ---- ps_data_decode (data of this frame is available)
    env_decode(P.iid, P.iid.mode < 0 ? nullptr : &ki, num_env);
    env_decode(P.icc, P.icc.mode < 0 ? nullptr : &kc, num_env);
    const bool ext = P.ext_enabled && P.ext_data;
    if (ext && P.ext_data_enabled) {
        const PsKind kpi = pd_kind(P.ipd.mode, false), kpo = pd_kind(P.opd.mode, true);
        env_decode(P.ipd, P.ipd.mode < 0 ? nullptr : &kpi, num_env);
        env_decode(P.opd, P.opd.mode < 0 ? nullptr : &kpo, num_env);
    }
    if (num_env == 0) num_env = 1;
    env_update(P.iid, num_env);
    env_update(P.icc, num_env);
    if (ext) {
        env_update(P.ipd, num_env);
        env_update(P.opd, num_env);
    }
    if (!P.var_borders) {
        P.border[0] = 0;
        for (int e = 1; e < num_env; e++) P.border[e] = e * 32 / num_env;
        P.border[num_env] = 32;
    } else {
        P.border[0] = 0;
        if (P.border[num_env] < 32) {
            env_restore(P.iid, num_env);
            env_restore(P.icc, num_env);
            if (ext) {  // ExtData.restore calls update (A/ps/ExtData.java:42-45)
                env_update(P.ipd, num_env);
                env_update(P.opd, num_env);
            }
            ++num_env;
            P.border[num_env] = 32;
        }
        int bpl = P.border[0];
        for (int e = 1; e < num_env; e++) {
            const int bp = P.border[e], mx = 32 - (num_env - e);
            bpl = bp < bpl + 1 ? bpl + 1 : bp;  // Utils.clip: max with the low bound first
            bpl = bpl > mx ? mx : bpl;
            if (bpl != bp) P.border[e] = bpl;
        }
    }
    // ---- record (jaad_ps_frame)
    std::memset(&out, 0, sizeof out);
    out.iid_mode = (uint8_t)(P.iid.mode < 0 ? 0 : P.iid.mode);
    out.icc_mode = (uint8_t)(P.icc.mode < 0 ? 1 : P.icc.mode);
    out.num_env = (uint8_t)num_env;
    out.nr_ipdopd_par = (uint8_t)(ext ? (kPdNrPar[P.ipd.mode] < 11 ? 11 : kPdNrPar[P.ipd.mode]) : 0);
    for (int e = 0; e <= num_env; e++) out.border[e] = (uint8_t)P.border[e];
    // IID / ICC: the decoded bands of the mode (the T20 filterbank reads the first 20); the
    // IPD / OPD rows go out whole: nr_ipdopd_par may exceed the mode's nr_par, and the reference
    // then reads entries left from earlier frames
    const int iid_valid = P.iid.mode % 3 == 2 ? 34 : 20, icc_valid = P.icc.mode % 3 == 2 ? 34 : 20;
    for (int e = 0; e < num_env; e++) {
        for (int b = 0; b < 34; b++) {
            out.iid[e][b] = (int8_t)(b < iid_valid ? P.iid.index[e][b] : 0);
            out.icc[e][b] = (int8_t)(b < icc_valid ? P.icc.index[e][b] : 0);
        }
        if (ext)
            for (int b = 0; b < 17; b++) {
                out.ipd[e][b] = (int8_t)P.ipd.index[e][b];
                out.opd[e][b] = (int8_t)P.opd.index[e][b];
            }
    }
    return JAAD_OK;
}

// the record carries the meaningful entries only (the Java arrays keep stale ones past them)
void to_record(const ChWork& w, const SbrParseState& S, jaad_sbr_channel& c)
{
    std::memset(&c, 0, sizeof c);
    if (w.add_harmonic_flag) c.add_harmonic = w.add_harmonic;
    for (int l = 0; l < w.L_E; l++)
        for (int k = 0; k < S.n[w.f[l] & 1]; k++) c.E[l][k] = (int16_t)w.E[k][l];
    for (int l = 0; l < w.L_Q; l++)
        for (int k = 0; k < S.N_Q; k++) c.Q[l][k] = (int16_t)w.Q[k][l];
    c.frame_class = (uint8_t)w.frame_class;
    c.L_E = (uint8_t)w.L_E;
    c.L_Q = (uint8_t)w.L_Q;
    c.bs_pointer = (uint8_t)w.bs_pointer;
    for (int i = 0; i <= w.L_E; i++) c.t_E[i] = (uint8_t)w.t_E[i];
    for (int i = 0; i <= w.L_Q && i < 3; i++) c.t_Q[i] = (uint8_t)w.t_Q[i];  // past L_Q: stale (Channel.couple)
    for (int i = 0; i < w.L_E; i++) c.f[i] = (uint8_t)w.f[i];
    for (int i = 0; i < S.N_Q; i++) c.invf_mode[i] = (uint8_t)w.invf[i];
    c.add_harmonic_flag = (uint8_t)w.add_harmonic_flag;
}

// sbr_save_prev_data (A/sbr/SBR.java:256-284): what the next frame's delta decoding reads
void save_prev(ChWork& w)
{
    w.f_prev = w.f[w.L_E - 1];
    for (int k = 0; k < 49; k++) {  // MAX_M
        w.E_prev[k] = w.E[k][w.L_E - 1];
        w.Q_prev[k] = w.Q[k][w.L_Q - 1];
    }
}

// Channel.couple (A/sbr/Channel.java:103-122)
void couple(ChWork& w, const ChWork& o, int N_Q)
{
    w.frame_class = o.frame_class;
    w.L_E = o.L_E;
    w.L_Q = o.L_Q;
    w.bs_pointer = o.bs_pointer;
    for (int n = 0; n <= o.L_E; n++) w.t_E[n] = o.t_E[n], w.f[n] = o.f[n];
    for (int n = 0; n <= o.L_Q; n++) w.t_Q[n] = o.t_Q[n];
    for (int n = 0; n < N_Q; n++) w.invf[n] = o.invf[n];
}

}  // namespace

int parse_sbr(BitReader& br, const Cfg& C, int nch, bool crc, SbrParseState& S, jaad_sbr_frame& rec)
{
    std::memset(&rec, 0, sizeof rec);
    if (crc) {
        if (br.left() < 10) return JAAD_ERR_EOS;
        br.skip(10);  // bs_sbr_crc_bits
    }
    if (br.left() < 1) return JAAD_ERR_EOS;
    if (br.read(1)) {  // SBR.readHeader
        jaad_sbr_header h;
        const int rc = read_header(br, h);
        if (rc) return rc;
        if (!S.have_hdr || header_differs(h, S.hdr)) {
            SbrFbt t;
            // calc_sbr_tables failing would make the reference revert to its previous header;
            // the DSP path has no record for that, so the frame is rejected
            if (!sbr_tables_for_parse(C.cfg.ext_sf_index, h, t)) return JAAD_ERR_BITSTREAM;
            S.n[0] = t.n[0];
            S.n[1] = t.n[1];
            S.N_Q = t.N_Q;
            S.N_high = t.N_high;
            S.N_low = t.N_low;
            for (int r = 0; r < 2; r++)
                for (int k = 0; k < 65; k++) S.f_table_res[r][k] = t.f_table_res[r][k];
        }
        S.hdr = h;
        S.have_hdr = true;
        rec.header_present = 1;
    }
    // no SBR header yet: SBR.decode skips sbr_data and marks the data valid (A/sbr/SBR.java:179-184);
    // the DSP stage then runs the QMF banks on the low band (the record stays header-less)
    if (!S.have_hdr) return JAAD_OK;
    rec.hdr = S.hdr;
    if (S.N_Q > 5 || S.n[0] > 49 || S.n[1] > 49 || S.N_high > 64) return JAAD_ERR_BITSTREAM;
    ChWork* w = S.ch;
    int rc;
    // a grid whose borders do not fit makes sbr_data return early: the reference restores the
    // grid fields of the channels it had read (frame class, L_E, L_Q; channel 0's borders too,
    // A/sbr/Channel.java:427-432, A/sbr/SBR2.java:89-103), marks the SBR data invalid and upsamples
    // the core for this frame (JAAD_SBR_UPSAMPLE); nothing after the grid is read
    struct Grid {  // what sbr_grid writes
        int frame_class, L_E, L_Q, bs_pointer, t_E[6], t_Q[3], f[6];
    } saved[2];
    for (int c = 0; c < 2; c++) {
        Grid& g = saved[c];
        g.frame_class = w[c].frame_class, g.L_E = w[c].L_E, g.L_Q = w[c].L_Q, g.bs_pointer = w[c].bs_pointer;
        std::memcpy(g.t_E, w[c].t_E, sizeof g.t_E);
        std::memcpy(g.t_Q, w[c].t_Q, sizeof g.t_Q);
        std::memcpy(g.f, w[c].f, sizeof g.f);
    }
    auto grid = [&](ChWork& c) { return read_grid(br, c); };
    auto invalid = [&]() {
        for (int c = 0; c < 2; c++) {
            const Grid& g = saved[c];
            w[c].frame_class = g.frame_class, w[c].L_E = g.L_E, w[c].L_Q = g.L_Q, w[c].bs_pointer = g.bs_pointer;
            std::memcpy(w[c].t_E, g.t_E, sizeof g.t_E);
            std::memcpy(w[c].t_Q, g.t_Q, sizeof g.t_Q);
            std::memcpy(w[c].f, g.f, sizeof g.f);
        }
        rec.status = JAAD_SBR_UPSAMPLE;
        return JAAD_OK;
    };
    if (nch == 1) {  // SBR1.sbr_data (A/sbr/SBR1.java:34-60)
        if (br.left() < 1) return JAAD_ERR_EOS;
        if (br.read(1)) br.skip(4);
        if ((rc = grid(w[0])) == kGridInvalid) return invalid();
        if (rc || (rc = read_dtdf(br, w[0])) || (rc = read_invf(br, w[0], S.N_Q)) ||
            (rc = read_envelope(br, w[0], S, false)) || (rc = read_noise(br, w[0], S, false)) ||
            (rc = read_harmonics(br, w[0], S.N_high)))
            return rc;
    } else {  // SBR2.sbr_data (A/sbr/SBR2.java:35-135)
        if (br.left() < 2) return JAAD_ERR_EOS;
        if (br.read(1)) br.skip(8);
        const bool coupling = br.read(1) != 0;
        rec.coupling = coupling;
        if (coupling) {
            // ch1.sbr_dtdf runs with ch1's L_E / L_Q of the previous frame, before couple()
            if ((rc = grid(w[0])) == kGridInvalid) return invalid();
            if (rc || (rc = read_dtdf(br, w[0])) || (rc = read_dtdf(br, w[1])) || (rc = read_invf(br, w[0], S.N_Q)))
                return rc;
            couple(w[1], w[0], S.N_Q);
            if ((rc = read_envelope(br, w[0], S, false)) || (rc = read_noise(br, w[0], S, false)) ||
                (rc = read_envelope(br, w[1], S, true)) || (rc = read_noise(br, w[1], S, true)))
                return rc;
        } else {
            if ((rc = grid(w[0])) == kGridInvalid || (!rc && (rc = grid(w[1])) == kGridInvalid)) return invalid();
            if (rc || (rc = read_dtdf(br, w[0])) || (rc = read_dtdf(br, w[1])) ||
                (rc = read_invf(br, w[0], S.N_Q)) || (rc = read_invf(br, w[1], S.N_Q)) ||
                (rc = read_envelope(br, w[0], S, false)) || (rc = read_envelope(br, w[1], S, false)) ||
                (rc = read_noise(br, w[0], S, false)) || (rc = read_noise(br, w[1], S, false)))
                return rc;
        }
        if ((rc = read_harmonics(br, w[0], S.N_high)) || (rc = read_harmonics(br, w[1], S.N_high))) return rc;
    }
    // SBR.readExtendedData (:226-240): the PS payload of an SCE (SBR1.sbr_extension)
    if (br.left() < 1) return JAAD_ERR_EOS;
    if (br.read(1)) {
        if (br.left() < 4) return JAAD_ERR_EOS;
        int cnt = (int)br.read(4);
        if (cnt == 15) {
            if (br.left() < 8) return JAAD_ERR_EOS;
            cnt += (int)br.read(8);
        }
        if (br.left() < 8 * cnt) return JAAD_ERR_EOS;
        BitReader sub = br.sub(8 * cnt);
        br.skip(8 * cnt);
        while (sub.left() > 7) {
            const int id = (int)sub.read(2);
            if (id != 2 || nch != 1) continue;  // EXTENSION_ID_PS, SCE only
            // psEnabled is on by default (A/DecoderConfig.java:36): PS data in a stream whose
            // configuration has no PS would be applied by the reference; not representable here
            if (!C.cfg.ps) return JAAD_ERR_UNSUPPORTED;
            rc = ps_decode(sub, S.ps, rec.ps);
            if (rc) return rc;
            rec.ps_present = 1;
        }
    }
    for (int c = 0; c < nch; c++) {
        to_record(w[c], S, rec.ch[c]);
        save_prev(w[c]);
    }
    return JAAD_OK;
}

int sbr_missing(const Cfg&, ParseState&, jaad_sbr_frame& rec)
{
    // a frame of an SBR stream without SBR payload after its channel element: ChannelElement.decode
    // invalidated the element's SBR (A/syntax/ChannelElement.java:56-59) and nothing revalidated
    // it, so the reference upsamples the core (A/syntax/CPE.java:201-204, SCE.java:129-131)
    std::memset(&rec, 0, sizeof rec);
    rec.status = JAAD_SBR_UPSAMPLE;
    return JAAD_OK;
}

}  // namespace parse
}  // namespace jaad
