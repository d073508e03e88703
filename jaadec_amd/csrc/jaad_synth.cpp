// Seeded synthetic parsed-frame batches (include/jaad_synth.h).  Host-only.
#include "jaad_synth.h"

#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "tables/jaad_tables.inc"

namespace {

struct SplitMix64 {
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
    uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * n >> 32); }
    bool percent(uint32_t p) { return below(100) < p; }
};

// smallest spectral codebook able to code max|q| (A/huffman/Codebooks.java: 1/2 |q|<=1,
// 3/4 <=2, 5/6 <=4, 7/8 <=7, 9/10 <=12, 11 escape); pick one of the pair at random
uint8_t codebook_for(int maxabs, SplitMix64& r)
{
    if (maxabs == 0) return JAAD_ZERO_HCB;
    int base = maxabs <= 1 ? 1 : maxabs <= 2 ? 3 : maxabs <= 4 ? 5 : maxabs <= 7 ? 7 : maxabs <= 12 ? 9 : 11;
    return (uint8_t)(base == 11 ? 11 : base + (int)r.below(2));
}

struct Gen {
    const jaad_synth_params* p;
    int16_t* q;
    uint8_t* sf;
    uint8_t* cb;
    jaad_ics_info* ics;
    uint64_t* ms;
    jaad_tns* tns;
};

void gen_stream(const Gen& G, uint32_t s)
{
    const jaad_synth_params& P = *G.p;
    const int nch = P.channel_config == 2 ? 2 : 1;
    SplitMix64 r{P.seed ^ (0xA5A5A5A5ull + (uint64_t)(P.first_stream + s) * 0x9E3779B97F4A7C15ull)};
    for (int i = 0; i < 4; i++) r.next();
    const short* offL = JAAD_SWB_OFFSET_LONG_WINDOW[P.sf_index];
    const short* offS = JAAD_SWB_OFFSET_SHORT_WINDOW[P.sf_index];
    const int nswbL = JAAD_SWB_LONG_WINDOW_COUNT[P.sf_index], nswbS = JAAD_SWB_SHORT_WINDOW_COUNT[P.sf_index];
    int prev_seq = JAAD_ONLY_LONG_SEQUENCE, shorts_left = 0;
    int prev_shape[2] = {0, 0};  // ICSInfo.windowShape starts {0,0} (A/syntax/ICSInfo.java:77)
    int sfwalk[2] = {P.global_gain, P.global_gain};
    for (uint32_t fi = 0; fi < P.frames_per_stream; fi++) {
        const size_t f = (size_t)s * P.frames_per_stream + fi;
        // ---- window sequence state machine (ONLY_LONG -> START -> SHORT x1..4 -> STOP -> ONLY_LONG)
        int seq = JAAD_ONLY_LONG_SEQUENCE;
        if (P.window_switching) {
            if (prev_seq == JAAD_ONLY_LONG_SEQUENCE || prev_seq == JAAD_LONG_STOP_SEQUENCE)
                seq = r.percent(25) ? JAAD_LONG_START_SEQUENCE : JAAD_ONLY_LONG_SEQUENCE;
            else if (prev_seq == JAAD_LONG_START_SEQUENCE) {
                seq = JAAD_EIGHT_SHORT_SEQUENCE;
                shorts_left = 1 + (int)r.below(4);
            } else {  // EIGHT_SHORT
                seq = (--shorts_left > 0) ? JAAD_EIGHT_SHORT_SEQUENCE : JAAD_LONG_STOP_SEQUENCE;
            }
        }
        prev_seq = seq;
        const bool is_short = seq == JAAD_EIGHT_SHORT_SEQUENCE;
        const int shape = (int)r.below(2);
        const uint8_t grouping = is_short ? (uint8_t)(r.next() & 0x7f) : 0;
        const int ngroups = is_short ? 8 - __builtin_popcount(grouping) : 1;
        int glen[8], gn = 1;
        glen[0] = 1;
        if (is_short)
            for (int i = 0; i < 7; i++) {
                if (grouping & (1u << i)) glen[gn - 1]++;
                else glen[gn++] = 1;
            }
        const int nswb = is_short ? nswbS : nswbL;
        const short* off = is_short ? offS : offL;
        const int max_sfb = nswb;
        const int nbands = ngroups * max_sfb;
        const bool cw = nch == 2 && P.common_window;
        uint64_t msw[2] = {0, 0};
        bool ms_present = false;
        if (cw && P.ms_mode) {
            ms_present = true;
            for (int i = 0; i < nbands; i++)
                if (P.ms_mode == 2 || r.below(2)) msw[i >> 6] |= 1ull << (i & 63);
        }
        if (G.ms) {
            G.ms[2 * f] = msw[0];
            G.ms[2 * f + 1] = msw[1];
        }
        for (int c = 0; c < nch; c++) {
            const size_t cf = f * nch + c;
            int16_t* qq = G.q + cf * 1024;
            uint8_t* ss = G.sf + cf * 128;
            uint8_t* cc = G.cb + cf * 128;
            std::memset(qq, 0, 1024 * sizeof(int16_t));
            std::memset(ss, 0, 128);
            std::memset(cc, 0, 128);
            jaad_ics_info& ic = G.ics[cf];
            std::memset(&ic, 0, sizeof(ic));
            ic.window_sequence = (uint8_t)seq;
            ic.window_shape = (uint8_t)shape;
            ic.window_shape_prev = (uint8_t)prev_shape[c];
            prev_shape[c] = shape;
            ic.max_sfb = (uint8_t)max_sfb;
            ic.grouping = grouping;
            if (cw) ic.flags |= JAAD_ICS_COMMON_WINDOW;
            if (c == 0 && ms_present) ic.flags |= JAAD_ICS_MS_PRESENT;
            // short windows: IMDCT(256) has 8x the gain of IMDCT(2048) -> lower the scalefactors
            const int sfbias = is_short ? -12 : 0;
            for (int g = 0, idx = 0, win0 = 0; g < ngroups; g++) {
                for (int b = 0; b < max_sfb; b++, idx++) {
                    // scalefactor random walk in [gg-6, gg+6]
                    sfwalk[c] += (int)r.below(3) - 1;
                    if (sfwalk[c] < P.global_gain - 6) sfwalk[c] = P.global_gain - 6;
                    if (sfwalk[c] > P.global_gain + 6) sfwalk[c] = P.global_gain + 6;
                    const bool noise = P.pns_percent && r.percent(P.pns_percent);
                    const bool intensity = !noise && c == 1 && P.is_percent && r.percent(P.is_percent);
                    if (noise) {
                        cc[idx] = JAAD_NOISE_HCB;
                        ss[idx] = (uint8_t)(100 + 20 + (int)r.below(30));  // clip(off1)+100
                        ic.flags |= JAAD_ICS_HAS_PNS;
                        continue;
                    }
                    if (intensity) {
                        cc[idx] = r.below(2) ? JAAD_INTENSITY_HCB : JAAD_INTENSITY_HCB2;
                        ss[idx] = (uint8_t)(100 - ((int)r.below(25) - 4));  // 100-clip(off2)
                        ic.flags |= JAAD_ICS_HAS_IS;
                        continue;
                    }
                    int maxabs = 0;
                    for (int w = 0; w < glen[g]; w++) {
                        const int wbase = (win0 + w) * 128;
                        for (int k = off[b]; k < off[b + 1]; k++) {
                            const int bin = is_short ? k * 8 : k;  // spectral position in 0..1023
                            double bscale = 12.0 - 11.0 * bin / 1023.0;
                            double u = r.uniform();
                            double mag = -bscale * std::log(1.0 - u);
                            int v = (int)std::floor(mag + 0.5);
                            if (P.escape_permille && r.below(1000) < P.escape_permille) v = 16 + (int)r.below(1008);
                            if (v > 8190) v = 8190;
                            if (r.below(2)) v = -v;
                            qq[wbase + k] = (int16_t)v;
                            if (std::abs(v) > maxabs) maxabs = std::abs(v);
                        }
                    }
                    cc[idx] = codebook_for(maxabs, r);
                    ss[idx] = cc[idx] == JAAD_ZERO_HCB ? 0 : (uint8_t)(sfwalk[c] + sfbias);
                    if (cc[idx] == JAAD_ZERO_HCB)
                        for (int w = 0; w < glen[g]; w++)
                            for (int k = off[b]; k < off[b + 1]; k++) qq[(win0 + w) * 128 + k] = 0;
                }
                win0 += glen[g];
            }
            // ---- TNS side info (TNS.decode, A/tools/TNS.java:35-61)
            if (G.tns) {
                jaad_tns& t = G.tns[cf];
                std::memset(&t, 0, sizeof(t));
                if (P.tns_percent && r.percent(P.tns_percent)) {
                    ic.flags |= JAAD_ICS_TNS;
                    const int nwin = is_short ? 8 : 1;
                    for (int w = 0; w < nwin; w++) {
                        jaad_tns_filter& F = t.filt[t.n_filters++];
                        F.window = (uint8_t)w;
                        F.length = (uint8_t)(is_short ? 1 + r.below(nswb) : 8 + r.below(nswb - 7));
                        F.order = (uint8_t)(is_short ? 1 + r.below(7) : 8);
                        const int res = is_short ? (int)r.below(2) : 1, compress = (int)r.below(2);
                        F.flags = (uint8_t)(r.below(2) | (res << 1) | (compress << 2));
                        const int bits = res + 3 - compress;
                        for (int i = 0; i < F.order; i++) {
                            // keep the filter tame: small reflection coefficients
                            int mag = (int)r.below(3);
                            int idx = r.below(2) ? mag : ((1 << bits) - 1 - mag);
                            F.coef[i] = (uint8_t)(idx & ((1 << bits) - 1));
                        }
                    }
                }
            }
        }
    }
}

void gen_sbr_stream(const jaad_synth_params& P, jaad_sbr_frame* out, uint32_t s)
{
    const int nch = P.channel_config == 2 ? 2 : 1;
    SplitMix64 r{P.seed ^ (0x5B5B5B5Bull + (uint64_t)(P.first_stream + s) * 0xD1B54A32D192ED03ull)};
    for (int i = 0; i < 4; i++) r.next();
    int lvl[2][64], qv[2][5], iid[34], icc[34];
    for (int b = 0; b < 34; b++) {
        iid[b] = (int)r.below(9) - 4;
        icc[b] = (int)r.below(8);
    }
    for (int c = 0; c < 2; c++) {
        for (int k = 0; k < 64; k++) lvl[c][k] = P.sbr_level - (int)r.below(5);
        for (int k = 0; k < 5; k++) qv[c][k] = 8 + (int)r.below(16);
    }
    int bal[64], qbal[5];  // coupled channel 1: balance walks (even values 0..24)
    for (int k = 0; k < 64; k++) bal[k] = 2 * (int)r.below(13);
    for (int k = 0; k < 5; k++) qbal[k] = 2 * (int)r.below(13);
    for (uint32_t fi = 0; fi < P.frames_per_stream; fi++) {
        jaad_sbr_frame& F = out[(size_t)s * P.frames_per_stream + fi];
        std::memset(&F, 0, sizeof F);
        // Header.java defaults (A/sbr/Header.java:12-22,44-60) with start 5 / stop 9 / xover 0
        F.hdr = jaad_sbr_header{1, 5, 9, 0, 2, 1, 2, 2, 2, 1, 1, 0};
        if (fi < P.nohdr_frames) continue;  // before the first header: no SBR data is read
        F.header_present = 1;
        // drawn first so that the other fields do not depend on the options (the default stream
        // is the same with and without them)
        const bool ups = P.upsample_percent && r.percent(P.upsample_percent);
        const bool coupled = nch == 2 && P.coupling_percent && r.percent(P.coupling_percent);
        if (ups) {  // the element's SBR data is missing or unusable this frame
            F.status = JAAD_SBR_UPSAMPLE;
            F.header_present = 0;
            continue;
        }
        F.coupling = coupled ? 1 : 0;
        for (int c = 0; c < nch; c++) {
            if (c == 1 && coupled) {  // Channel.couple (A/sbr/Channel.java:103-122), balance data
                jaad_sbr_channel& C1 = F.ch[1];
                const jaad_sbr_channel& C0 = F.ch[0];
                C1.frame_class = C0.frame_class;
                C1.L_E = C0.L_E;
                C1.L_Q = C0.L_Q;
                C1.bs_pointer = C0.bs_pointer;
                std::memcpy(C1.t_E, C0.t_E, sizeof C1.t_E);
                std::memcpy(C1.t_Q, C0.t_Q, sizeof C1.t_Q);
                std::memcpy(C1.f, C0.f, sizeof C1.f);
                std::memcpy(C1.invf_mode, C0.invf_mode, sizeof C1.invf_mode);
                const bool amp_res = !(C0.L_E == 1);
                for (int l = 0; l < C1.L_E; l++)
                    for (int k = 0; k < 64; k++) {  // E << delta: even, pan 0..24 (x2 at 1.5 dB)
                        bal[k] += 2 * ((int)r.below(3) - 1);
                        bal[k] = bal[k] < 0 ? 0 : (bal[k] > 24 ? 24 : bal[k]);
                        C1.E[l][k] = (int16_t)(amp_res ? bal[k] : 2 * bal[k]);
                    }
                for (int l = 0; l < C1.L_Q; l++)
                    for (int k = 0; k < 5; k++) {
                        qbal[k] += 2 * ((int)r.below(3) - 1);
                        qbal[k] = qbal[k] < 0 ? 0 : (qbal[k] > 24 ? 24 : qbal[k]);
                        C1.Q[l][k] = (int16_t)qbal[k];
                    }
                C1.add_harmonic_flag = (uint8_t)r.percent(30);
                if (C1.add_harmonic_flag)
                    for (int k = 0; k < 64; k++)
                        if (r.percent(5)) C1.add_harmonic |= 1ull << k;
                continue;
            }
            jaad_sbr_channel& C = F.ch[c];
            const int L_E = 1 + (int)r.below(2);  // FIXFIX: bs_num_env = 1 << (0|1)
            const int fres = (int)r.below(2);
            C.frame_class = 0;
            C.L_E = (uint8_t)L_E;
            C.L_Q = (uint8_t)(L_E > 1 ? 2 : 1);
            C.bs_pointer = 0;
            // envelope_time_border_vector / noise_floor_time_border_vector for FIXFIX (A/sbr/Channel.java:455-556)
            C.t_E[0] = 0;
            C.t_E[L_E] = 32;
            if (L_E == 2) C.t_E[1] = 16;
            C.t_Q[0] = 0;
            C.t_Q[1] = (uint8_t)(L_E == 1 ? 32 : 16);
            C.t_Q[2] = (uint8_t)(L_E == 1 ? 0 : 32);
            for (int l = 0; l < L_E; l++) C.f[l] = (uint8_t)fres;
            const bool amp_res = !(L_E == 1);  // amp_res 1 in the header; FIXFIX with one envelope -> 1.5 dB
            for (int l = 0; l < L_E; l++)
                for (int k = 0; k < 64; k++) {
                    int d = (int)r.below(3) - 1;
                    lvl[c][k] += d;
                    if (lvl[c][k] > P.sbr_level) lvl[c][k] = P.sbr_level;
                    if (lvl[c][k] < P.sbr_level - 6) lvl[c][k] = P.sbr_level - 6;
                    C.E[l][k] = (int16_t)(amp_res ? lvl[c][k] : 2 * lvl[c][k] + (int)r.below(2));
                }
            for (int l = 0; l < C.L_Q; l++)
                for (int k = 0; k < 5; k++) {
                    qv[c][k] += (int)r.below(5) - 2;
                    if (qv[c][k] < 0) qv[c][k] = 0;
                    if (qv[c][k] > 30) qv[c][k] = 30;
                    C.Q[l][k] = (int16_t)qv[c][k];
                }
            for (int k = 0; k < 5; k++) C.invf_mode[k] = (uint8_t)r.below(4);
            C.add_harmonic_flag = (uint8_t)r.percent(30);
            if (C.add_harmonic_flag)
                for (int k = 0; k < 64; k++)
                    if (r.percent(5)) C.add_harmonic |= 1ull << k;
        }
        if (P.sbr == 2 && nch == 1) {
            // PS: header every frame, IID mode 1 / ICC mode 1 (20 bands), no extension,
            // var_borders = 0 with 1 or 2 envelopes (PSImpl.java:103-134, 162-168)
            F.ps_present = 1;
            jaad_ps_frame& S = F.ps;
            S.iid_mode = 1;
            S.icc_mode = 1;
            S.nr_ipdopd_par = 0;
            const int ne = 1 + (int)r.below(2);
            S.num_env = (uint8_t)ne;
            for (int e = 0; e <= ne; e++) S.border[e] = (uint8_t)(e * 32 / ne);
            for (int e = 0; e < ne; e++)
                for (int b = 0; b < 20; b++) {
                    iid[b] += (int)r.below(3) - 1;
                    iid[b] = iid[b] < -7 ? -7 : (iid[b] > 7 ? 7 : iid[b]);
                    icc[b] += (int)r.below(3) - 1;
                    icc[b] = icc[b] < 0 ? 0 : (icc[b] > 7 ? 7 : icc[b]);
                    S.iid[e][b] = (int8_t)iid[b];
                    S.icc[e][b] = (int8_t)icc[b];
                }
        }
    }
}

}  // namespace

extern "C" {

void jaad_synth_default(int config_id, jaad_synth_params* p)
{
    std::memset(p, 0, sizeof(*p));
    p->seed = 0x4A41414400000000ull + (uint64_t)config_id;
    p->global_gain = 130;
    p->escape_permille = 1;
    p->common_window = 1;
    p->pns_state0 = 0x1F2E3D4Cu;  // ICStream.randomState initial value (A/syntax/ICStream.java:26)
    switch (config_id) {
    case 4:  // C4: HE-AAC v1 24 -> 48 kHz stereo, 32 768 frames = 128 streams x 256
        p->n_streams = 128;
        p->frames_per_stream = 256;
        p->sf_index = 6;
        p->channel_config = 2;
        p->ms_mode = 1;
        p->sbr = 1;
        p->sbr_level = 18;
        break;
    case 5:  // C5: HE-AAC v2 mono core -> SBR -> PS stereo, 262 144 frames = 2048 streams x 128
        p->n_streams = 2048;
        p->frames_per_stream = 128;
        p->sf_index = 6;
        p->channel_config = 1;
        p->sbr = 2;
        p->sbr_level = 18;
        break;
    case 1:  // C1: AAC-LC 44.1 kHz mono, one frame
        p->n_streams = 1;
        p->frames_per_stream = 1;
        p->sf_index = 4;
        p->channel_config = 1;
        break;
    case 3:  // C3: C2 + window switching + TNS in 50 % of ch-frames
        p->n_streams = 256;
        p->frames_per_stream = 256;
        p->sf_index = 3;
        p->channel_config = 2;
        p->window_switching = 1;
        p->tns_percent = 50;
        p->ms_mode = 1;
        break;
    default:  // C2: 65 536 AAC-LC 48 kHz stereo frames = 256 streams x 256, long windows
        p->n_streams = 256;
        p->frames_per_stream = 256;
        p->sf_index = 3;
        p->channel_config = 2;
        p->ms_mode = 1;
        break;
    }
}

int jaad_synth_generate(const jaad_synth_params* p, int16_t* q, uint8_t* sf, uint8_t* cb, jaad_ics_info* ics,
                        uint64_t* ms_used, jaad_tns* tns, uint32_t* stream_slot, uint32_t* frame_begin, int threads)
{
    if (!p || !q || !sf || !cb || !ics || !stream_slot || !frame_begin) return JAAD_ERR_INVALID_ARG;
    if (p->sf_index > 11 || (p->channel_config != 1 && p->channel_config != 2)) return JAAD_ERR_INVALID_ARG;
    if (p->channel_config == 2 && !ms_used) return JAAD_ERR_INVALID_ARG;
    if (p->first_stream && p->pns_percent) return JAAD_ERR_INVALID_ARG;
    Gen G{p, q, sf, cb, ics, ms_used, tns};
    const uint32_t ns = p->n_streams;
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > ns) threads = (int)(ns ? ns : 1);
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
        pool.emplace_back([&, t] {
            for (uint32_t s = t; s < ns; s += threads) gen_stream(G, s);
        });
    for (auto& th : pool) th.join();
    // static PNS LCG in parse order (stream-major, frame, channel): A/syntax/ICStream.java:26,247
    const int nch = p->channel_config == 2 ? 2 : 1;
    uint32_t rs = p->pns_state0;
    const size_t ncf = (size_t)ns * p->frames_per_stream * nch;
    for (size_t cf = 0; cf < ncf; cf++) {
        jaad_ics_info& ic = ics[cf];
        ic.pns_state = rs;
        if (!(ic.flags & JAAD_ICS_HAS_PNS)) continue;
        const bool is_short = ic.window_sequence == JAAD_EIGHT_SHORT_SEQUENCE;
        const short* off = is_short ? JAAD_SWB_OFFSET_SHORT_WINDOW[p->sf_index] : JAAD_SWB_OFFSET_LONG_WINDOW[p->sf_index];
        int glen[8], gn = 1;
        glen[0] = 1;
        if (is_short)
            for (int i = 0; i < 7; i++) {
                if (ic.grouping & (1u << i)) glen[gn - 1]++;
                else glen[gn++] = 1;
            }
        uint64_t steps = 0;
        for (int g = 0, idx = 0; g < gn; g++)
            for (int b = 0; b < ic.max_sfb; b++, idx++)
                if (cb[cf * 128 + idx] == JAAD_NOISE_HCB) steps += (uint64_t)glen[g] * (off[b + 1] - off[b]);
        for (uint64_t i = 0; i < steps; i++) rs = 1664525u * rs + 1013904223u;
    }
    for (uint32_t s = 0; s < ns; s++) {
        stream_slot[s] = s;
        frame_begin[s] = s * p->frames_per_stream;
    }
    frame_begin[ns] = ns * p->frames_per_stream;
    return JAAD_OK;
}

int jaad_synth_sbr(const jaad_synth_params* p, jaad_sbr_frame* out, int threads)
{
    if (!p || !out || (p->channel_config != 1 && p->channel_config != 2)) return JAAD_ERR_INVALID_ARG;
    const uint32_t ns = p->n_streams;
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > ns) threads = (int)(ns ? ns : 1);
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
        pool.emplace_back([&, t] {
            for (uint32_t s = t; s < ns; s += threads) gen_sbr_stream(*p, out, s);
        });
    for (auto& th : pool) th.join();
    return JAAD_OK;
}

}  // extern "C"
