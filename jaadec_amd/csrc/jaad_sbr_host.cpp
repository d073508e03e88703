// SBR host-side record builder: the parameter-only half of the reference's SBR path, evaluated in
// stream order on the host (A/ = aac/src/main/java/net/sourceforge/jaad/aac/).
//
//   FBT tables on header reset ........ A/sbr/SBR.java:125-158, A/sbr/FBT.java:29-416
//   patch construction ................. A/sbr/HFGeneration.java:247-309
//   chirp factors ...................... A/sbr/HFGeneration.java:199-245
//   envelope/noise dequantisation ...... A/sbr/NoiseEnvelope.java:190-344
//   l_A, S_mapped, S_index_mapped ...... A/sbr/HFAdjustment.java:20-80, 250-336
//   noise / sine index carry ........... A/sbr/HFAdjustment.java:143-237
//   prev-frame data .................... A/sbr/SBR.java:256-284
// The signal path (analysis, HF generation, gains, assembly, synthesis) is in jaad_sbr.hip.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "jaad_sbr.h"
#include "tables/jaad_sbr_tables.inc"

namespace jaad {
namespace {

enum { LO_RES = 0, HI_RES = 1, FIXFIX = 0, FIXVAR = 1, VARFIX = 2, VARVAR = 3 };
const int kFreq[12] = {96000, 88200, 64000, 48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000};

int find_bands(int warp, int bands, int a0, int a1)
{
    float div = (float)std::log(2.0);
    if (warp) div *= 1.3f;
    return (int)(bands * std::log((double)((float)a1 / (float)a0)) / div + 0.5);
}

float find_initial_power(int bands, int a0, int a1)
{
    return (float)std::pow((double)((float)a1 / (float)a0), (double)(1.0f / (float)bands));
}

// master frequency band table, bs_freq_scale == 0 (FBT.java:84-129)
bool master_fs0(SbrFbt& t, int k0, int k2, bool alter)
{
    if (k2 <= k0) return false;
    const int dk = alter ? 2 : 1;
    int nr = alter ? (((k2 - k0 + 2) >> 2) << 1) : (((k2 - k0) >> 1) << 1);
    nr = std::min(nr, 63);
    if (nr <= 0) return false;
    int vDk[64];
    for (int k = 0; k < nr; k++) vDk[k] = dk;
    int diff = k2 - (k0 + nr * dk);
    if (diff) {
        const int incr = diff > 0 ? -1 : 1;
        for (int k = diff > 0 ? nr - 1 : 0; diff; k += incr, diff += incr) vDk[k] -= incr;
    }
    t.f_master[0] = k0;
    for (int k = 1; k <= nr; k++) t.f_master[k] = t.f_master[k - 1] + vDk[k - 1];
    t.N_master = std::min(nr, 64);
    return true;
}

// geometric band steps of one region (FBT.java:181-189 / :215-223)
void region_steps(int* vDk, int nr, int a0, int a1, int count)
{
    const float q = find_initial_power(nr, a0, a1);
    float qk = (float)a0;
    int A1 = (int)(qk + 0.5f);
    for (int k = 0; k < count; k++) {
        const int A0 = A1;
        qk *= q;
        A1 = (int)(qk + 0.5f);
        vDk[k] = A1 - A0;
    }
}

// bs_freq_scale > 0 (FBT.java:150-256); bs_alter_scale is not used by the reference
bool master_fs(SbrFbt& t, int k0, int k2, int freq_scale)
{
    if (k2 <= k0) return false;
    static const int kBands[3] = {6, 5, 4};
    const int bands = kBands[freq_scale - 1];
    const bool two = (double)((float)k2 / (float)k0) > 2.2449;
    const int k1 = two ? k0 << 1 : k2;
    int vDk0[65] = {0}, vDk1[65] = {0}, vk0[65], vk1[65];
    const int nr0 = std::min(2 * find_bands(0, bands, k0, k1), 63);
    if (nr0 <= 0) return false;
    region_steps(vDk0, nr0, k0, k1, nr0 + 1);
    std::sort(vDk0, vDk0 + nr0);
    vk0[0] = k0;
    for (int k = 1; k <= nr0; k++) {
        vk0[k] = vk0[k - 1] + vDk0[k - 1];
        if (vDk0[k - 1] == 0) return false;
    }
    if (!two) {
        for (int k = 0; k <= nr0; k++) t.f_master[k] = vk0[k];
        t.N_master = std::min(nr0, 64);
        return true;
    }
    const int nr1 = std::min(2 * find_bands(1, bands, k1, k2), 63);
    region_steps(vDk1, nr1, k1, k2, nr1);
    if (vDk1[0] < vDk0[nr0 - 1]) {
        std::sort(vDk1, vDk1 + nr1 + 1);
        const int change = vDk0[nr0 - 1] - vDk1[0];
        vDk1[0] = vDk0[nr0 - 1];
        vDk1[nr1 - 1] -= change;
    }
    std::sort(vDk1, vDk1 + nr1);
    vk1[0] = k1;
    for (int k = 1; k <= nr1; k++) {
        vk1[k] = vk1[k - 1] + vDk1[k - 1];
        if (vDk1[k - 1] == 0) return false;
    }
    t.N_master = std::min(nr0 + nr1, 64);
    for (int k = 0; k <= nr0; k++) t.f_master[k] = vk0[k];
    for (int k = nr0 + 1; k <= t.N_master; k++) t.f_master[k] = vk1[k - nr0];
    return true;
}

bool derived_tables(SbrFbt& t, int xover, int noise_bands)  // FBT.java:259-320
{
    if (t.N_master <= xover) return false;
    t.N_high = t.N_master - xover;
    t.N_low = (t.N_high >> 1) + (t.N_high - ((t.N_high >> 1) << 1));
    t.n[0] = t.N_low;
    t.n[1] = t.N_high;
    for (int k = 0; k <= t.N_high; k++) t.f_table_res[HI_RES][k] = t.f_master[k + xover];
    t.M = t.f_table_res[HI_RES][t.N_high] - t.f_table_res[HI_RES][0];
    t.kx = t.f_table_res[HI_RES][0];
    if (t.kx > 32 || t.kx + t.M > 64) return false;
    const int minus = t.N_high & 1;
    for (int k = 0, i = 0; k <= t.N_low; k++) {
        if (k > 0) i = 2 * k - minus;
        t.f_table_res[LO_RES][k] = t.f_table_res[HI_RES][i];
    }
    t.N_Q = noise_bands == 0 ? 1 : std::min(5, std::max(1, find_bands(0, noise_bands, t.kx, t.k2)));
    for (int k = 0, i = 0; k <= t.N_Q; k++) {
        if (k > 0) i += (t.N_low - i) / (t.N_Q + 1 - k);
        t.f_table_noise[k] = t.f_table_res[LO_RES][i];
    }
    for (int k = 0; k < 64; k++) {
        t.table_map_k_to_g[k] = 0;
        for (int g = 0; g < t.N_Q; g++)
            if (t.f_table_noise[g] <= k && k < t.f_table_noise[g + 1]) {
                t.table_map_k_to_g[k] = g;
                break;
            }
    }
    return true;
}

void patches(SbrFbt& t, int sfi)  // HFGeneration.java:247-309
{
    int msb = t.k0, usb = t.kx, k = 0;
    const int goal = JAAD_SBR_GOAL_SB[sfi];
    t.noPatches = 0;
    if (goal < t.kx + t.M) {
        for (int i = 0; t.f_master[i] < goal; i++) k = i + 1;
    } else {
        k = t.N_master;
    }
    if (t.N_master == 0) {
        t.patchNoSubbands[0] = t.patchStartSubband[0] = 0;
        return;
    }
    int sb;
    do {
        int j = k + 1, odd;
        do {
            j--;
            sb = t.f_master[j];
            odd = (sb - 2 + t.k0) % 2;
        } while (sb > t.k0 - 1 + msb - odd);
        t.patchNoSubbands[t.noPatches] = std::max(sb - usb, 0);
        t.patchStartSubband[t.noPatches] = t.k0 - odd - t.patchNoSubbands[t.noPatches];
        if (t.patchNoSubbands[t.noPatches] > 0) {
            usb = msb = sb;
            t.noPatches++;
        } else {
            msb = t.kx;
        }
        if (t.f_master[k] - sb < 3) k = t.N_master;
    } while (sb != t.kx + t.M);
    if (t.patchNoSubbands[t.noPatches - 1] < 3 && t.noPatches > 1) t.noPatches--;
    t.noPatches = std::min(t.noPatches, 5);
}

void limiter_tables(SbrFbt& t)  // FBT.java:330-416
{
    t.f_table_lim[0][0] = t.f_table_res[LO_RES][0] - t.kx;
    t.f_table_lim[0][1] = t.f_table_res[LO_RES][t.N_low] - t.kx;
    t.N_L[0] = 1;
    for (int s = 1; s < 4; s++) {
        int lim[100] = {0}, pb[64] = {0};
        pb[0] = t.kx;
        for (int k = 1; k <= t.noPatches; k++) pb[k] = pb[k - 1] + t.patchNoSubbands[k - 1];
        for (int k = 0; k <= t.N_low; k++) lim[k] = t.f_table_res[LO_RES][k];
        for (int k = 1; k < t.noPatches; k++) lim[k + t.N_low] = pb[k];
        std::sort(lim, lim + t.noPatches + t.N_low);
        int k = 1, nrLim = t.noPatches + t.N_low - 1;
        if (nrLim < 0) return;
        auto is_border = [&](int v) {
            for (int i = 0; i <= t.noPatches; i++)
                if (v == pb[i]) return true;
            return false;
        };
        while (k <= nrLim) {
            const float oct = lim[k - 1] != 0 ? (float)lim[k] / (float)lim[k - 1] : 0.0f;
            if (oct < JAAD_SBR_LIMITER_COMPARE[s - 1]) {
                if (lim[k] != lim[k - 1] && is_border(lim[k])) {
                    if (is_border(lim[k - 1])) {
                        k++;
                    } else {
                        lim[k - 1] = t.f_table_res[LO_RES][t.N_low];
                        std::sort(lim, lim + t.noPatches + t.N_low);
                        nrLim--;
                    }
                    continue;
                }
                lim[k] = t.f_table_res[LO_RES][t.N_low];
                std::sort(lim, lim + nrLim);
                nrLim--;
            } else {
                k++;
            }
        }
        t.N_L[s] = nrLim;
        for (int l = 0; l <= nrLim; l++) t.f_table_lim[s][l] = lim[l] - t.kx;
    }
}

// counters of calculate_gain as the reference walks the limiter bands (HFAdjustment.java:264-323)
void band_maps(SbrFbt& t)
{
    std::memset(t.visited, 0, sizeof t.visited);
    for (int s = 0; s < 4; s++) {
        for (int f = 0; f < 2; f++) {
            int res = 0, noise = 0, hi = 0;
            for (int k = 0; k < t.N_L[s]; k++)
                for (int m = t.f_table_lim[s][k]; m < t.f_table_lim[s][k + 1]; m++) {
                    if (m < 0 || m >= 64) continue;
                    if (m + t.kx == t.f_table_noise[noise + 1]) noise++;
                    if (m + t.kx == t.f_table_res[f][res + 1]) res++;
                    if (m + t.kx == t.f_table_res[HI_RES][hi + 1]) hi++;
                    t.res_map[s][f][m] = res;
                    if (f == 0) {
                        t.noise_map[s][m] = noise;
                        t.hi_map[s][m] = hi;
                        t.visited[s][m] = 1;
                    }
                }
        }
    }
}

float mapNewBw(int mode, int prev)  // HFGeneration.java:199-223
{
    switch (mode) {
    case 1: return prev == 0 ? 0.6f : 0.75f;
    case 2: return 0.9f;
    case 3: return 0.98f;
    default: return prev == 1 ? 0.6f : 0.0f;
    }
}

bool header_differs(const jaad_sbr_header& a, const jaad_sbr_header& b)  // Header.java:70-78
{
    return a.start_freq != b.start_freq || a.stop_freq != b.stop_freq || a.freq_scale != b.freq_scale ||
           a.alter_scale != b.alter_scale || a.xover_band != b.xover_band || a.noise_bands != b.noise_bands;
}

}  // namespace

SbrHost::SbrHost(int out_sf_index) : out_sf_(out_sf_index)
{
    tabs_.reserve(kMaxTables);
    fbt_.reserve(kMaxTables);
    keys_.reserve(kMaxTables);
    // table 0: before the first SBR header (Channel.process_channel with sbr.hdr == null,
    // A/sbr/Channel.java:589-617) the analysis keeps 32 bands and nothing is generated or
    // adjusted: kx = 32, M = 0, no patch, no limiter band.  Its key never matches a header
    // (start_freq is a 4-bit field).
    auto t = std::make_unique<SbrFbt>();
    std::memset(t.get(), 0, sizeof(SbrFbt));
    t->kx = 32;
    t->max_src = -1;
    SbrTab g;
    std::memset(&g, 0, sizeof g);
    g.kx = 32;
    std::memset(g.src_p, 0xFF, sizeof g.src_p);
    jaad_sbr_header key;
    std::memset(&key, 0, sizeof key);
    key.start_freq = 0xFF;
    keys_.push_back(key);
    fbt_.push_back(std::move(t));
    tabs_.push_back(g);
}

bool SbrHost::header_changes(const jaad_sbr_header& a, const jaad_sbr_header& b) { return header_differs(a, b); }

void SbrHost::reset_slot(SbrHostSlot& s)
{
    std::memset(&s, 0, sizeof s);
    s.table = -1;
    for (auto& c : s.ch) c.prevEnvIsShort = -1;
}

// the frequency tables the bitstream parse needs (band counts, f_table_res): SBR.calc_sbr_tables
// (A/sbr/SBR.java:125-158) for a header at output rate index out_sf; false where the reference's
// table checks fail
bool sbr_tables_for_parse(int out_sf, const jaad_sbr_header& h, SbrFbt& t)
{
    std::memset(&t, 0, sizeof t);
    const int sfi = out_sf;
    if (sfi < 0 || sfi > 11) return false;
    t.k0 = JAAD_SBR_START_MIN[sfi] + JAAD_SBR_OFFSET[JAAD_SBR_OFFSET_INDEX[sfi]][h.start_freq & 15];
    if (h.stop_freq == 15) t.k2 = std::min(64, t.k0 * 3);
    else if (h.stop_freq == 14) t.k2 = std::min(64, t.k0 * 2);
    else t.k2 = std::min(64, JAAD_SBR_STOP_MIN[sfi] + JAAD_SBR_STOP_OFFSET[sfi][std::min((int)h.stop_freq, 13)]);
    const int fs = kFreq[sfi];
    const int span = t.k2 - t.k0;
    if ((fs >= 48000 && span > 32) || (fs <= 32000 && span > 48) || (fs > 32000 && fs < 48000 && span > 45))
        return false;
    const bool ok = h.freq_scale == 0 ? master_fs0(t, t.k0, t.k2, h.alter_scale != 0) : master_fs(t, t.k0, t.k2, h.freq_scale);
    return ok && derived_tables(t, h.xover_band, h.noise_bands);
}

int SbrHost::table_for(const jaad_sbr_header& h)
{
    std::lock_guard<std::mutex> lock(mu_);
    for (size_t i = 0; i < keys_.size(); i++)
        if (!header_differs(keys_[i], h)) return (int)i;
    if (keys_.size() >= kMaxTables) return -1;
    auto tp = std::make_unique<SbrFbt>();
    SbrFbt& t = *tp;
    std::memset(&t, 0, sizeof t);
    // SBR.calc_sbr_tables with bs_samplerate_mode = 1 (A/sbr/SBR.java:105,125-158)
    const int sfi = out_sf_;
    t.k0 = JAAD_SBR_START_MIN[sfi] + JAAD_SBR_OFFSET[JAAD_SBR_OFFSET_INDEX[sfi]][h.start_freq & 15];
    if (h.stop_freq == 15) t.k2 = std::min(64, t.k0 * 3);
    else if (h.stop_freq == 14) t.k2 = std::min(64, t.k0 * 2);
    else t.k2 = std::min(64, JAAD_SBR_STOP_MIN[sfi] + JAAD_SBR_STOP_OFFSET[sfi][std::min((int)h.stop_freq, 13)]);
    const int fs = kFreq[sfi];
    const int span = t.k2 - t.k0;
    if ((fs >= 48000 && span > 32) || (fs <= 32000 && span > 48) || (fs > 32000 && fs < 48000 && span > 45))
        return -1;
    const bool ok = h.freq_scale == 0 ? master_fs0(t, t.k0, t.k2, h.alter_scale != 0)
                                      : master_fs(t, t.k0, t.k2, h.freq_scale);
    if (!ok || !derived_tables(t, h.xover_band, h.noise_bands)) return -1;
    patches(t, sfi);
    t.max_src = -1;
    t.gen_cnt = 0;
    for (int i = 0; i < t.noPatches; i++) {
        t.gen_cnt += t.patchNoSubbands[i];
        if (t.patchNoSubbands[i] > 0) t.max_src = std::max(t.max_src, t.patchStartSubband[i] + t.patchNoSubbands[i] - 1);
    }
    limiter_tables(t);
    band_maps(t);
    return push_table(std::move(tp), h);
}

// the kernels' copy of a derived table set; appended under mu_ (held by the caller)
int SbrHost::push_table(std::unique_ptr<SbrFbt> tp, const jaad_sbr_header& h)
{
    if (keys_.size() >= kMaxTables) return -1;
    const SbrFbt& t = *tp;
    SbrTab g;
    std::memset(&g, 0, sizeof g);
    g.kx = (uint8_t)t.kx;
    g.M = (uint8_t)t.M;
    g.N_Q = (uint8_t)t.N_Q;
    g.N_high = (uint8_t)t.N_high;
    g.N_low = (uint8_t)t.N_low;
    g.n_lo = (uint8_t)t.n[0];
    g.n_hi = (uint8_t)t.n[1];
    for (int s = 0; s < 4; s++) {
        g.N_L[s] = (uint8_t)t.N_L[s];
        for (int k = 0; k <= t.N_L[s] && k < 64; k++) g.lim[s][k] = (uint8_t)t.f_table_lim[s][k];
        for (int m = 0; m < 64; m++) {
            g.res_map[s][0][m] = (uint8_t)t.res_map[s][0][m];
            g.res_map[s][1][m] = (uint8_t)t.res_map[s][1][m];
            g.noise_map[s][m] = (uint8_t)t.noise_map[s][m];
        }
    }
    std::memset(g.src_p, 0xFF, sizeof g.src_p);
    for (int i = 0, k = t.kx; i < t.noPatches; i++)
        for (int x = 0; x < t.patchNoSubbands[i]; x++, k++)
            if (k < 64) g.src_p[k] = (uint8_t)(t.patchStartSubband[i] + x);
    for (int k = 0; k < 64; k++) g.g_of_k[k] = (uint8_t)t.table_map_k_to_g[k];
    for (int f = 0; f < 2; f++)
        for (int k = 0; k <= t.n[f] && k < 64; k++) g.f_res[f][k] = (uint8_t)t.f_table_res[f][k];
    keys_.push_back(h);
    fbt_.push_back(std::move(tp));
    tabs_.push_back(g);
    return (int)tabs_.size() - 1;
}

int SbrHost::mixed_for(const jaad_sbr_header& h, const jaad_sbr_header& ph)
{
    const int a = table_for(h), b = table_for(ph);
    if (a < 0 || b < 0) return -1;
    if (a == b) return a;
    std::lock_guard<std::mutex> lock(mu_);
    for (size_t i = 0; i < mixed_keys_.size(); i++)
        if (!header_differs(mixed_keys_[i].first, h) && !header_differs(mixed_keys_[i].second, ph)) return mixed_idx_[i];
    const SbrFbt& N = *fbt_[a];
    const SbrFbt& O = *fbt_[b];
    // the reference would index outside its arrays (patches past band 63, limiter bands against
    // another M) or read sources the new analysis leaves zero: not reproduced
    if (N.M != O.M || N.kx + O.gen_cnt > 64 || O.max_src >= N.kx) return -1;
    auto tp = std::make_unique<SbrFbt>(N);
    SbrFbt& t = *tp;
    t.noPatches = O.noPatches;
    std::memcpy(t.patchNoSubbands, O.patchNoSubbands, sizeof t.patchNoSubbands);
    std::memcpy(t.patchStartSubband, O.patchStartSubband, sizeof t.patchStartSubband);
    t.max_src = O.max_src;
    t.gen_cnt = O.gen_cnt;
    std::memcpy(t.f_table_lim, O.f_table_lim, sizeof t.f_table_lim);
    std::memcpy(t.N_L, O.N_L, sizeof t.N_L);
    band_maps(t);
    jaad_sbr_header key = h;
    key.start_freq = 0xFF;  // the pure-table lookup must never find this one (a 4-bit field)
    const int idx = push_table(std::move(tp), key);
    if (idx < 0) return -1;
    mixed_keys_.push_back({h, ph});
    mixed_idx_.push_back(idx);
    return idx;
}

int SbrHost::take_header(SbrHostSlot& st, const jaad_sbr_header& h)
{
    if (!st.have_hdr) return JAAD_ERR_UNSUPPORTED;  // no patches or limiter bands yet
    if (!header_differs(h, st.hdr)) {                // the same tables: the other fields move
        st.hdr = h;
        return JAAD_OK;
    }
    const jaad_sbr_header ph = st.mixed ? st.phdr : st.hdr;
    const int idx = mixed_for(h, ph);
    if (idx < 0) return JAAD_ERR_UNSUPPORTED;
    st.mixed = header_differs(h, ph) ? 1 : 0;
    st.phdr = ph;
    st.hdr = h;
    st.table = idx;
    return JAAD_OK;
}

int SbrHost::frame(SbrHostSlot& st, const jaad_sbr_frame& fr, int nch, bool first, uint32_t slot, SbrRec* rec,
                   float* epool, uint32_t& epos, uint32_t e_base)
{
    bool reset = false;
    if (fr.header_present) {
        reset = !st.have_hdr || header_differs(fr.hdr, st.hdr);
        st.hdr = fr.hdr;
        st.have_hdr = 1;
        if (reset) {
            st.table = table_for(fr.hdr);
            st.mixed = 0;  // patch_construction and the limiter tables run with this reset
            if (st.table < 0) return JAAD_ERR_BITSTREAM;
        }
    }
    if (!st.have_hdr) {
        // no SBR header yet: SBR.decode marks the data valid without reading it and
        // process_channel only analyses and resynthesises the low band (A/sbr/SBR.java:179-184,
        // A/sbr/Channel.java:589-617); nothing of the parameter state moves (sbr_save_prev_data
        // runs only with a header, A/sbr/SBR2.java:150-153)
        for (int c = 0; c < nch; c++) {
            SbrRec& r = rec[c];
            std::memset(&r, 0, sizeof r);
            r.L_E = 1;
            r.t_E[1] = 32;  // one envelope over the frame: the HF stage copies rows 2..33
            r.table = kNoHeaderTable;
            r.first = first ? 1 : 0;
            r.slot = slot;
            r.kx_prev = (uint8_t)st.kx_prev;
            r.M_prev = (uint8_t)st.M_prev;
            r.e_off = e_base + epos;
            // X = the 32 analysis bands (Channel.java:604-613; rows l < t_E[0] none: t_E[0] = 0)
            r.blim = 32;
        }
        return JAAD_OK;
    }
    const bool coupled = nch == 2 && fr.coupling;
    const SbrFbt& t = *fbt_[st.table];
    const jaad_sbr_header& h = st.hdr;
    const int s_lim = h.limiter_bands & 3;
    for (int c = 0; c < nch; c++) {
        const jaad_sbr_channel& in = fr.ch[c];
        SbrHostCh& ch = st.ch[c];
        SbrRec& r = rec[c];
        std::memset(&r, 0, sizeof r);
        const int L_E = in.L_E, L_Q = in.L_Q;
        if (L_E < 1 || L_E > 5 || L_Q < 1 || L_Q > 2) return JAAD_ERR_BITSTREAM;
        for (int l = 0; l <= L_E; l++)
            if (in.t_E[l] > 38 || (l > 0 && in.t_E[l] < in.t_E[l - 1])) return JAAD_ERR_BITSTREAM;
        // envelope_time_border_vector: lead border <= 2*3, trail border >= 2*16 (Channel.java:455-542)
        if (in.t_E[0] > 6 || in.t_E[L_E] < 32) return JAAD_ERR_BITSTREAM;
        for (int l = 0; l < L_E; l++)
            if (in.f[l] > 1) return JAAD_ERR_BITSTREAM;
        r.L_E = (uint8_t)L_E;
        r.table = (uint16_t)st.table;
        r.lim_bands = (uint8_t)s_lim;
        r.flags = (uint8_t)((reset ? kSbrReset : 0) | (h.smoothing_mode ? 0 : kSbrSmooth) |
                            (h.interpol_freq ? kSbrInterpol : 0) | kSbrProcess);
        r.first = first ? 1 : 0;
        r.slot = slot;
        r.kx_prev = (uint8_t)st.kx_prev;
        r.M_prev = (uint8_t)st.M_prev;
        // X is zero from kx + M up (rows l < t_E[0]: kx_prev + M_prev, Channel.java:618-645)
        r.blim = (uint8_t)std::min(64, std::max(t.kx + t.M, st.kx_prev + st.M_prev));
        for (int l = 0; l <= L_E; l++) r.t_E[l] = in.t_E[l];
        for (int l = 0; l < L_E; l++) r.f[l] = in.f[l];
        r.lim_gain = JAAD_SBR_LIM_GAIN[h.limiter_gains & 3];

        // l_A (HFAdjustment.java:23-37)
        int l_A;
        if (in.frame_class == FIXFIX) l_A = -1;
        else if (in.frame_class == VARFIX) l_A = in.bs_pointer > 1 ? in.bs_pointer - 1 : -1;
        else l_A = in.bs_pointer == 0 ? -1 : L_E + 1 - in.bs_pointer;
        r.l_A = (int8_t)l_A;
        for (int l = 0; l < L_E; l++)
            if (l == l_A || l == ch.prevEnvIsShort) r.no_noise |= (uint8_t)(1u << l);

        // current_t_noise_band per envelope (HFAdjustment.java:260-262)
        for (int l = 0, tnb = 0; l < L_E; l++) {
            if (in.t_E[l + 1] > in.t_Q[tnb + 1]) tnb++;
            if (tnb > 1) return JAAD_ERR_BITSTREAM;
            r.tnb[l] = (uint8_t)tnb;
        }

        // chirp factors (HFGeneration.java:226-245)
        for (int i = 0; i < t.N_Q; i++) {
            float bw = mapNewBw(in.invf_mode[i], ch.invf_prev[i]);
            if (bw < ch.bwArray_prev[i]) bw = (bw * 0.75f) + (ch.bwArray_prev[i] * 0.25f);
            else bw = (bw * 0.90625f) + (ch.bwArray_prev[i] * 0.09375f);
            if (bw < 0.015625f) bw = 0.0f;
            if (bw >= 0.99609375f) bw = 0.99609375f;
            r.bw[i] = bw;
            ch.bwArray_prev[i] = bw;
            ch.invf_prev[i] = in.invf_mode[i];
        }

        // dequantisation: NoiseEnvelope.dequantChannel, or unmap for a coupled pair
        // (A/sbr/NoiseEnvelope.java:250-281, :299-344; SBR2.sbr_data :125-129)
        auto amp_of = [&](const jaad_sbr_channel& x) {  // Channel.sbr_envelope (A/sbr/Channel.java:130-133)
            return (!(x.L_E == 1 && x.frame_class == FIXFIX) && h.amp_res) ? 0 : 1;
        };
        r.e_off = e_base + epos;
        if (!coupled) {
            const int amp = amp_of(in);
            for (int l = 0; l < L_E; l++) {
                const int nb = t.n[in.f[l]];
                const int16_t* Er = in.E[l];
                float* out = epool + epos;
                for (int k = 0; k < nb; k++) {
                    const int E = Er[k];
                    const int e = E >> amp;
                    float v = 0.0f;
                    if (e >= 0 && e < 64) {
                        v = JAAD_SBR_E_DEQ[e];
                        if (amp != 0 && (E & 1) != 0) v = v * 1.414213562f;
                    }
                    out[k] = v;
                }
                epos += (uint32_t)nb;
            }
            for (int l = 0; l < L_Q; l++)
                for (int k = 0; k < t.N_Q; k++) {
                    const int q = in.Q[l][k];
                    const bool ok = q >= 0 && q <= 30;
                    r.q_div[l][k] = ok ? JAAD_SBR_Q_DIV[q] : 0.0f;
                    r.q_div2[l][k] = ok ? JAAD_SBR_Q_DIV2[q] : 0.0f;
                }
        } else {
            // both channels from channel 0's level and channel 1's balance, over channel 0's
            // envelopes (channel 1's grid is a copy of it, Channel.couple)
            const jaad_sbr_channel& c0 = fr.ch[0];
            const jaad_sbr_channel& c1 = fr.ch[1];
            const int amp0 = amp_of(c0), amp1 = amp_of(c1);
            for (int l = 0; l < c0.L_E; l++) {
                const int nb = t.n[c0.f[l]];
                float* out = epool + epos;
                for (int k = 0; k < nb; k++) {
                    const int ch0E = c0.E[l][k];
                    const int exp0 = (ch0E >> amp0) + 1;
                    const int exp1 = c1.E[l][k] >> amp1;
                    float v = 0.0f;
                    if (!(exp0 < 0 || exp0 >= 64 || exp1 < 0 || exp1 > 24)) {
                        float tmp = JAAD_SBR_E_DEQ[exp0];
                        // tmp *= 1.414213562: a double literal, so the product is rounded once
                        // from double (unlike dequantChannel's float constant)
                        if (amp0 != 0 && (ch0E & 1) != 0) tmp = (float)((double)tmp * 1.414213562);
                        v = tmp * JAAD_SBR_E_PAN[c == 0 ? exp1 : 24 - exp1];
                    }
                    out[k] = v;
                }
                epos += (uint32_t)nb;
            }
            const float(*qd)[13] = c == 0 ? JAAD_SBR_Q_DIV_LEFT : JAAD_SBR_Q_DIV_RIGHT;
            const float(*qd2)[13] = c == 0 ? JAAD_SBR_Q_DIV2_LEFT : JAAD_SBR_Q_DIV2_RIGHT;
            for (int l = 0; l < c0.L_Q; l++)
                for (int k = 0; k < t.N_Q; k++) {
                    const int q0 = c0.Q[l][k], q1 = c1.Q[l][k];
                    const bool ok = !((q0 < 0 || q0 > 30) || (q1 < 0 || q1 > 24));
                    r.q_div[l][k] = ok ? qd[q0][q1 >> 1] : 0.0f;
                    r.q_div2[l][k] = ok ? qd2[q0][q1 >> 1] : 0.0f;
                }
        }

        // sinusoids: bs_add_harmonic cleared, then N_high flags (SBR2.java:63-72, SBR.java:249-254)
        const uint64_t hmask = t.N_high >= 64 ? ~0ull : ((1ull << t.N_high) - 1);
        const uint64_t harm = in.add_harmonic_flag ? (in.add_harmonic & hmask) : 0;  // bit n = bs_add_harmonic[n]
        const bool any_harm = harm != 0;
        auto hbit = [](uint64_t m, int b) { return b >= 0 && b < 64 ? (int)((m >> b) & 1u) : 0; };
        auto s_mapped = [&](int l, int band) {  // get_S_mapped (HFAdjustment.java:46-80)
            if (in.f[l] == HI_RES) {
                if (l >= l_A || (hbit(ch.add_harmonic_prev, band) && ch.add_harmonic_flag_prev)) return hbit(harm, band);
                return 0;
            }
            const int odd = (t.N_high & 1) ? 1 : 0;
            for (int b = 2 * band - odd; b < 2 * (band + 1) - odd; b++)
                if (l >= l_A || (hbit(ch.add_harmonic_prev, b) && ch.add_harmonic_flag_prev))
                    if (hbit(harm, b)) return 1;
            return 0;
        };
        for (int l = 0; l < L_E && any_harm; l++) {  // no sinusoid flag set: both masks are 0
            uint64_t mi = 0, mm = 0;
            for (int m = 0; m < t.M && m < 64; m++) {
                if (!t.visited[s_lim][m]) continue;
                const int hb = t.hi_map[s_lim][m];
                if (l >= l_A || (hbit(ch.add_harmonic_prev, hb) && ch.add_harmonic_flag_prev))
                    if (m + t.kx == (t.f_table_res[HI_RES][hb + 1] + t.f_table_res[HI_RES][hb]) >> 1 && hbit(harm, hb))
                        mi |= 1ull << m;
                if (s_mapped(l, t.res_map[s_lim][in.f[l]][m])) mm |= 1ull << m;
            }
            r.s_index[l] = mi;
            r.s_mapped[l] = mm;
        }

        // noise / sine table indices (HFAdjustment.java:151-158, 206, 227, 236-237)
        const int rows = in.t_E[L_E] - in.t_E[0];
        const int n0 = reset ? 0 : ch.index_noise_prev;
        r.noise0 = (uint16_t)n0;
        r.sine0 = (uint8_t)ch.psi_is_prev;
        ch.index_noise_prev = (n0 + rows * t.M) & 511;
        ch.psi_is_prev = (ch.psi_is_prev + rows) & 3;
        // G/Q ring position (HFAdjustment.java:166-173, 229-232)
        const int gq0 = reset ? 4 : ch.gq_index;
        r.gq0 = (uint8_t)gq0;
        ch.gq_index = (gq0 + rows) % 5;

        // sbr_save_prev_data (SBR.java:256-284)
        ch.add_harmonic_prev = harm & ((1ull << 49) - 1);
        ch.add_harmonic_flag_prev = in.add_harmonic_flag;
        ch.prevEnvIsShort = (l_A == L_E) ? 0 : -1;

        // kSbrDep: the frame reads the high band frame f-1 left in Xsbr rows 32..39 (its rows
        // 0..7 here, SBR.sbr_save_matrix A/sbr/SBR.java:286-300), which the frame-parallel HF
        // pass does not have (sbr_hf_kernel): a source band at or above kx_prev (auto_correlation
        // and the generation read rows 0..39 of it, A/sbr/HFGeneration.java:100-159,56-85), or,
        // when frame f-1 adjusted rows 34.. (its last border past slot 32), rows 2..7 of bands
        // [kx_prev, kx) going out as X (kx raised, Channel.java:619-645) or of a band no patch
        // generates (patch_construction dropped its last patch) entering estimate_current_envelope
        if (!first && (t.max_src >= st.kx_prev || (ch.last_prev > 32 && (t.kx > st.kx_prev || t.gen_cnt < t.M))))
            r.flags |= kSbrDep;
        ch.last_prev = in.t_E[L_E];
    }
    st.kx_prev = t.kx;
    st.M_prev = t.M;
    return JAAD_OK;
}

}  // namespace jaad
