// Host bitstream front end (include/jaad_parse.h): raw_data_block -> jaad_gpu.h records.
//
// Follows the reference's parse (A/ = aac/src/main/java/net/sourceforge/jaad/aac/), element by
// element, with the same validity checks; where the reference would throw (AACException,
// EOSException, or an ArrayIndexOutOfBounds its tables would raise) the frame is rejected
// with JAAD_ERR_BITSTREAM / JAAD_ERR_EOS / JAAD_ERR_UNSUPPORTED.  The parser's state is left as
// it was, except after JAAD_ERR_EOS, where it moves as far as the reference's reads got
// (parse_frame).  SBR/PS extension payloads go to jaad_parse_sbr.cpp.
#include "../../include/jaad_parse.h"

#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "jaad_parse_internal.h"
#include "tables/jaad_huffman_tables.inc"
#include "tables/jaad_tables.inc"

namespace jaad {
namespace parse {

// ------------------------------------------------------------------------------------------
// Huffman codebooks (A/huffman/Codebooks.java rows {length, codeword, values...}) as two-level
// lookup tables over the next `maxlen` bits.  For every valid codeword the result is the row
// Huffman.findOffset's linear scan (A/huffman/Huffman.java:15-28) stops at; a bit pattern that
// no codeword prefixes (the scan would run off the table) is an error.
// ------------------------------------------------------------------------------------------
struct Lut {
    int maxlen = 0, pbits = 0;
    std::vector<uint32_t> e;  // primary [1<<pbits], then secondaries; entry: len<<16 | row,
                              // 0x80000000 | base of a secondary table, or 0xFFFFFFFF invalid
    void build(const int* rows, int nrows, int stride)
    {
        maxlen = 0;
        for (int i = 0; i < nrows; i++) maxlen = rows[i * stride] > maxlen ? rows[i * stride] : maxlen;
        pbits = maxlen < 10 ? maxlen : 10;
        const int sbits = maxlen - pbits;
        e.assign((size_t)1 << pbits, 0xFFFFFFFFu);
        for (int i = 0; i < nrows; i++) {
            const int len = rows[i * stride];
            const uint32_t cw = (uint32_t)rows[i * stride + 1];
            const uint32_t ent = ((uint32_t)len << 16) | (uint32_t)i;
            if (len <= pbits) {
                const uint32_t lo = cw << (pbits - len), n = 1u << (pbits - len);
                for (uint32_t k = 0; k < n; k++) e[lo + k] = ent;
            } else {
                const uint32_t pre = cw >> (len - pbits);
                if (e[pre] == 0xFFFFFFFFu) {
                    e[pre] = 0x80000000u | (uint32_t)e.size();
                    e.resize(e.size() + ((size_t)1 << sbits), 0xFFFFFFFFu);
                }
                const uint32_t base = e[pre] & 0x7FFFFFFFu;
                const int rest = len - pbits;
                const uint32_t lo = (cw & ((1u << rest) - 1u)) << (sbits - rest), n = 1u << (sbits - rest);
                for (uint32_t k = 0; k < n; k++) e[base + lo + k] = ent;
            }
        }
    }
    // decode() on a register window (the caller keeps >= maxlen bits in it)
    int decode(BitReader::Window& br) const
    {
        const uint32_t peek = br.peek(maxlen);
        uint32_t ent = e[peek >> (maxlen - pbits)];
        if (ent != 0xFFFFFFFFu && (ent & 0x80000000u))
            ent = e[(ent & 0x7FFFFFFFu) + (peek & ((1u << (maxlen - pbits)) - 1u))];
        if (ent == 0xFFFFFFFFu) return br.left() < maxlen ? -2 : -1;
        const int len = (int)(ent >> 16);
        if (br.left() < len) return -2;
        br.skip(len);
        return (int)(ent & 0xFFFFu);
    }
    // row index, or -1 (no codeword) / -2 (bitstream ended)
    int decode(BitReader& br) const
    {
        const uint32_t peek = br.peek(maxlen);
        uint32_t ent = e[peek >> (maxlen - pbits)];
        if (ent != 0xFFFFFFFFu && (ent & 0x80000000u))
            ent = e[(ent & 0x7FFFFFFFu) + (peek & ((1u << (maxlen - pbits)) - 1u))];
        if (ent == 0xFFFFFFFFu) return br.left() < maxlen ? -2 : -1;
        const int len = (int)(ent >> 16);
        if (br.left() < len) return -2;
        br.skip(len);
        return (int)(ent & 0xFFFFu);
    }
};

struct Books {
    Lut spec[11], sf;
    const int* rows[11];
    int stride[11];
};

const Books& books()
{
    static Books B;
    static std::once_flag once;
    std::call_once(once, [] {
        const int* r[11] = {&JAAD_HCB1[0][0], &JAAD_HCB2[0][0], &JAAD_HCB3[0][0], &JAAD_HCB4[0][0], &JAAD_HCB5[0][0],
                            &JAAD_HCB6[0][0], &JAAD_HCB7[0][0], &JAAD_HCB8[0][0], &JAAD_HCB9[0][0], &JAAD_HCB10[0][0],
                            &JAAD_HCB11[0][0]};
        const int n[11] = {81, 81, 81, 81, 81, 81, 64, 64, 169, 169, 289};
        for (int i = 0; i < 11; i++) {
            B.rows[i] = r[i];
            B.stride[i] = i < 4 ? 6 : 4;
            B.spec[i].build(r[i], n[i], B.stride[i]);
        }
        B.sf.build(&JAAD_HCB_SF[0][0], 121, 3);
    });
    return B;
}

// ------------------------------------------------------------------------------------------
// ICS parse
// ------------------------------------------------------------------------------------------
struct IcsInfo {  // ICSInfo after decode / setCommonData
    int seq = 0, shape = 0, max_sfb = 0, grouping = 0;
    int ngroups = 1, glen[8] = {1};
};

// ICSInfo.decode (A/syntax/ICSInfo.java:86-119); prediction data is not part of AAC LC
// (readPredictionData throws for every other profile, :122-138).  `shape_state` (the channel's
// windowShape[CURRENT]) takes the new shape as soon as its bit is read, as the reference's field
// does: a frame that ends later in its bitstream (EOSException) has moved it already (:90-91).
int read_ics_info(BitReader& br, const Cfg& C, IcsInfo& I, int* shape_state)
{
    if (br.left() < 4) return JAAD_ERR_EOS;
    br.skip(1);  // ics_reserved_bit
    I.seq = (int)br.read(2);
    I.shape = (int)br.read(1);
    if (shape_state) *shape_state = I.shape;
    I.ngroups = 1;
    I.glen[0] = 1;
    I.grouping = 0;
    if (I.seq == JAAD_EIGHT_SHORT_SEQUENCE) {
        if (br.left() < 11) return JAAD_ERR_EOS;
        I.max_sfb = (int)br.read(4);
        for (int i = 0; i < 7; i++) {
            if (br.read(1)) {
                I.glen[I.ngroups - 1]++;
                I.grouping |= 1 << i;
            } else {
                I.glen[I.ngroups++] = 1;
            }
        }
        if (I.max_sfb > C.nswb_s) return JAAD_ERR_BITSTREAM;
    } else {
        if (br.left() < 6) return JAAD_ERR_EOS;
        I.max_sfb = (int)br.read(6);
        if (br.left() < 1) return JAAD_ERR_EOS;
        if (br.read(1)) return JAAD_ERR_UNSUPPORTED;  // predictor_data_present: AAC Main / LTP only
        if (I.max_sfb > C.nswb_l) return JAAD_ERR_BITSTREAM;
    }
    return br.overrun() ? JAAD_ERR_EOS : JAAD_OK;
}

// ICStream.decode (A/syntax/ICStream.java:60-111) of one channel into its records.
// State moves as the reference's does while it reads, so that a frame whose bitstream ends early
// (JAAD_ERR_EOS: the reference's EOSException, which Decoder.decodeFrame swallows) leaves what the
// next frame sees: `shape_state` takes the window shape once its bit is read (non-common window),
// and `pns` (the static randomState) has advanced over the noise bands decodeSpectralData
// reached before the read that ran out (A/syntax/ICStream.java:222-275: bands in order, a noise
// band consuming its LCG steps without reading bits).
// `prev_shape` is ICSInfo.windowShape[CURRENT] of the previous frame of this channel.
int read_ics(BitReader& br, const Cfg& C, bool common_window, IcsInfo& I, int prev_shape, int* shape_state,
             uint32_t& pns, ChOut& o)
{
    const Books& B = books();
    if (br.left() < 8) return JAAD_ERR_EOS;
    const int global_gain = (int)br.read(8);
    if (!common_window) {
        const int st = read_ics_info(br, C, I, shape_state);
        if (st) return st;
    }
    const bool is_short = I.seq == JAAD_EIGHT_SHORT_SEQUENCE;
    const short* swb = is_short ? JAAD_SWB_OFFSET_SHORT_WINDOW[C.sf_index] : JAAD_SWB_OFFSET_LONG_WINDOW[C.sf_index];
    const int nswb = is_short ? C.nswb_s : C.nswb_l;
    const int max_sfb = I.max_sfb;

    // ---- section data (decodeSectionData, :113-146)
    uint8_t cb[128] = {0};
    uint8_t sect_end[128] = {0};
    {
        const int bits = is_short ? 3 : 5, esc = (1 << bits) - 1;
        int idx = 0;
        for (int g = 0; g < I.ngroups; g++) {
            for (int k = 0; k < max_sfb;) {
                int end = k;
                if (br.left() < 4) return JAAD_ERR_EOS;
                const int c = (int)br.read(4);
                if (c == 12) return JAAD_ERR_BITSTREAM;  // "invalid huffman codebook: 12"
                int incr;
                do {
                    if (br.left() < bits) return JAAD_ERR_EOS;
                    incr = (int)br.read(bits);
                    end += incr;
                } while (incr == esc);
                if (end > max_sfb) return JAAD_ERR_BITSTREAM;  // "too many bands"
                for (; k < end; k++, idx++) {
                    cb[idx] = (uint8_t)c;
                    sect_end[idx] = (uint8_t)end;
                }
            }
        }
    }
    // ---- scalefactors (decodeScaleFactors, :172-220) -> table index - 100
    uint8_t sf[128] = {0};
    int has_pns = 0, has_is = 0;
    {
        int off0 = global_gain, off1 = global_gain - 90, off2 = 0;
        bool noise_flag = true;
        for (int g = 0, idx = 0; g < I.ngroups; g++) {
            for (int s = 0; s < max_sfb;) {
                const int end = sect_end[idx];
                const int c = cb[idx];
                for (; s < end; s++, idx++) {
                    if (c == JAAD_ZERO_HCB) {
                        sf[idx] = 0;
                        continue;
                    }
                    int d;
                    if (c == JAAD_NOISE_HCB && noise_flag) {
                        if (br.left() < 9) return JAAD_ERR_EOS;
                        d = (int)br.read(9) - 256;
                        noise_flag = false;
                    } else {
                        const int r = B.sf.decode(br);
                        if (r < 0) return r == -2 ? JAAD_ERR_EOS : JAAD_ERR_BITSTREAM;
                        d = JAAD_HCB_SF[r][2] - 60;
                    }
                    if (c == JAAD_INTENSITY_HCB || c == JAAD_INTENSITY_HCB2) {
                        off2 += d;
                        const int t = off2 < -155 ? -155 : (off2 > 100 ? 100 : off2);
                        sf[idx] = (uint8_t)(100 - t);  // SCALEFACTOR_TABLE[-t + 200]
                        has_is = 1;
                    } else if (c == JAAD_NOISE_HCB) {
                        off1 += d;
                        const int t = off1 < -100 ? -100 : (off1 > 155 ? 155 : off1);
                        sf[idx] = (uint8_t)(t + 100);  // -SCALEFACTOR_TABLE[t + 200]
                        has_pns = 1;
                    } else {
                        off0 += d;
                        if (off0 > 255) return JAAD_ERR_BITSTREAM;  // "scalefactor out of range"
                        if (off0 < 0) return JAAD_ERR_BITSTREAM;    // (table index < 100: outside the sf range)
                        sf[idx] = (uint8_t)off0;                      // SCALEFACTOR_TABLE[off0 - 100 + 200]
                    }
                }
            }
        }
    }
    // ---- pulse data (:17, :148-170): parsed and, as in the reference, not applied -- except in
    // spec mode (cfg.tns_mode == JAAD_TNS_SPEC, the "spec tools" switch of SURVEY 8(f)-4), where
    // ISO/IEC 14496-3 4.6.3.3 adds the pulses to the quantised values below
    int pulse_n = 0, pulse_off[4] = {0, 0, 0, 0}, pulse_amp[4] = {0, 0, 0, 0};
    if (br.left() < 1) return JAAD_ERR_EOS;
    if (br.read(1)) {
        if (is_short) return JAAD_ERR_BITSTREAM;  // "pulse data not allowed for short frames"
        if (br.left() < 8) return JAAD_ERR_EOS;
        const int count = (int)br.read(2) + 1;
        const int start = (int)br.read(6);
        if (start >= nswb) return JAAD_ERR_BITSTREAM;
        int offs = swb[start];
        for (int i = 0; i < count; i++) {
            if (br.left() < 9) return JAAD_ERR_EOS;
            offs += (int)br.read(5);
            pulse_amp[i] = (int)br.read(4);
            pulse_off[i] = offs;
            if (i > 0 && offs > 1023) return JAAD_ERR_BITSTREAM;
        }
        pulse_n = count;
    }
    // ---- TNS data (TNS.decode, A/tools/TNS.java:35-61)
    jaad_tns tns;
    std::memset(&tns, 0, sizeof tns);
    if (br.left() < 1) return JAAD_ERR_EOS;
    const bool tns_present = br.read(1) != 0;
    if (tns_present) {
        const int nwin = is_short ? 8 : 1;
        const int b0 = is_short ? 1 : 2, b1 = is_short ? 4 : 6, b2 = is_short ? 3 : 5;
        for (int w = 0; w < nwin; w++) {
            if (br.left() < b0) return JAAD_ERR_EOS;
            const int nf = (int)br.read(b0);
            if (!nf) continue;
            if (br.left() < 1) return JAAD_ERR_EOS;
            const int res = (int)br.read(1);
            for (int f = 0; f < nf; f++) {
                if (br.left() < b1 + b2) return JAAD_ERR_EOS;
                jaad_tns_filter& F = tns.filt[tns.n_filters < 8 ? tns.n_filters : 7];
                if (tns.n_filters >= 8) return JAAD_ERR_BITSTREAM;
                tns.n_filters++;
                F.window = (uint8_t)w;
                F.length = (uint8_t)br.read(b1);
                const int order = (int)br.read(b2);
                if (order > 20) return JAAD_ERR_BITSTREAM;  // "TNS filter out of range"
                F.order = (uint8_t)order;
                F.flags = (uint8_t)(res << 1);
                if (order) {
                    if (br.left() < 2) return JAAD_ERR_EOS;
                    const int dir = (int)br.read(1), comp = (int)br.read(1);
                    const int len = res + 3 - comp;
                    F.flags = (uint8_t)(dir | (res << 1) | (comp << 2));
                    for (int i = 0; i < order; i++) {
                        if (br.left() < len) return JAAD_ERR_EOS;
                        F.coef[i] = (uint8_t)br.read(len);
                    }
                }
            }
        }
    }
    // ---- gain control: AAC SSR only
    if (br.left() < 1) return JAAD_ERR_EOS;
    if (br.read(1)) return JAAD_ERR_UNSUPPORTED;

    // ---- spectral data (decodeSpectralData, :222-275): quantised values, window-major
    int16_t q[1024];
    std::memset(q, 0, sizeof q);
    uint64_t noise_steps = 0;
    auto lcg = [&]() {  // the static LCG advances once per noise bin (ICStream.java:247)
        for (uint64_t i = 0; i < noise_steps; i++) pns = 1664525u * pns + 1013904223u;
    };
    auto eos = [&]() {  // the bands before this one are done, noise bands included
        lcg();
        return JAAD_ERR_EOS;
    };
    BitReader::Window bw = br.window();  // (br's position is handed back after the loop)
    for (int g = 0, idx = 0, group_off = 0; g < I.ngroups; g++) {
        const int gl = I.glen[g];
        for (int s = 0; s < max_sfb; s++, idx++) {
            const int c = cb[idx];
            const int width = swb[s + 1] - swb[s];
            if (c == JAAD_ZERO_HCB || c == JAAD_INTENSITY_HCB || c == JAAD_INTENSITY_HCB2) continue;
            if (c == JAAD_NOISE_HCB) {
                noise_steps += (uint64_t)gl * (uint64_t)width;
                continue;
            }
            if (c > JAAD_ESCAPE_HCB) return JAAD_ERR_BITSTREAM;  // "unknown spectral codebook"
            const Lut& L = B.spec[c - 1];
            const int* rows = B.rows[c - 1];
            const int stride = B.stride[c - 1];
            const int num = c >= JAAD_FIRST_PAIR_HCB ? 2 : 4;
            const bool unsigned_cb = c == 3 || c == 4 || c == 7 || c == 8 || c == 9 || c == 10 || c == 11;
            for (int w = 0; w < gl; w++) {
                const int off = group_off + w * 128 + swb[s];
                for (int k = 0; k < width; k += num) {
                    bw.need(L.maxlen + 4);  // the codeword and its sign bits
                    const int r = L.decode(bw);
                    if (r < 0) return r == -2 ? eos() : JAAD_ERR_BITSTREAM;
                    int v[4];
                    for (int j = 0; j < num; j++) v[j] = rows[r * stride + 2 + j];
                    if (unsigned_cb) {  // Huffman.signValues (:30-37): one sign bit per nonzero value
                        int nz = 0;
                        for (int j = 0; j < num; j++) nz += v[j] != 0;
                        if (bw.left() < nz) return eos();
                        uint32_t bits = nz ? bw.read(nz) << (32 - nz) : 0u;  // next sign bit on top
                        for (int j = 0; j < num; j++) {  // (branch-free: the bits are data)
                            const uint32_t has = v[j] != 0;
                            const bool neg = (bits >> 31) & has;
                            bits <<= has;
                            v[j] = neg ? -v[j] : v[j];
                        }
                    }
                    if (c == JAAD_ESCAPE_HCB)  // Huffman.getEscape (:39-50)
                        for (int j = 0; j < 2; j++) {
                            if (v[j] != 16 && v[j] != -16) continue;
                            // escape_sequence prefix: n = 4 + the 1-bits before the first 0-bit, read
                            // bit by bit in the reference -- counted at once here with the same
                            // outcomes (EOS when the bits end first, an error at the 9th 1-bit)
                            bw.need(9 + 13);  // the escape prefix and its value bits
                            const int avail = bw.left() < 9 ? (int)bw.left() : 9;
                            const int ones = avail > 0 ? __builtin_clz(~(bw.peek(avail) << (32 - avail))) : 0;
                            if (ones >= 9) return JAAD_ERR_BITSTREAM;  // |q| > 8191: beyond IQ_TABLE
                            if (ones == avail) return eos();            // no 0-bit before the end
                            bw.skip(ones + 1);
                            const int n = 4 + ones;
                            if (bw.left() < n) return eos();
                            const int m = (int)bw.read(n) | (1 << n);
                            // IQ_TABLE has 8191 entries (A/syntax/IQTable.java): |q| <= 8190
                            if (m > 8190) return JAAD_ERR_BITSTREAM;
                            v[j] = v[j] < 0 ? -m : m;
                        }
                    for (int j = 0; j < num; j++)
                        if (k + j < width) q[off + k + j] = (int16_t)v[j];
                }
            }
        }
        group_off += gl << 7;
    }
    br.commit(bw);
    if (br.overrun()) return JAAD_ERR_EOS;
    if (C.cfg.tns_mode == JAAD_TNS_SPEC)  // spec-mode pulse tool (4.6.3.3, long windows only)
        for (int i = 0; i < pulse_n; i++) {
            const int k = pulse_off[i];
            if (k > 1023) return JAAD_ERR_BITSTREAM;  // the first offset is not range-checked above
            const int v = q[k] > 0 ? q[k] + pulse_amp[i] : q[k] - pulse_amp[i];
            if (v > 8190 || v < -8190) return JAAD_ERR_BITSTREAM;  // beyond IQ_TABLE
            q[k] = (int16_t)v;
        }

    // ---- records
    std::memcpy(o.q, q, sizeof q);
    std::memcpy(o.sf, sf, 128);
    std::memcpy(o.cb, cb, 128);
    jaad_ics_info& ic = *o.ics;
    std::memset(&ic, 0, sizeof ic);
    ic.window_sequence = (uint8_t)I.seq;
    ic.window_shape = (uint8_t)I.shape;
    ic.window_shape_prev = (uint8_t)prev_shape;
    ic.max_sfb = (uint8_t)max_sfb;
    ic.grouping = (uint8_t)I.grouping;
    ic.flags = (uint8_t)((has_pns ? JAAD_ICS_HAS_PNS : 0) | (has_is ? JAAD_ICS_HAS_IS : 0) |
                         (tns_present ? JAAD_ICS_TNS : 0) | (common_window ? JAAD_ICS_COMMON_WINDOW : 0));
    ic.pns_state = pns;
    lcg();
    if (o.tns) *o.tns = tns;
    return JAAD_OK;
}

}  // namespace parse
}  // namespace jaad

using namespace jaad::parse;

struct jaad_parser {
    Cfg C;
    ParseState st;  // st.sbr: the SBR state of channel element 0
    // multichannel HE-AAC: the SBR state of channel elements 1.. (each ChannelElement owns its SBR,
    // A/syntax/ChannelElement.java:39-74); empty otherwise
    std::vector<SbrParseState> sbr_el;
};

namespace {

int sf_counts(int sf_index, Cfg& C)
{
    if (sf_index < 0 || sf_index > 11) return JAAD_ERR_UNSUPPORTED;
    C.sf_index = sf_index;
    C.nswb_l = JAAD_SWB_LONG_WINDOW_COUNT[sf_index];
    C.nswb_s = JAAD_SWB_SHORT_WINDOW_COUNT[sf_index];
    return JAAD_OK;
}

// DSE (A/syntax/DSE.java:37-48)
int skip_dse(BitReader& br)
{
    if (br.left() < 9) return JAAD_ERR_EOS;
    const bool align = br.read(1) != 0;
    int count = (int)br.read(8);
    if (count == 255) {
        if (br.left() < 8) return JAAD_ERR_EOS;
        count += (int)br.read(8);
    }
    if (align) br.byte_align();
    if (br.left() < 8 * count) return JAAD_ERR_EOS;
    br.skip(8 * count);
    return JAAD_OK;
}

// PCE (A/syntax/PCE.java:110-160): read and dropped
int skip_pce(BitReader& br)
{
    if (br.left() < 2 + 4 + 4 + 4 + 4 + 2 + 3 + 4) return JAAD_ERR_EOS;
    br.skip(2 + 4);  // profile, SampleFrequency.decode (4 bits, A/SampleFrequency.java:112-115)
    const int nfront = (int)br.read(4), nside = (int)br.read(4), nback = (int)br.read(4);
    const int nlfe = (int)br.read(2), nassoc = (int)br.read(3), ncc = (int)br.read(4);
    if (br.read(1)) br.skip(4);
    if (br.read(1)) br.skip(4);
    if (br.read(1)) br.skip(3);
    br.skip(5 * (nfront + nside + nback) + 4 * nlfe + 4 * nassoc + 5 * ncc);
    br.byte_align();
    if (br.left() < 8) return JAAD_ERR_EOS;
    const int ncomment = (int)br.read(8);
    br.skip(8 * ncomment);
    return br.overrun() ? JAAD_ERR_EOS : JAAD_OK;
}

// program_config_element of an AudioSpecificConfig with channelConfiguration 0 (PCE.decode,
// A/syntax/PCE.java:133-188).  The reference replaces the config's profile, sample rate and channel
// configuration with the PCE's (DecoderConfig.setAudioDecoderInfo, A/DecoderConfig.java:60-65);
// the configuration is the one of the PCE's channel count (PCE.getChannelConfiguration ->
// ChannelConfiguration.forChannelCount, :221-223; 7 channels throw, 8 are 7.1), and the frames'
// elements are then decoded in bitstream order whatever the configuration says
// (SyntacticElements.decode, A/syntax/SyntacticElements.java:60-86).  This library decodes the
// element list of channel configurations 1..7, so a PCE is accepted when its front, side, back
// and LFE elements (the order they appear in) have exactly those channel counts.
int read_pce_layout(BitReader& br, int& profile, int& sfi, int& chc)
{
    if (br.left() < 4 + 2 + 4) return JAAD_ERR_EOS;
    br.skip(4);                     // element_instance_tag (PCE.read, :47-52)
    profile = 1 + (int)br.read(2);  // Profile.forInt(1 + object_type)
    sfi = (int)br.read(4);  // SampleFrequency.decode: 4 bits, no explicit frequency
    if (br.left() < 4 + 4 + 4 + 2 + 3 + 4) return JAAD_ERR_EOS;
    const int nfront = (int)br.read(4), nside = (int)br.read(4), nback = (int)br.read(4);
    const int nlfe = (int)br.read(2), nassoc = (int)br.read(3), ncc = (int)br.read(4);
    if (br.read(1)) br.skip(4);  // mono mixdown
    if (br.read(1)) br.skip(4);  // stereo mixdown
    if (br.read(1)) br.skip(3);  // matrix mixdown
    uint8_t nch[8 + 3];
    int n = 0, channels = nlfe;
    for (int i = 0; i < nfront + nside + nback; i++) {
        const int cpe = (int)br.read(1);
        br.skip(4);  // element tag
        if (n < 8) nch[n] = (uint8_t)(1 + cpe);
        n++;
        channels += 1 + cpe;
    }
    for (int i = 0; i < nlfe; i++) {
        br.skip(4);
        if (n < 8 + 3) nch[n] = 1;
        n++;
    }
    br.skip(4 * nassoc + 5 * ncc);
    br.byte_align();
    if (br.left() < 8) return JAAD_ERR_EOS;
    br.skip(8 * (int)br.read(8));  // comment field
    if (br.overrun()) return JAAD_ERR_EOS;
    if (channels == 7 || channels < 1 || channels > 8) return JAAD_ERR_UNSUPPORTED;  // forChannelCount(7) throws
    chc = channels == 8 ? 7 : channels;
    // the element list the parser and the device path decode for that configuration
    static const uint8_t kList[8][5] = {{}, {1}, {2}, {1, 2}, {1, 2, 1}, {1, 2, 2}, {1, 2, 2, 1}, {1, 2, 2, 2, 1}};
    static const int kN[8] = {0, 1, 1, 2, 3, 3, 4, 5};
    if (n != kN[chc]) return JAAD_ERR_UNSUPPORTED;
    for (int i = 0; i < n; i++)
        if (nch[i] != kList[chc][i]) return JAAD_ERR_UNSUPPORTED;
    if (chc == 1 && nlfe) return JAAD_ERR_UNSUPPORTED;  // a lone LFE: the mono path decodes an SCE
    return JAAD_OK;
}

}  // namespace

extern "C" {

int jaad_asc_parse(const uint8_t* asc, size_t bytes, jaad_stream_cfg* cfg)
{
    if (!asc || !cfg) return JAAD_ERR_INVALID_ARG;
    BitReader br(asc, bytes);
    auto profile = [&]() {  // DecoderConfig.readProfile
        int i = (int)br.read(5);
        if (i == 31) i = 32 + (int)br.read(6);
        return i;
    };
    auto rate = [&]() {  // SampleRate.decode -> nominal index (SampleFrequency.nominalFrequency)
        int idx = (int)br.read(4);
        if (idx != 15) return idx;
        const int freq = (int)br.read(24);
        static const int F[12] = {96000, 88200, 64000, 48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000};
        int best = 0;
        float dev = 1e30f;
        for (int i = 0; i < 12; i++) {
            const float d = (float)(freq > F[i] ? freq - F[i] : F[i] - freq) / (float)F[i];
            if (d == 0.0f) return i;
            if (d < dev) {
                best = i;
                dev = d;
            }
            if (F[i] < freq) break;
        }
        return best;
    };
    std::memset(cfg, 0, sizeof *cfg);
    cfg->abi_version = JAAD_ABI_VERSION;
    cfg->tns_mode = JAAD_TNS_COMPAT;
    int aot = profile();
    int sfi = rate();
    int chc = (int)br.read(4);
    if (aot == 5 || aot == 29) {  // AAC_SBR / AAC_PS: extension rate, core profile; no GASpecificConfig
        cfg->sbr = 1;
        cfg->ps = aot == 29 || chc == 1;  // mono: PS enabled by default (jaad_parse.h)
        cfg->ext_sf_index = (uint8_t)rate();
        aot = profile();
    } else if (aot == 2) {
        if (br.read(1)) return br.overrun() ? JAAD_ERR_EOS : JAAD_ERR_UNSUPPORTED;  // frameLengthFlag: 960
        if (br.read(1)) br.skip(14);                  // dependsOnCoreCoder -> coreCoderDelay
        if (br.read(1)) br.skip(1);                   // extensionFlag -> extensionFlag3
        if (br.overrun()) return JAAD_ERR_EOS;
        if (chc == 0) {  // DecoderConfig.decode: PCE.read + setAudioDecoderInfo (A/DecoderConfig.java:231-235)
            int pprof = 0, psfi = sfi;
            const int st = read_pce_layout(br, pprof, psfi, chc);
            if (st) return st;
            // outputFrequency was set to the ASC's rate before the PCE (A/DecoderConfig.java:180);
            // setAudioDecoderInfo then takes the PCE's.  With different rates the reference's
            // getSampleLength turns 2048 and it outputs at the ASC's rate: not reproduced, refused.
            if (psfi != sfi) return JAAD_ERR_UNSUPPORTED;
            aot = pprof;
        }
        // readSyncExtension (A/DecoderConfig.java:238, 260-291; sbrEnabled is always on): a
        // backward-compatible 0x2B7 extension can signal SBR (and PS, 0x548) with its output
        // rate.  Without it the output rate stays the core rate (:180): SBR met later in the
        // frames (implicit signalling) then runs downsampled (the facade's implicit_sbr_cfg).
        if (!br.overrun() && br.left() > 10 && br.read(11) == 0x2B7) {
            const int ext = (int)br.read(5);
            if (ext == 5 || ext == 22) {  // AAC_SBR, ER_BSAC
                if (br.read(1)) {         // sbrPresent
                    const int esf = rate();
                    if (ext == 5) {
                        cfg->sbr = 1;
                        cfg->ext_sf_index = (uint8_t)esf;
                        cfg->ps = chc == 1;  // psPresent (0x548) or not: PS data is applied when present
                    } else {
                        return JAAD_ERR_UNSUPPORTED;  // BSAC
                    }
                }
                if (ext == 5 && br.left() > 12 && br.read(11) == 0x548) br.skip(1);  // psPresent
            }
        }
    }
    if (br.overrun()) return JAAD_ERR_EOS;
    if (aot != 2) return JAAD_ERR_UNSUPPORTED;
    if (sfi > 11 || (cfg->sbr && cfg->ext_sf_index > 11)) return JAAD_ERR_UNSUPPORTED;
    if (chc < 1 || chc > 7) return JAAD_ERR_UNSUPPORTED;
    if (chc > 2 && cfg->ps) cfg->ps = 0;  // PS only in a mono (SCE) stream
    cfg->profile = 2;
    cfg->sf_index = (uint8_t)sfi;
    cfg->channel_config = (uint8_t)chc;
    return JAAD_OK;
}

int jaad_adts_find(const uint8_t* buf, size_t bytes, size_t* offset, jaad_adts_header* h)
{
    if (!buf || !offset || !h) return JAAD_ERR_INVALID_ARG;
    // ADTSDemultiplexer.findNextFrame: scan at most MAXIMUM_FRAME_SIZE bytes for 0xFF followed
    // by a byte with (b & 0xF6) == 0xF0
    const size_t lim = bytes < 6144 ? bytes : 6144;
    for (size_t i = 0; i + 1 < lim || (i + 1 < bytes && i < lim); i++) {
        if (buf[i] != 0xFF || (buf[i + 1] & 0xF6) != 0xF0) continue;
        if (i + 7 > bytes) return JAAD_ERR_EOS;
        const uint8_t* b = buf + i + 1;  // ADTSFrame.readHeader starts after the 0xFF
        std::memset(h, 0, sizeof *h);
        h->protection_absent = b[0] & 1;
        h->profile = (uint8_t)(((b[1] & 0xC0) >> 6) + 1);
        h->sf_index = (uint8_t)((b[1] & 0x3C) >> 2);
        h->channel_config = (uint8_t)(((b[1] & 0x01) << 2) | ((b[2] & 0xC0) >> 6));
        h->frame_length = (uint32_t)(((b[2] & 0x03) << 11) | (b[3] << 3) | ((b[4] & 0xE0) >> 5));
        h->n_raw_blocks = (uint8_t)((b[5] & 0x03) + 1);
        h->header_bytes = h->protection_absent ? 7 : 9;
        *offset = i;
        return JAAD_OK;
    }
    return JAAD_ERR_EOS;
}

int jaad_raw_pce_cfg(const uint8_t* raw, size_t bytes, jaad_stream_cfg* cfg)
{
    if (!raw || !cfg) return JAAD_ERR_INVALID_ARG;
    BitReader br(raw, bytes);
    if (br.left() < 3) return JAAD_ERR_EOS;
    if (br.read(3) != 5) return JAAD_ERR_BITSTREAM;  // the frame does not start with a PCE
    int profile = 0, sfi = 0, chc = 0;
    const int st = read_pce_layout(br, profile, sfi, chc);
    if (st) return st;
    if (profile != 2 || sfi > 11) return JAAD_ERR_UNSUPPORTED;
    std::memset(cfg, 0, sizeof *cfg);
    cfg->abi_version = JAAD_ABI_VERSION;
    cfg->profile = 2;
    cfg->sf_index = (uint8_t)sfi;
    cfg->channel_config = (uint8_t)chc;
    cfg->tns_mode = JAAD_TNS_COMPAT;
    return JAAD_OK;
}

int jaad_adts_cfg(const jaad_adts_header* h, jaad_stream_cfg* cfg)
{
    if (!h || !cfg) return JAAD_ERR_INVALID_ARG;
    // channel_config 0: the layout comes from the PCE the frames carry (jaad_raw_pce_cfg)
    if (h->profile != 2 || h->sf_index > 11 || h->channel_config > 7) return JAAD_ERR_UNSUPPORTED;
    std::memset(cfg, 0, sizeof *cfg);
    cfg->abi_version = JAAD_ABI_VERSION;
    cfg->profile = 2;
    cfg->sf_index = h->sf_index;
    cfg->channel_config = h->channel_config;
    cfg->tns_mode = JAAD_TNS_COMPAT;
    return JAAD_OK;
}

int jaad_parser_create(const jaad_stream_cfg* cfg, jaad_parser** out)
{
    if (!cfg || !out) return JAAD_ERR_INVALID_ARG;
    *out = nullptr;
    if (cfg->abi_version != JAAD_ABI_VERSION) return JAAD_ERR_ABI;
    if (cfg->profile != 2 || cfg->channel_config < 1 || cfg->channel_config > 7) return JAAD_ERR_UNSUPPORTED;
    if (cfg->ps && (!cfg->sbr || cfg->channel_config != 1)) return JAAD_ERR_UNSUPPORTED;
    jaad_parser* p = new (std::nothrow) jaad_parser;
    if (!p) return JAAD_ERR_NOMEM;
    p->C.cfg = *cfg;
    p->C.nch = cfg->channel_config == 2 ? 2 : 1;
    p->C.elem_nch[0] = (uint8_t)p->C.nch;
    {  // ISO/IEC 14496-3 Table 1.19 channel elements of configurations 3..7
        static const uint8_t kLayouts[5][6] = {{1, 2}, {1, 2, 1}, {1, 2, 2}, {1, 2, 2, 1}, {1, 2, 2, 2, 1}};
        static const int kCount[5] = {2, 3, 3, 4, 5};
        if (cfg->channel_config > 2) {
            const int k = cfg->channel_config - 3;
            p->C.n_elem = kCount[k];
            p->C.nch = 0;
            for (int i = 0; i < kCount[k]; i++) {
                p->C.elem_nch[i] = kLayouts[k][i];
                p->C.nch += kLayouts[k][i];
            }
        }
    }
    const int st = sf_counts(cfg->sf_index, p->C);
    if (st) {
        delete p;
        return st;
    }
    if (cfg->sbr && p->C.n_elem > 1) p->sbr_el.resize((size_t)p->C.n_elem - 1);
    books();
    *out = p;
    return JAAD_OK;
}

void jaad_parser_destroy(jaad_parser* p) { delete p; }

int jaad_parser_clone(const jaad_parser* src, jaad_parser** out)
{
    if (!src || !out) return JAAD_ERR_INVALID_ARG;
    *out = new (std::nothrow) jaad_parser(*src);
    return *out ? JAAD_OK : JAAD_ERR_NOMEM;
}

int jaad_parser_copy(jaad_parser* dst, const jaad_parser* src)
{
    if (!dst || !src) return JAAD_ERR_INVALID_ARG;
    if (std::memcmp(&dst->C.cfg, &src->C.cfg, sizeof(jaad_stream_cfg)) != 0) return JAAD_ERR_INVALID_ARG;
    *dst = *src;
    return JAAD_OK;
}

uint32_t jaad_parser_pns_state(const jaad_parser* p) { return p ? p->st.pns : 0u; }
void jaad_parser_set_pns_state(jaad_parser* p, uint32_t s)
{
    if (p) p->st.pns = s;
}

}  // extern "C"

namespace {

// coupling_channel_element as CCE.decode reads it (A/syntax/CCE.java:112-175)
struct CceElem {
    int point = 0;                 // couplingPoint: 0 BEFORE_TNS, 1 AFTER_TNS, 3 (ind_sw: never applied)
    int count = 0;                 // coupledCount
    bool pair[8] = {false};
    int id[8] = {0}, chs[8] = {0};
    int gain_count = 0;
    float gain[16][120] = {{0.0f}};
    int rec = 0;                   // record index in the frame's CCE output
};
struct ChElem {                    // a channel element of the frame: SCE / LFE / CPE
    bool cpe;
    int tag, ch0;
};

// a gain the library applies (jaad_gpu.h JAAD_CCE_GAIN_MAX): finite and at most 2^60 in magnitude
static bool cce_gain_ok(float g) { return std::fabs(g) <= JAAD_CCE_GAIN_MAX; }  // false for NaN, +-inf

int read_cce(BitReader& br, const Cfg& C, ParseState& ns, ChOut& o, CceElem& E)
{
    static const float kScale[4] = {1.09050773266525765921f, 1.18920711500272106672f, 1.4142135623730950488016887f, 2.0f};
    if (br.left() < 4) return JAAD_ERR_EOS;
    E.point = 2 * (int)br.read(1);
    E.count = (int)br.read(3);
    E.gain_count = 0;
    for (int i = 0; i <= E.count; i++) {
        if (br.left() < 5) return JAAD_ERR_EOS;
        E.gain_count++;
        E.pair[i] = br.read(1) != 0;
        E.id[i] = (int)br.read(4);
        if (E.pair[i]) {
            if (br.left() < 2) return JAAD_ERR_EOS;
            E.chs[i] = (int)br.read(2);
            if (E.chs[i] == 3) E.gain_count++;
        } else {
            E.chs[i] = 2;
        }
    }
    if (br.left() < 4) return JAAD_ERR_EOS;
    E.point += (int)br.read(1);
    E.point |= E.point >> 1;
    const bool sign = br.read(1) != 0;
    const double scale = kScale[br.read(2)];
    IcsInfo I;
    int st = read_ics(br, C, false, I, 0, nullptr, ns.pns, o);
    if (st) return st;
    const Books& B = books();
    auto sfcode = [&](int& v) {  // Huffman.decodeScaleFactor
        const int r = B.sf.decode(br);
        if (r < 0) return r == -2 ? JAAD_ERR_EOS : JAAD_ERR_BITSTREAM;
        v = JAAD_HCB_SF[r][2];
        return JAAD_OK;
    };
    for (int i = 0; i < E.gain_count; i++) {
        int cge = 1, xg = 0;
        float gc = 1.0f;
        if (i > 0) {
            if (br.left() < 1 && E.point != 2) return JAAD_ERR_EOS;
            cge = E.point == 2 ? 1 : (int)br.read(1);
            if (cge) {
                if ((st = sfcode(xg))) return st;
                xg -= 60;
            }
            gc = (float)std::pow(scale, (double)-xg);
        }
        if (E.point == 2) {
            if (!cce_gain_ok(gc)) return JAAD_ERR_UNSUPPORTED;
            E.gain[i][0] = gc;
            continue;
        }
        for (int g = 0, idx = 0; g < I.ngroups; g++)
            for (int sfb = 0; sfb < I.max_sfb; sfb++, idx++) {
                if (o.cb[idx] == JAAD_ZERO_HCB) continue;
                if (cge == 0) {
                    int t;
                    if ((st = sfcode(t))) return st;
                    t -= 60;
                    if (t != 0) {
                        int sgn = 1;
                        t = xg += t;
                        if (!sign) {
                            sgn -= 2 * (t & 1);
                            t >>= 1;
                        }
                        gc = (float)(std::pow(scale, (double)-t) * sgn);
                    }
                }
                if (!cce_gain_ok(gc)) return JAAD_ERR_UNSUPPORTED;
                E.gain[i][idx] = gc;
            }
    }
    return br.overrun() ? JAAD_ERR_EOS : JAAD_OK;
}

// ChannelElement.processDependentCoupling (A/syntax/ChannelElement.java:105-130) for every channel
// element of the frame, as terms in the reference's order per target channel
int cce_terms(const CceElem* cces, int n_cce, const ChElem* els, int n_el, jaad_frame_out* out)
{
    uint32_t n = 0;
    auto emit = [&](const CceElem& E, int ch, int index) {
        if (n >= out->term_cap) return false;
        jaad_cce_term& t = out->cce_terms[n++];
        std::memset(&t, 0, sizeof t);
        t.channel = (uint8_t)ch;
        t.point = (uint8_t)E.point;
        t.cce = (uint16_t)E.rec;
        std::memcpy(t.gain, E.gain[index], sizeof t.gain);
        return true;
    };
    for (int k = 0; k < n_cce; k++) {
        const CceElem& E = cces[k];
        if (E.point != 0 && E.point != 1) continue;  // ind_sw CCEs (point 3) match no coupling point
        for (int e = 0; e < n_el; e++) {
            int index = 0;
            for (int c = 0; c <= E.count; c++) {
                const int chs = E.chs[c];
                if (E.pair[c] == els[e].cpe && E.id[c] == els[e].tag) {
                    if (chs != 1) {
                        if (!emit(E, els[e].ch0, index)) return JAAD_ERR_UNSUPPORTED;
                        if (chs != 0) index++;
                    }
                    if (chs != 2) {
                        if (!emit(E, els[e].ch0 + 1, index)) return JAAD_ERR_UNSUPPORTED;
                        index++;
                    }
                } else {
                    index += 1 + (chs == 3 ? 1 : 0);
                }
            }
        }
    }
    out->n_cce_terms = n;
    return JAAD_OK;
}

// the LFE position of a multichannel layout (configurations 6 and 7 end with the LFE, ISO/IEC
// 14496-3 Table 1.19; configuration 4 ends with a back SCE)
bool mc_lfe(const Cfg& C, int e) { return (C.cfg.channel_config == 6 || C.cfg.channel_config == 7) && e == C.n_elem - 1; }

// One raw_data_block into `out`, moving the parse state ns / nsel (multichannel HE-AAC: SBR
// state of elements 1..) as the reference moves its fields; parse_frame commits them.
// probe != nullptr: stop at the first SBR extension payload after the channel element (bit 0 of
// *probe).
int parse_frame_body(const jaad_parser* p, const uint8_t* data, size_t bytes, jaad_frame_out* out, uint32_t* probe,
                     ParseState& ns, std::vector<SbrParseState>& nsel)
{
    if (!p || !out || (!data && bytes) || !out->q || !out->sf || !out->cb || !out->ics) return JAAD_ERR_INVALID_ARG;
    const Cfg& C = p->C;
    int n_cpe = 0;
    for (int k = 0; k < C.n_elem; k++) n_cpe += C.elem_nch[k] == 2;
    if (n_cpe && !out->ms_used) return JAAD_ERR_INVALID_ARG;
    if (C.cfg.sbr && !out->sbr) return JAAD_ERR_INVALID_ARG;
    BitReader br(data, bytes);
    bool have_channels = false;
    int elem = 0, ch0 = 0, cpe = 0;  // channel elements parsed so far, their channels, CPEs
    // SBR records: one per channel element (multichannel: out->sbr[0 .. n_elem), element order)
    uint32_t sbr_seen = 0;           // bit k: element k carried an SBR payload this frame
    if (C.cfg.sbr) std::memset(out->sbr, 0, sizeof *out->sbr * (size_t)C.n_elem);
    ChElem els[8];
    int n_els = 0;
    std::vector<CceElem> cces;  // 7.7 KB each: only when the frame has CCEs
    int n_cce = 0;
    out->n_cce = out->n_cce_terms = 0;
    for (;;) {
        if (br.left() < 3) return JAAD_ERR_EOS;
        const int id = (int)br.read(3);
        if (id == 7) break;  // END
        if (id == 6) {       // FIL (SyntacticElements.decodeFIL, :169-203)
            if (br.left() < 4) return JAAD_ERR_EOS;
            int count = (int)br.read(4);
            if (count == 15) {
                if (br.left() < 8) return JAAD_ERR_EOS;
                count += (int)br.read(8) - 1;
            }
            if (!count) continue;
            if (br.left() < 8 * count) return JAAD_ERR_EOS;
            BitReader sub = br.sub(8 * count);
            br.skip(8 * count);
            const int type = (int)sub.read(4);
            if ((type == 13 || type == 14) && have_channels) {  // EXT_SBR_DATA(_CRC)
                // implicit SBR: the reference (sbrEnabled by default, A/DecoderConfig.java:47-53)
                // would decode it and double the output rate; the caller must re-open the
                // stream with cfg.sbr = 1 (and cfg.ps = 1 for a mono core, SCE.isStereo)
                if (probe) {
                    *probe |= 1u;
                    return JAAD_OK;
                }
                if (!C.cfg.sbr) return JAAD_ERR_UNSUPPORTED;
                // SyntacticElements.decodeSBR: the payload belongs to the last audio element
                // (A/syntax/SyntacticElements.java:207-211).  SBR on the LFE of a multichannel
                // stream would add a channel to the reference's output (LFE extends SCE): refused.
                const int e = elem - 1;
                if (C.n_elem > 1 && mc_lfe(C, e)) return JAAD_ERR_UNSUPPORTED;
                SbrParseState& S = e == 0 ? ns.sbr : nsel[(size_t)e - 1];
                const SbrParseState before = S;
                const int st = parse_sbr(sub, C, C.elem_nch[e], type == 14, S, out->sbr[e]);
                if (st == JAAD_ERR_EOS) {
                    // The bitstream ends inside the SBR payload.  The reference has read as much of
                    // it as was there when its EOSException comes (SBR.decode: readHeader with its
                    // header swap and calc_sbr_tables, then part of sbr_data, A/sbr/SBR.java:162-184),
                    // a partial state change that no record here describes: the frame is refused
                    // instead of dropped, so the stream cannot go on out of step (the parser keeps
                    // its state).  A frame cut after its SBR payload is dropped with the payload's
                    // record, header included (jaad_decode_batch applies it).
                    S = before;
                    return JAAD_ERR_UNSUPPORTED;
                }
                if (st) return st;
                sbr_seen |= 1u << e;
            }
            continue;
        }
        if (br.left() < 4) return JAAD_ERR_EOS;
        const int tag = (int)br.read(4);  // element_instance_tag
        if (id == 4) {  // DSE
            const int st = skip_dse(br);
            if (st) return st;
            continue;
        }
        if (id == 5) {  // PCE
            const int st = skip_pce(br);
            if (st) return st;
            continue;
        }
        if (id == 2) {  // CCE: its ICStream as a record, its gains for the terms made at the end
            if (!out->cce_q || !out->cce_sf || !out->cce_cb || !out->cce_ics || !out->cce_terms) return JAAD_ERR_UNSUPPORTED;
            if ((uint32_t)n_cce >= out->cce_cap || n_cce >= 8) return JAAD_ERR_UNSUPPORTED;
            cces.emplace_back();
            CceElem& E = cces.back();
            E.rec = n_cce;
            ChOut o{out->cce_q + (size_t)n_cce * 1024, out->cce_sf + n_cce * 128, out->cce_cb + n_cce * 128,
                    out->cce_ics + n_cce, nullptr};
            const int st = read_cce(br, C, ns, o, E);
            if (st) return st;
            n_cce++;
            continue;
        }
        // SCE (0) / LFE (3) / CPE (1): the configuration's channel elements in their ISO order (one
        // SCE or CPE for mono / stereo); LFE decodes as an SCE (A/syntax/LFE.java)
        if (elem >= C.n_elem || (id == 1) != (C.elem_nch[elem] == 2) || (id == 3 && C.n_elem == 1))
            return JAAD_ERR_UNSUPPORTED;
        have_channels = true;
        els[n_els++] = ChElem{id == 1, tag, ch0};
        if (id == 0 || id == 3) {
            IcsInfo I;
            ChOut o{out->q + (size_t)ch0 * 1024, out->sf + ch0 * 128, out->cb + ch0 * 128, out->ics + ch0,
                    out->tns ? out->tns + ch0 : nullptr};
            const int st = read_ics(br, C, false, I, ns.shape[ch0], &ns.shape[ch0], ns.pns, o);
            if (st) return st;
        } else {
            // CPE.decode (A/syntax/CPE.java:85-123)
            if (br.left() < 1) return JAAD_ERR_EOS;
            const bool common = br.read(1) != 0;
            IcsInfo IL, IR;
            uint64_t ms[2] = {0, 0};
            bool ms_present = false;
            const int prevL = ns.shape[ch0], prevR = ns.shape[ch0 + 1];
            if (common) {
                int st = read_ics_info(br, C, IL, &ns.shape[ch0]);
                if (st) return st;
                IR = IL;  // ICSInfo.setCommonData, right after infoL.decode (A/syntax/CPE.java:93-94)
                ns.shape[ch0 + 1] = IR.shape;
                if (br.left() < 2) return JAAD_ERR_EOS;
                const int mask = (int)br.read(2);
                const int nb = IL.ngroups * IL.max_sfb;
                if (mask == 1) {
                    if (br.left() < nb) return JAAD_ERR_EOS;
                    for (int i = 0; i < nb; i++)
                        if (br.read(1)) ms[i >> 6] |= 1ull << (i & 63);
                } else if (mask == 2) {
                    for (int i = 0; i < nb; i++) ms[i >> 6] |= 1ull << (i & 63);
                } else if (mask == 3) {
                    return JAAD_ERR_BITSTREAM;  // "reserved MS mask type used"
                }
                ms_present = mask != 0;
            }
            ChOut oL{out->q + (size_t)ch0 * 1024, out->sf + ch0 * 128, out->cb + ch0 * 128, out->ics + ch0,
                     out->tns ? out->tns + ch0 : nullptr};
            ChOut oR{out->q + (size_t)(ch0 + 1) * 1024, out->sf + (ch0 + 1) * 128, out->cb + (ch0 + 1) * 128,
                     out->ics + ch0 + 1, out->tns ? out->tns + ch0 + 1 : nullptr};
            int st = read_ics(br, C, common, IL, prevL, &ns.shape[ch0], ns.pns, oL);
            if (st) return st;
            st = read_ics(br, C, common, IR, prevR, &ns.shape[ch0 + 1], ns.pns, oR);
            if (st) return st;
            if (ms_present) out->ics[ch0].flags |= JAAD_ICS_MS_PRESENT;
            out->ms_used[2 * cpe] = ms[0];
            out->ms_used[2 * cpe + 1] = ms[1];
            cpe++;
        }
        ch0 += C.elem_nch[elem];
        elem++;
    }
    if (!have_channels) return JAAD_ERR_BITSTREAM;  // a frame without audio: nothing to decode
    if (elem != C.n_elem) return JAAD_ERR_UNSUPPORTED;  // a frame without all the configuration's elements
    if (C.cfg.sbr)
        for (int e = 0; e < C.n_elem; e++) {
            if (sbr_seen & (1u << e)) continue;
            // an SCE of a multichannel stream without SBR data would drop to one output channel in
            // the reference (SCE.process accepts dataR only with SBR, A/syntax/SCE.java:122-132),
            // changing the frame's channel count: refused.  CPEs and LFEs are upsampled.
            if (C.n_elem > 1 && C.elem_nch[e] == 1 && !mc_lfe(C, e)) return JAAD_ERR_UNSUPPORTED;
            const int st = sbr_missing(C, ns, out->sbr[e]);
            if (st) return st;
        }
    if (n_cce) {
        const int st = cce_terms(cces.data(), n_cce, els, n_els, out);
        if (st) return st;
        out->n_cce = (uint32_t)n_cce;
    }
    return JAAD_OK;
}

// The state moves with a frame that parsed, and with one whose bitstream ended early as far as the
// reference's reads got before its EOSException (Decoder.decodeFrame drops that frame and the next
// one sees those fields: A/Decoder.java:89-101).  Any other error leaves the parser as it was (the
// reference throws an AACException out of decodeFrame; this decoder rejects the frame whole).
int parse_frame(jaad_parser* p, const uint8_t* data, size_t bytes, jaad_frame_out* out, uint32_t* probe)
{
    if (!p) return JAAD_ERR_INVALID_ARG;
    ParseState ns = p->st;
    std::vector<SbrParseState> nsel = p->sbr_el;
    const int st = parse_frame_body(p, data, bytes, out, probe, ns, nsel);
    if (!probe && (st == JAAD_OK || st == JAAD_ERR_EOS)) {
        p->st = ns;
        p->sbr_el.swap(nsel);
    }
    return st;
}
}  // namespace

extern "C" {

int jaad_parse_frame(jaad_parser* p, const uint8_t* data, size_t bytes, jaad_frame_out* out)
{
    return parse_frame(p, data, bytes, out, nullptr);
}

int jaad_probe_sbr(const jaad_stream_cfg* cfg, const uint8_t* data, size_t bytes, uint32_t* found)
{
    if (!cfg || !found || (!data && bytes)) return JAAD_ERR_INVALID_ARG;
    *found = 0;
    jaad_stream_cfg core = *cfg;
    core.sbr = core.ps = 0;
    core.ext_sf_index = 0;
    jaad_parser* p = nullptr;
    int st = jaad_parser_create(&core, &p);
    if (st) return st;
    std::vector<int16_t> q(8 * 1024);  // up to 8 channels (configuration 7)
    std::vector<uint8_t> sf(8 * 128), cb(8 * 128);
    jaad_ics_info ics[8];
    jaad_tns tns[8];
    uint64_t ms[8];
    std::vector<int16_t> cq(8 * 1024);
    std::vector<uint8_t> csf(8 * 128), ccb(8 * 128);
    jaad_ics_info cics[8];
    std::vector<jaad_cce_term> terms(128);
    jaad_frame_out o{q.data(), sf.data(), cb.data(), ics, ms, tns, nullptr, cq.data(), csf.data(), ccb.data(), cics,
                     terms.data(), 8, 128, 0, 0};
    st = parse_frame(p, data, bytes, &o, found);
    jaad_parser_destroy(p);
    return st;
}

}  // extern "C"
