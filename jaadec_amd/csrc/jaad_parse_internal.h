// Internal pieces shared by the host bitstream front end (jaad_parse.cpp, jaad_parse_sbr.cpp).
#pragma once
#include <stdint.h>

#include <cstddef>

#include "../../include/jaad_gpu.h"

namespace jaad {
namespace parse {

// MSB-first bit reader over [data, data + bytes) (A/syntax/ByteArrayBitStream.java).  Reads
// past the end return zero bits and set overrun(); callers check left() first where the
// reference would throw EOSException.  sub() is readSubStream: a window of the next n bits
// sharing the parent's absolute position (byte alignment stays absolute, as in the reference).
class BitReader {
public:
    BitReader(const uint8_t* d, size_t bytes) : d_(d), end_(bytes * 8), pos_(0) {}
    int64_t left() const { return (int64_t)end_ - (int64_t)pos_; }
    bool overrun() const { return pos_ > end_; }
    size_t pos() const { return pos_; }
    uint32_t peek(int n) const
    {
        uint64_t v = 0;
        size_t p = pos_;
        for (int i = 0; i < n; i++, p++) v = (v << 1) | (p < end_ ? ((d_[p >> 3] >> (7 - (p & 7))) & 1u) : 0u);
        return (uint32_t)v;
    }
    uint32_t read(int n)
    {
        if (n <= 0) return 0;
        uint32_t v;
        if (pos_ + (size_t)n <= end_ && n <= 25) {  // fast path: one unaligned 32-bit window
            const size_t byte = pos_ >> 3;
            const int sh = (int)(pos_ & 7);
            uint32_t w = 0;
            const size_t avail = (end_ + 7) / 8 - byte;
            for (size_t i = 0; i < 4; i++) w = (w << 8) | (i < avail ? d_[byte + i] : 0u);
            v = (w << sh) >> (32 - n);
        } else {
            v = peek(n);
        }
        pos_ += (size_t)n;
        return v;
    }
    void skip(int64_t n) { pos_ += (size_t)(n > 0 ? n : 0); }
    void byte_align() { pos_ = (pos_ + 7) & ~(size_t)7; }
    BitReader sub(int64_t n) const
    {
        BitReader r = *this;
        r.end_ = pos_ + (size_t)n < end_ ? pos_ + (size_t)n : end_;
        return r;
    }

private:
    const uint8_t* d_;
    size_t end_, pos_;
};

struct Cfg {
    jaad_stream_cfg cfg;
    int nch = 1;            // channel-frame records per frame (1 SCE, 2 CPE, 3..8 multichannel)
    int sf_index = 0, nswb_l = 0, nswb_s = 0;
    // the frame's channel elements in bitstream order (1 = SCE/LFE, 2 = CPE): one for
    // configurations 1 / 2, the ISO layout for 3..7 (jaad_capi.cpp mc_elements)
    int n_elem = 1;
    uint8_t elem_nch[8] = {1};
};

// SBR / PS bitstream state that persists between frames (jaad_parse_sbr.cpp): what the
// reference keeps in SBR (header, derived band counts), Channel (grid, E/Q of the previous frame,
// A/sbr/Channel.java, A/sbr/SBR.java:256-284) and PSImpl / EnvData (A/ps/PSImpl.java,
// A/ps/EnvData.java, A/ps/Envelope.java) between frames
struct PsEnvData {
    int mode = -1;              // EnvMode id, -1 = null (disabled)
    int first[34] = {0};        // EnvData.first: the last envelope of the previous PS frame
    int index[5][34] = {{0}};   // Envelope.index of envs[0..4] (persist across frames)
    bool dt[5] = {false};
};
struct SbrParseState {
    bool have_hdr = false;
    jaad_sbr_header hdr{};
    int n[2] = {0, 0}, N_Q = 0, N_high = 0, N_low = 0;  // derived tables of the current header
    int f_table_res[2][65] = {{0}};
    struct Ch {  // the parse-side fields of Channel; arrays keep stale entries as the Java ones do
        int frame_class = 0, L_E = 0, L_Q = 0, bs_pointer = 0;
        int t_E[6] = {0}, t_Q[3] = {0}, f[6] = {0};
        int df_env[9] = {0}, df_noise[3] = {0}, invf[5] = {0};
        int E[64][5] = {{0}}, Q[64][2] = {{0}};
        int add_harmonic_flag = 0;
        uint64_t add_harmonic = 0;
        int E_prev[64] = {0}, Q_prev[64] = {0}, f_prev = 0;  // sbr_save_prev_data
    } ch[2];
    struct Ps {
        bool var_borders = false;
        int border[6] = {0};
        PsEnvData iid, icc, ipd, opd;
        bool ext_enabled = false, ext_data = false, ext_data_enabled = false;
    } ps;
};

struct ParseState {
    uint32_t pns = 0x1F2E3D4Cu;  // static ICStream.randomState (A/syntax/ICStream.java:26)
    int shape[8] = {0};          // ICSInfo.windowShape[CURRENT] of the previous frame, per channel
    SbrParseState sbr;
};

struct ChOut {
    int16_t* q;
    uint8_t* sf;
    uint8_t* cb;
    jaad_ics_info* ics;
    jaad_tns* tns;
};

// one sbr_extension_data payload (after the 4-bit extension type) of a channel element with nch
// channels (1 SCE/LFE: SBR1, 2 CPE: SBR2) into rec, with that element's SBR state S
int parse_sbr(BitReader& br, const Cfg& C, int nch, bool crc, SbrParseState& S, jaad_sbr_frame& rec);
// a frame of an SBR configuration that carried no SBR payload
int sbr_missing(const Cfg& C, ParseState& st, jaad_sbr_frame& rec);

}  // namespace parse
}  // namespace jaad
