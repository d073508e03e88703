// Internal pieces shared by the host bitstream front end (jaad_parse.cpp, jaad_parse_sbr.cpp).
#pragma once
#include <stdint.h>

#include <cstddef>
#include <cstring>

#include "../../include/jaad_gpu.h"

namespace jaad {
namespace parse {

// MSB-first bit reader over [data, data + bytes) (A/syntax/ByteArrayBitStream.java).  Reads
// past the end return zero bits and set overrun(); callers check left() first where the
// reference would throw EOSException.  sub() is readSubStream: a window of the next n bits
// sharing the parent's absolute position (byte alignment stays absolute, as in the reference).
class BitReader {
public:
    BitReader(const uint8_t* d, size_t bytes) : d_(d), phys_(bytes), end_(bytes * 8), pos_(0) {}
    int64_t left() const { return (int64_t)end_ - (int64_t)pos_; }
    bool overrun() const { return pos_ > end_; }
    size_t pos() const { return pos_; }
    // the next n <= 32 bits, MSB first (zero past the end).  Fast path: one big-endian 64-bit
    // window at the current byte (the reads stay inside the caller's buffer), bits at or past the
    // window's end masked off; the tail of the buffer goes bit by bit.
    uint32_t peek(int n) const
    {
        if (n <= 0) return 0;
        const size_t byte = pos_ >> 3;
        if (byte + 8 <= phys_) {
            uint64_t w;
            std::memcpy(&w, d_ + byte, 8);
            w = __builtin_bswap64(w) << (pos_ & 7);
            uint32_t v = (uint32_t)(w >> (64 - n));
            if (pos_ + (size_t)n > end_)  // sub-stream window: bits from end_ on read as zero
                v = pos_ >= end_ ? 0u : v & ~((1u << (pos_ + (size_t)n - end_)) - 1u) ;
            return v;
        }
        uint64_t v = 0;
        size_t p = pos_;
        for (int i = 0; i < n; i++, p++) v = (v << 1) | (p < end_ ? ((d_[p >> 3] >> (7 - (p & 7))) & 1u) : 0u);
        return (uint32_t)v;
    }
    uint32_t read(int n)
    {
        const uint32_t v = peek(n);
        pos_ += (size_t)(n > 0 ? n : 0);
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

    // The same stream with its next bits held in a 64-bit register (the spectral data's inner
    // loop: a codeword's peek is then one shift, not a load).  Valid peeks need n <= cnt; refill()
    // reloads the window at pos (>= 57 bits, zero from the end on).  commit() hands the position back.
    struct Window {
        const uint8_t* d;
        size_t phys, end, pos;
        uint64_t buf = 0;
        int cnt = 0;
        void refill()
        {
            const size_t byte = pos >> 3;
            const int sh = (int)(pos & 7);
            uint64_t w = 0;
            if (byte + 8 <= phys) {
                std::memcpy(&w, d + byte, 8);
                w = __builtin_bswap64(w);
            } else {
                for (size_t i = 0; i < 8; i++) w = (w << 8) | (byte + i < phys ? d[byte + i] : 0u);
            }
            w <<= sh;
            cnt = 64 - sh;
            if (pos + (size_t)cnt > end) {  // bits from end on read as zero
                const size_t keep = end > pos ? end - pos : 0;
                w = keep ? w & ~(~0ull >> keep) : 0;
            }
            buf = w;
        }
        void need(int n)
        {
            if (cnt < n) refill();
        }
        int64_t left() const { return (int64_t)end - (int64_t)pos; }
        uint32_t peek(int n) const { return n ? (uint32_t)(buf >> (64 - n)) : 0u; }  // n <= cnt, <= 32
        void skip(int n)
        {
            buf <<= n;
            cnt -= n;
            pos += (size_t)n;
        }
        uint32_t read(int n)
        {
            const uint32_t v = peek(n);
            skip(n);
            return v;
        }
    };
    Window window() const
    {
        Window w{d_, phys_, end_, pos_};
        w.refill();
        return w;
    }
    void commit(const Window& w) { pos_ = w.pos; }

private:
    const uint8_t* d_;
    size_t phys_;  // bytes of the caller's buffer (a sub-stream keeps its parent's)
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
