// Mutation fuzz of the host bitstream front end (include/jaad_parse.h), built for the host with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_fuzz_parse.py: seed frames (valid
// LC / HE-AAC v1 / v2 raw_data_blocks from the test writer) get random bit flips and truncations;
// every status is acceptable, a sanitizer report is not.  Usage: fuzz_parse <seeds.bin> <iters>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "jaad_mp4.h"
#include "jaad_parse.h"
static uint64_t rs = 0x1234567ull;
static uint32_t rnd() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (uint32_t)(rs >> 11); }
struct Seed { int cfg; std::vector<uint8_t> d; };
// mode "mp4": bit flips / truncations of one MP4 file image through jaad_mp4_open + the frame table
static int fuzz_mp4(const char* path, int iters)
{
    FILE* f = fopen(path, "rb");
    if (!f) return 2;
    std::vector<uint8_t> img;
    int ch;
    while ((ch = fgetc(f)) != EOF) img.push_back((uint8_t)ch);
    fclose(f);
    int ok = 0;
    for (int it = 0; it < iters; it++) {
        std::vector<uint8_t> d = img;
        const int nflip = 1 + rnd() % 6;
        for (int j = 0; j < nflip; j++) { size_t b = rnd() % (d.size() * 8); d[b >> 3] ^= (uint8_t)(0x80 >> (b & 7)); }
        if (rnd() % 4 == 0) d.resize(rnd() % (d.size() + 1));
        uint8_t* data = d.empty() ? nullptr : (uint8_t*)malloc(d.size());
        if (data) memcpy(data, d.data(), d.size());
        jaad_mp4* m = nullptr;
        if (jaad_mp4_open(data, d.size(), &m) == 0) {
            ok++;
            for (int t = 0; t < jaad_mp4_track_count(m); t++) {
                jaad_mp4_track ti;
                jaad_mp4_track_info(m, t, &ti);
                const uint8_t* dsi;
                size_t n;
                jaad_mp4_decoder_specific_info(m, t, &dsi, &n);
                jaad_stream_cfg c;
                if (n) jaad_asc_parse(dsi, n, &c);
                for (uint32_t i = 0; i < ti.n_frames; i++) {
                    uint64_t o;
                    uint32_t s2;
                    double tm;
                    jaad_mp4_frame(m, t, i, &o, &s2, &tm);
                }
            }
            jaad_mp4_close(m);
        }
        free(data);
    }
    printf("mp4 opened: %d\n", ok);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 4 && !strcmp(argv[1], "mp4")) return fuzz_mp4(argv[2], atoi(argv[3]));
    if (argc < 3) return 2;
    const int iters = atoi(argv[2]);
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<Seed> seeds;
    unsigned char hdr[5];
    while (fread(hdr, 1, 5, f) == 5) {
        Seed s; s.cfg = hdr[0]; uint32_t n; memcpy(&n, hdr + 1, 4); s.d.resize(n);
        if (fread(s.d.data(), 1, n, f) != n) break;
        seeds.push_back(s);
    }
    fclose(f);
    int counts[16] = {0};
    jaad_parser* ps[3];
    jaad_stream_cfg cfgs[3];
    for (int k = 0; k < 3; k++) {
        jaad_stream_cfg& c = cfgs[k]; memset(&c, 0, sizeof c);
        c.abi_version = JAAD_ABI_VERSION; c.profile = 2;
        if (k == 0) { c.sf_index = 6; c.channel_config = 2; c.sbr = 1; c.ext_sf_index = 3; }
        if (k == 1) { c.sf_index = 6; c.channel_config = 1; c.sbr = 1; c.ps = 1; c.ext_sf_index = 3; }
        if (k == 2) { c.sf_index = 3; c.channel_config = 2; c.tns_mode = 1; }
        jaad_parser_create(&c, &ps[k]);
    }
    std::vector<int16_t> q(2048); std::vector<uint8_t> sf(256), cb(256);
    jaad_ics_info ics[2]; jaad_tns tns[2]; uint64_t ms[2]; jaad_sbr_frame sbr;
    for (int it = 0; it < iters; it++) {
        const Seed& s = seeds[rnd() % seeds.size()];
        const int k = s.cfg == 4 ? 0 : s.cfg == 5 ? 1 : 2;
        std::vector<uint8_t> d = s.d;
        const int nflip = 1 + rnd() % 4;
        for (int j = 0; j < nflip; j++) { size_t b = rnd() % (d.size() * 8); d[b >> 3] ^= (uint8_t)(0x80 >> (b & 7)); }
        if (rnd() % 4 == 0) d.resize(rnd() % (d.size() + 1));
        uint8_t* data = d.empty() ? nullptr : (uint8_t*)malloc(d.size());
        if (data) memcpy(data, d.data(), d.size());
        jaad_frame_out o{q.data(), sf.data(), cb.data(), ics, ms, tns, cfgs[k].sbr ? &sbr : nullptr};
        const int st = jaad_parse_frame(ps[k], data, d.size(), &o);
        counts[-st < 16 ? -st : 15]++;
        free(data);
        // keep the parsers' history moving with valid frames too
        jaad_parse_frame(ps[k], s.d.data(), s.d.size(), &o);
    }
    for (int k = 0; k < 3; k++) jaad_parser_destroy(ps[k]);
    for (int i = 0; i < 16; i++) if (counts[i]) printf("status %d: %d\n", -i, counts[i]);
    return 0;
}
