// Host front-end timing: jaad_parse_frame (include/jaad_parse.h) over a bitstream corpus
// (tests/golden/parse_c*.bin, tests/golden/make_parse_corpus.py), no GPU involved.
//
// The reference parses on the decoding thread, frame by frame (Decoder.decode0 ->
// SyntacticElements.decode, A/Decoder.java:103-121; Huffman + inverse-quant index reads fused at
// A/syntax/ICStream.java:222-275, A/huffman/Huffman.java:15-84).  In the drop-in the host parse
// feeds every GPU frame, so its rate per core says how many cores keep one MI355X busy.
//
// Each thread owns its own parser per corpus stream and parses that stream's frames in order, then
// starts over from a copy of the stream's initial parser state, into one frame's worth of
// jaad_frame_out records (the caller's batch slot), until the time budget is spent.
//
//     tools/bench_parse CORPUS THREADS SECONDS            -> one JSON line (parse only, no GPU)
//     tools/bench_parse CORPUS THREADS SECONDS STREAMS    -> bitstream -> PCM on GPU 0
// The second form is the drop-in's whole host path: batches of STREAMS streams x the corpus' frames
// are parsed by THREADS threads into a jaad_batch (the corpus' streams reused round robin, each
// batch stream with its own parser) while the previous batch decodes through jaad_decode_batch
// (host buffers in, host PCM out, registered once as a JNI caller pins its buffers).
// Built by jaadec_amd/build.py (build_tools) against libjaadgpu.so.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "jaad_gpu.h"
#include "jaad_parse.h"

namespace {

struct Corpus {
    jaad_stream_cfg cfg{};
    uint32_t streams = 0, frames = 0;
    std::vector<uint32_t> pns;                              // [stream] initial LCG state
    std::vector<std::vector<std::pair<size_t, size_t>>> fr;  // [stream][frame] (offset, bytes)
    std::vector<uint8_t> data;
    size_t bytes = 0;  // bitstream bytes of one pass over every stream
};

bool load(const char* path, Corpus& c)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    c.data.resize((size_t)std::ftell(f));
    std::fseek(f, 0, SEEK_SET);
    const bool ok = std::fread(c.data.data(), 1, c.data.size(), f) == c.data.size();
    std::fclose(f);
    if (!ok || c.data.size() < 8 || std::memcmp(c.data.data(), "JPC1", 4) != 0) return false;
    size_t at = 4;
    auto u32 = [&](uint32_t& v) {
        if (at + 4 > c.data.size()) return false;
        std::memcpy(&v, &c.data[at], 4);
        at += 4;
        return true;
    };
    uint32_t cb = 0;
    if (!u32(cb) || cb != sizeof(jaad_stream_cfg) || at + cb > c.data.size()) return false;
    std::memcpy(&c.cfg, &c.data[at], cb);
    at += cb;
    if (!u32(c.streams) || !u32(c.frames)) return false;
    c.pns.resize(c.streams);
    c.fr.assign(c.streams, {});
    for (uint32_t s = 0; s < c.streams; s++) {
        if (!u32(c.pns[s])) return false;
        for (uint32_t j = 0; j < c.frames; j++) {
            uint32_t n = 0;
            if (!u32(n) || at + n > c.data.size()) return false;
            c.fr[s].push_back({at, n});
            c.bytes += n;
            at += n;
        }
    }
    return true;
}

// one frame's records (a batch slot), reused frame after frame
struct Slot {
    std::vector<int16_t> q;
    std::vector<uint8_t> sf, cb;
    std::vector<jaad_ics_info> ics;
    uint64_t ms[2 * 8];
    std::vector<jaad_tns> tns;
    std::vector<jaad_sbr_frame> sbr;
    jaad_frame_out out{};
    explicit Slot(int nch)
        : q((size_t)nch * 1024), sf((size_t)nch * 128), cb((size_t)nch * 128), ics(nch), tns(nch), sbr(8)
    {
        out.q = q.data();
        out.sf = sf.data();
        out.cb = cb.data();
        out.ics = ics.data();
        out.ms_used = ms;
        out.tns = tns.data();
        out.sbr = sbr.data();
    }
};

// one batch of S streams x F frames in the jaad_batch layout (host memory, registered with ctx)
struct HostBatch {
    uint32_t S, F, nch;
    std::vector<int16_t> q;
    std::vector<uint8_t> sf, cb;
    std::vector<jaad_ics_info> ics;
    std::vector<uint64_t> ms;
    std::vector<jaad_tns> tns;
    std::vector<jaad_sbr_frame> sbr;
    std::vector<uint32_t> slot, begin;
    jaad_batch b{};
    HostBatch(uint32_t S_, uint32_t F_, int nch_, bool sbr_)
        : S(S_), F(F_), nch((uint32_t)nch_), q((size_t)S_ * F_ * nch_ * 1024), sf((size_t)S_ * F_ * nch_ * 128),
          cb((size_t)S_ * F_ * nch_ * 128), ics((size_t)S_ * F_ * nch_), ms((size_t)S_ * F_ * 2), tns((size_t)S_ * F_ * nch_),
          sbr(sbr_ ? (size_t)S_ * F_ : 0), slot(S_), begin(S_ + 1)
    {
        for (uint32_t r = 0; r < S; r++) slot[r] = r;
        for (uint32_t r = 0; r <= S; r++) begin[r] = r * F;
        b.n_frames = S * F;
        b.n_runs = S;
        b.stream_slot = slot.data();
        b.frame_begin = begin.data();
        b.q = q.data();
        b.sf = sf.data();
        b.cb = cb.data();
        b.ics = ics.data();
        b.ms_used = nch == 2 ? ms.data() : nullptr;
        b.tns = tns.data();
        b.sbr = sbr_ ? sbr.data() : nullptr;
    }
    void reg(jaad_ctx* ctx)
    {
        jaad_host_register(ctx, q.data(), q.size() * sizeof(int16_t));
        jaad_host_register(ctx, sf.data(), sf.size());
        jaad_host_register(ctx, cb.data(), cb.size());
        jaad_host_register(ctx, ics.data(), ics.size() * sizeof(jaad_ics_info));
        jaad_host_register(ctx, ms.data(), ms.size() * sizeof(uint64_t));
        jaad_host_register(ctx, tns.data(), tns.size() * sizeof(jaad_tns));
    }
};

int pipeline(const Corpus& c, int T, double secs, uint32_t S)
{
    const int nch = c.cfg.channel_config;
    const uint32_t F = c.frames;
    jaad_ctx* ctx = nullptr;
    int rc = jaad_ctx_create(&c.cfg, S, 0, &ctx);
    if (rc) {
        std::fprintf(stderr, "jaad_ctx_create: %d\n", rc);
        return 1;
    }
    const size_t per = jaad_frame_pcm_bytes(&c.cfg, JAAD_PCM_BIG_ENDIAN);
    std::vector<uint8_t> pcm((size_t)S * F * per);
    jaad_host_register(ctx, pcm.data(), pcm.size());
    HostBatch hb[2] = {HostBatch(S, F, nch, c.cfg.sbr != 0), HostBatch(S, F, nch, c.cfg.sbr != 0)};
    for (auto& h : hb) h.reg(ctx);
    std::vector<jaad_parser*> init(c.streams), p(S);
    for (uint32_t s = 0; s < c.streams; s++) {
        if (jaad_parser_create(&c.cfg, &init[s])) return 1;
        jaad_parser_set_pns_state(init[s], c.pns[s]);
    }
    for (uint32_t s = 0; s < S; s++)
        if (jaad_parser_create(&c.cfg, &p[s])) return 1;
    std::atomic<int> bad{0};
    // parse batch h with T threads (stream s of the batch = corpus stream s % streams, from its start)
    auto parse_batch = [&](HostBatch& h, double* busy) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                for (uint32_t s = (uint32_t)t; s < S; s += (uint32_t)T) {
                    const uint32_t cs = s % c.streams;
                    jaad_parser_copy(p[s], init[cs]);
                    for (uint32_t j = 0; j < F; j++) {
                        const size_t f = (size_t)s * F + j, cf = f * (size_t)nch;
                        jaad_frame_out o{};
                        o.q = &h.q[cf * 1024];
                        o.sf = &h.sf[cf * 128];
                        o.cb = &h.cb[cf * 128];
                        o.ics = &h.ics[cf];
                        o.ms_used = &h.ms[f * 2];
                        o.tns = &h.tns[cf];
                        o.sbr = h.sbr.empty() ? nullptr : &h.sbr[f];
                        const auto& fb = c.fr[cs][j];
                        if (jaad_parse_frame(p[s], &c.data[fb.first], fb.second, &o)) bad = 1;
                    }
                }
            });
        for (auto& x : th) x.join();
        *busy += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    double t_parse = 0.0, t_dec = 0.0;
    parse_batch(hb[0], &t_parse);
    // one untimed decode (context warm-up: tables, staging, the GPU clock)
    if ((rc = jaad_decode_batch(ctx, &hb[0].b, pcm.data(), pcm.size(), JAAD_PCM_BIG_ENDIAN))) {
        std::fprintf(stderr, "jaad_decode_batch: %d\n", rc);
        return 1;
    }
    t_parse = 0.0;
    uint64_t frames = 0;
    int cur = 0;
    const auto t0 = std::chrono::steady_clock::now();
    double el = 0.0;
    while (el < secs && !bad) {
        // batch cur decodes on this thread while the workers parse the other one
        std::thread parser([&] { parse_batch(hb[cur ^ 1], &t_parse); });
        const auto d0 = std::chrono::steady_clock::now();
        rc = jaad_decode_batch(ctx, &hb[cur].b, pcm.data(), pcm.size(), JAAD_PCM_BIG_ENDIAN);
        t_dec += std::chrono::duration<double>(std::chrono::steady_clock::now() - d0).count();
        parser.join();
        if (rc) {
            std::fprintf(stderr, "jaad_decode_batch: %d\n", rc);
            bad = 1;
        }
        frames += (uint64_t)S * F;
        cur ^= 1;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    for (auto* x : init) jaad_parser_destroy(x);
    for (auto* x : p) jaad_parser_destroy(x);
    jaad_ctx_destroy(ctx);
    if (bad) return 1;
    const double batches = (double)frames / ((double)S * F);
    std::printf("{\"threads\": %d, \"batch_frames\": %u, \"batches\": %.0f, \"seconds\": %.3f, "
                "\"bitstream_to_pcm_frames_per_s\": %.1f, \"parse_ms_per_batch\": %.3f, \"decode_ms_per_batch\": %.3f}\n",
                T, S * F, batches, el, (double)frames / el, t_parse / batches * 1e3, t_dec / batches * 1e3);
    return 0;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s CORPUS THREADS SECONDS\n", argv[0]);
        return 2;
    }
    Corpus c;
    if (!load(argv[1], c)) {
        std::fprintf(stderr, "bad corpus %s\n", argv[1]);
        return 2;
    }
    const int T = std::max(1, std::atoi(argv[2]));
    const double secs = std::atof(argv[3]);
    if (c.cfg.channel_config < 1 || c.cfg.channel_config > 2) {  // one SCE or CPE per frame
        std::fprintf(stderr, "corpus: channel configuration %d not timed\n", (int)c.cfg.channel_config);
        return 2;
    }
    const int nch = c.cfg.channel_config;
    if (argc > 4 && std::atoi(argv[4]) > 0) return pipeline(c, T, secs, (uint32_t)std::atoi(argv[4]));
    std::atomic<int> bad{0};
    std::vector<uint64_t> frames(T, 0), bytes(T, 0);
    std::vector<double> elapsed(T, 0.0);
    auto worker = [&](int t) {
        Slot slot(nch);
        std::vector<jaad_parser*> init(c.streams), p(c.streams);
        for (uint32_t s = 0; s < c.streams; s++) {
            if (jaad_parser_create(&c.cfg, &init[s]) || jaad_parser_create(&c.cfg, &p[s])) {
                bad = 1;
                return;
            }
            jaad_parser_set_pns_state(init[s], c.pns[s]);
        }
        const auto t0 = std::chrono::steady_clock::now();
        double el = 0.0;
        uint64_t nf = 0, nb = 0;
        while (el < secs && !bad) {
            for (uint32_t s = 0; s < c.streams; s++) {
                jaad_parser_copy(p[s], init[s]);  // the stream from its start
                for (const auto& fb : c.fr[s]) {
                    const int rc = jaad_parse_frame(p[s], &c.data[fb.first], fb.second, &slot.out);
                    if (rc) {
                        std::fprintf(stderr, "parse failed: %d\n", rc);
                        bad = 1;
                        break;
                    }
                    nb += fb.second;
                }
                nf += c.frames;
            }
            el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        frames[t] = nf;
        bytes[t] = nb;
        elapsed[t] = el;
        for (uint32_t s = 0; s < c.streams; s++) {
            jaad_parser_destroy(init[s]);
            jaad_parser_destroy(p[s]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back(worker, t);
    for (auto& x : th) x.join();
    if (bad) return 1;
    uint64_t nf = 0, nb = 0;
    double el = 0.0;
    for (int t = 0; t < T; t++) {
        nf += frames[t];
        nb += bytes[t];
        el = std::max(el, elapsed[t]);
    }
    // aggregate rate = sum over threads of each thread's frames / its own time
    double fps = 0.0;
    for (int t = 0; t < T; t++) fps += (double)frames[t] / elapsed[t];
    std::printf("{\"threads\": %d, \"frames\": %llu, \"seconds\": %.3f, \"frames_per_s\": %.1f, "
                "\"frames_per_s_per_thread\": %.1f, \"bitstream_MB_per_s\": %.2f, \"bytes_per_frame\": %.1f}\n",
                T, (unsigned long long)nf, el, fps, fps / T, fps * ((double)nb / (double)nf) / 1e6,
                (double)nb / (double)nf);
    return 0;
}
