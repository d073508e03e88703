// Dev tool: time the SBR/PS host record builder (SbrHost::frame) single-threaded on the C4/C5
// synthetic records, no GPU needed.
//   g++ -O3 -std=c++17 -ffp-contract=off -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ \
//       tools/bench_sbr_host.cpp jaadec_amd/csrc/jaad_sbr_host.cpp jaadec_amd/csrc/jaad_synth.cpp -o /tmp/bsh
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../jaadec_amd/csrc/jaad_sbr.h"
#include "jaad_synth.h"

int main(int argc, char** argv)
{
    const int cfgid = argc > 1 ? std::atoi(argv[1]) : 4;
    jaad_synth_params p;
    jaad_synth_default(cfgid, &p);
    const int F = (int)(p.n_streams * p.frames_per_stream), nch = p.channel_config;
    std::vector<jaad_sbr_frame> fr(F);
    if (jaad_synth_sbr(&p, fr.data(), 0)) return 1;
    jaad::SbrHost host(p.sf_index - 3);
    std::vector<jaad::SbrHostSlot> slots(p.n_streams);
    std::vector<jaad::SbrRec> recs((size_t)F * nch);
    std::vector<float> pool((size_t)F * nch * jaad::SbrHost::kMaxEorig);
    for (int it = 0; it < 3; it++) {
        for (auto& s : slots) jaad::SbrHost::reset_slot(s);
        uint32_t epos = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (uint32_t s = 0; s < p.n_streams; s++)
            for (uint32_t j = 0; j < p.frames_per_stream; j++) {
                const size_t f = getenv("SMALL") ? ((size_t)s * p.frames_per_stream + j) % 64 : (size_t)s * p.frames_per_stream + j;
                if (getenv("PF") && j + 2 < p.frames_per_stream)
                    for (int o = 0; o < (int)sizeof(jaad_sbr_frame); o += 64)
                        __builtin_prefetch(reinterpret_cast<const char*>(&fr[f + 2]) + o);
                if (host.frame(slots[s], fr[f], nch, j == 0, s, &recs[f * nch], pool.data(), epos, 0)) return 2;
            }
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::printf("C%d: %d frames x %d ch: %.2f ms, %.1f ns per ch-frame, pool %zu floats\n", cfgid, F, nch, ms,
                    ms * 1e6 / ((double)F * nch), (size_t)epos);
    }
    return 0;
}
