// Internal (host <-> device) definitions of the AAC-LC DSP kernel.  Not part of the C-ABI.
#pragma once
#include <stdint.h>

#include "../../include/jaad_gpu.h"

namespace jaad {

constexpr int kMinChunkFrames = 8;  // shortest chunk the planner makes (one re-decoded prefix frame per chunk)
// |q| < kIqHead is inverse-quantised from an LDS copy of IQ_TABLE, larger values from global memory
constexpr int kIqHead = 1024;

// One unit of work = up to N consecutive frames of one run.  A chunk that does not start its
// run first re-decodes the frame before it to rebuild the IMDCT overlap (the overlap written by
// FilterBank.process depends only on the frame that writes it:
// A/filterbank/FilterBank.java:46-51,61-70,90-100,116-118 overwrite all 1024 samples).
struct ChunkDesc {
    uint32_t frame0; // batch frame of the chunk's first iteration (the re-decoded previous frame
                     // when bit16 is set)
    uint32_t info;   // [15:0] frames, bit16 recompute previous frame, bit17 load slot state,
                     // bit18 store slot state after the last frame
    uint32_t slot;
    uint32_t skip;   // batches with dropped frames: index of the first KernelArgs::skips entry
                     // past frame0 (0 otherwise)
};
enum : uint32_t { kChunkPrefix = 1u << 16, kChunkLoadState = 1u << 17, kChunkStoreState = 1u << 18 };

// Constant tables staged into LDS once per workgroup (reference tables carried as data,
// csrc/tables/jaad_tables.inc), pre-permuted so that every lane-parallel read is
// bank-conflict free.  Built by the host (build_lds_tables), copied verbatim by the prologue.
struct alignas(16) LdsTables {
    float win_pair[2][8][64][2];  // long window [shape][s][lane u][h] = W[long_pos(lane_pos(u),2s+h)] (SINE/KBD_1024)
    float mdct_l[512][2];       // MDCT_TABLE_2048 (A/filterbank/MDCTTables.java:5), k order (pre-twiddle)
    float mdct_post[8][64][2];  // the same table for the post-twiddle: [s][lane u] = entry lane_pos(u) + 64 s
    float tw3[7][64][2];        // 512-pt IFFT pass-3 twiddles [j][lane] (FFT_TABLE_512, A/filterbank/FFTTables.java:5)
    float tw2[7][8][2];         // 512-pt IFFT pass-2 twiddles [j][lane&7]
    float tw1[4][2];            // 512-pt IFFT pass-1 (i = 4) twiddles
    float win_short[2][128];    // SINE_128, KBD_128
    float mdct_s[64][2];        // MDCT_TABLE_128 (:519)
    float roots_s[32][2];       // FFT_TABLE_64[k], k < 32 (:519)
    float sf_gain[256];         // SCALEFACTOR_TABLE[100+i] (A/syntax/ScaleFactorTable.java)
    float iq_signed[2 * kIqHead]; // q = i-kIqHead: q>0 ? IQ_TABLE[q] : -IQ_TABLE[-q] (A/syntax/ICStream.java:266)
    uint8_t quad2band_l[256];   // long window: scalefactor band of bins 4i..4i+3 (255 = none)
    uint8_t quad2band_s[32];    // short window
    int32_t nswb_l, nswb_s, tns_max_l, tns_max_s;
    // +-1 LSB kernel (mode 4): the 512-point IFFT's passes 2 and 3 as radix-8 butterflies, the
    // twiddles of register r (r = 1..7) applied before each pass's 8-point DFT: pass 2
    // W64^(bitrev3(r) * (lane >> 3)), pass 3 W512^(bitrev3(r) * lane_pos(lane)) (FFT_TABLE_512 entries)
    float tw2f[7][8][2];
    float tw3f[7][64][2];
    // +-1 LSB kernel: the post-twiddles (mdct_post, and mdct_s as the short transform's
    // post-twiddle) times 1/32767, so that the IMDCT output, the overlap in registers and the OLA
    // sum are in PCM full-scale units: v_cvt_pknorm_i16_f32 takes them without a multiply
    float mdct_post_f[8][64][2];
    float mdct_s_f[64][2];
    // +-1 LSB kernel: LONG_STOP's rising window as a long window in win_pair's lane layout, W[P] = 0
    // (P < 448), SW[P - 448] (P < 576), 1: LONG_START's falling one is W[1023 - P] (FilterBank.java:
    // 61-70, 90-100), so both run the ONLY_LONG overlap-add with this table for one half
    float win_ss[2][8][64][2];
};

// Tables only the slow paths (PNS, spec TNS) need; read from global memory.
struct GlobalTables {
    float tns_coef[4][16];      // TNS_TABLES (A/tools/TNSTables.java), zero padded
    int16_t swb_l[64];          // SWB offsets long (ScaleFactorBands.java), count+1 entries
    int16_t swb_s[16];          // SWB offsets short
};
static_assert(sizeof(LdsTables) % 16 == 0, "LdsTables must be 16-byte granular");

struct KernelArgs {
    const int16_t* q;
    const uint8_t* sf;
    const uint8_t* cb;
    const jaad_ics_info* ics;
    const uint64_t* ms_used;
    const jaad_tns* tns;
    const float* iq_table;      // full IQ_TABLE[8191] (device)
    const LdsTables* tables;    // device copy of the LDS image
    const GlobalTables* gtab;   // slow-path tables
    const ChunkDesc* chunks;
    float* state_in;            // [slot][2][1024] overlap, read by chunks with kChunkLoadState
    float* state_out;           // written by chunks with kChunkStoreState
    void* pcm;                  // frame-major output
    uint32_t n_chunks;
    uint32_t nch;               // 1 (SCE) or 2 (CPE)
    uint32_t cf_stride;         // channel-frame records per frame in q/sf/cb/ics/tns (nch; a
                                // multichannel batch: all its channels, the pointers offset to
                                // this element's first channel)
    uint32_t ms_stride;         // ms_used pairs per frame (1; multichannel: the CPE count)
    uint32_t out_mode;          // JAAD_PCM_* flags, or kOutPlanarF32 (SBR input: float [ch-frame][1024])
    uint32_t tns_mode;          // JAAD_TNS_*
    float* dbg;                 // internal: stage dump of frame dbg_frame of chunk 0 (or null)
    int dbg_frame;
    // dependent coupling (CCE terms, jaad_gpu.h jaad_cce_term): null cce_off = none.  Frame f's
    // terms are [cce_off[f], cce_off[f+1]) (BEFORE_TNS terms first); term t is CCE record
    // cce_meta[t] & 0xFFFF, targets frame channel (cce_meta[t] >> 16) & 0xFF, point cce_meta[t] >> 24, and adds
    // cce_spec[t][0..1023] (cce_term_kernel); ch0 = this launch's first channel of the frame
    const uint32_t* cce_off;
    const uint32_t* cce_meta;
    const float* cce_spec;
    uint32_t ch0;
    // batches with dropped frames (jaad_batch.frame_status): the maximal runs of dropped batch
    // frames as (first frame, count) pairs in frame order, closed by (0xFFFFFFFF, 0).  A chunk's
    // wave steps from frame f to f + 1, or past the run of dropped frames that starts there.
    // Null: no frame is dropped.
    const uint32_t* skips;
    // bounds of this launch (round 6): the batch frames its chunks may touch
    // [frame_lo, frame_hi) (q/sf/cb/ics/ms/tns/pcm rows), the state slots, the skip-list pairs (incl.
    // the sentinel) and the coupling terms.  The kernel skips a chunk whose descriptor falls outside
    // them (plan() has validated the table on the host already); a JAAD_BOUNDS build checks every
    // global access against them and prints the chunk, frame and access that failed.
    uint32_t frame_lo, frame_hi, n_slots, n_skip_pairs, n_cce_terms;
    // jaad_stream_cfg.precision: JAAD_PRECISION_LSB1 selects the fused-multiply-add instantiation of
    // the TNS-compat, uncoupled kernel (mode 4); every other mode stays bit-exact
    uint32_t precision;
    // the batch holds EIGHT_SHORT frames (the host scanned its side info, or the device-entry caller
    // said so: JAAD_HINT_SHORT_WINDOWS): the mixed-window instantiation (modes 5, 6) runs a CPE's
    // two short-window transforms in lockstep.  Either instantiation decodes every window sequence.
    uint32_t short_pair;
};

// inputs of cce_term_kernel: one wave per term
struct CceArgs {
    const int16_t* q;           // CCE records (jaad_batch.cce_*)
    const uint8_t* sf;
    const uint8_t* cb;
    const jaad_ics_info* ics;
    const uint32_t* meta;       // [term]: CCE record (bits 0..15) | target channel << 16
    const float* gain;          // [term][120]
    float* spec;                // out: [term][1024] addend, -0.0 where the reference adds nothing
    const float* iq_table;
    const LdsTables* tables;
    const GlobalTables* gtab;
    uint32_t n_terms;
};

// IFFT output position (mod 64) that lane u holds after the register transposes of the long
// IMDCT (jaad_lc.hip, imdct_long_pk): (u >> 3) + 8 * bitrev3(u & 7).
inline int lane_pos_host(int u)
{
    return (u >> 3) | ((((u & 1) << 2) | (u & 2) | ((u >> 2) & 1)) << 3);
}
// position (0..1023) of lane u's IMDCT output slot o = 2s+h (see jaad_lc.hip, long_pos)
inline int long_pos_host(int u, int o)
{
    int s = o >> 1, h = o & 1, k = lane_pos_host(u) + 64 * s;
    if (s < 4) return h ? 512 + 2 * k : 511 - 2 * k;
    return h ? 1535 - 2 * k : 2 * k - 512;
}

void build_lds_tables(int sf_index, LdsTables* t, GlobalTables* g);

}  // namespace jaad

#ifdef __HIP_PLATFORM_AMD__
#include <hip/hip_runtime_api.h>
namespace jaad {
constexpr uint32_t kOutPlanarF32 = 4;  // internal output mode: core time samples for the SBR kernel

// one wave per chunk (grid derived from a.n_chunks)
hipError_t launch_lc(const KernelArgs& a, hipStream_t stream, bool tns_spec);
// the addends of a batch's coupling terms (CCE spectrum x band gain)
hipError_t launch_cce_terms(const CceArgs& a, hipStream_t stream);
// |q| <= 8190 over n int16 values (IQ_TABLE has 8191 entries; the reference's array index would
// throw): any value beyond sets *flag to 1 (plain stores; *flag is cleared by the caller)
hipError_t launch_check_q(const int16_t* q, size_t n, int* flag, hipStream_t stream);
// SampleBuffer.accept for a multichannel frame: planar f32 [frame][n_ch][1024] -> n_ch
// interleaved samples per instant (int16 BE/LE after Math.round + clamp, or f32; JAAD_PCM_*)
// multichannel HE-AAC output: output channel c of every (frame, sample) comes from channel chan[c] of
// the [frame][sample][2] PCM at src[c] (bps-byte samples, already in the output byte order)
struct McInterleave {
    const void* src[16];
    int chan[16];
    int n_out;
};
// (skips / n_skips: the dropped-frame runs as in KernelArgs::skips, whose PCM is left as it is)
hipError_t launch_mc_interleave(const McInterleave& m, void* pcm, uint32_t n_frames, uint32_t samples, int bps,
                                hipStream_t stream, const uint32_t* skips = nullptr, uint32_t n_skips = 0);
hipError_t launch_pack(const float* planar, void* pcm, uint32_t n_frames, int n_ch, uint32_t flags,
                       hipStream_t stream, const uint32_t* skips = nullptr, uint32_t n_skips = 0);
// LC kernel waves that can be resident on one CU (occupancy query; 0 on failure)
int lc_resident_waves_per_cu(bool tns_spec);
}
#endif
