// SBR (HE-AAC v1) GPU path: records shared by the host builder (jaad_sbr_host.cpp) and the
// kernel (jaad_sbr.hip).  A/ = aac/src/main/java/net/sourceforge/jaad/aac/ of the reference.
//
// Split (SURVEY.md 8a "host -> device per-frame records"): everything that depends only on
// bitstream parameters -- frequency band tables (A/sbr/FBT.java), patches and limiter tables,
// envelope/noise dequantisation (A/sbr/NoiseEnvelope.java), chirp factors, l_A, sinusoid maps,
// noise/sine table indices -- is computed on the host, in stream order, exactly as the Java does;
// everything that touches samples (QMF analysis, HF generation, envelope estimation, gains,
// HF assembly, QMF synthesis, PCM) runs in the kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <mutex>
#include <vector>

#include "jaad_gpu.h"

namespace jaad {

constexpr int kSbrMaxLE = 5;
constexpr int kSbrSynFrames = 4;  // frames per synthesis chunk (its v history is recomputed: 9 slots)

// Tables derived from one header at reset (calc_sbr_tables, patch_construction,
// limiter_frequency_table) plus the band-counter maps calculate_gain walks through
// (A/sbr/HFAdjustment.java:250-395), for each limiter-band setting.
struct SbrTab {
    uint8_t kx, M, N_Q, N_high, N_low, n_lo, n_hi, pad0;
    uint8_t N_L[4];
    uint8_t lim[4][64];       // f_table_lim[s][0..N_L[s]] - kx
    uint8_t src_p[64];        // HF generation source band of band k (0xFF: not generated)
    uint8_t g_of_k[64];       // table_map_k_to_g
    uint8_t res_map[4][2][64];  // [s][f][m]: current_res_band(2) when band m is visited
    uint8_t noise_map[4][64];   // [s][m]: current_f_noise_band
    uint8_t f_res[2][64];     // f_table_res (band borders, for interpol_freq == 0)
};

enum : uint8_t {
    kSbrReset = 1,       // sbr.reset: assembly ring refill + noise index restart
    kSbrSmooth = 2,      // bs_smoothing_mode == 0 (h_SL = 4 unless no_noise)
    kSbrInterpol = 4,    // bs_interpol_freq
    kSbrProcess = 8,     // a header has been seen (else analysis only, kx = 32)
    kSbrPsOn = 16,       // PS config: this frame carries PS data (SBR1.isPSUsed, A/sbr/SBR1.java:136)
    kSbrDep = 32,        // reads the high band of frame f-1's Xsbr rows 32..39: an HF fix pass
    kSbrLast = 64,       // the last record of its run in this call (its G/Q ring goes to the slot state)
};

// One channel-frame.  232 bytes.  The SBR stages run on the call's SBR-processed frames only,
// compacted (frames whose SBR data is unusable are upsampled instead and leave the SBR state
// alone, JAAD_SBR_UPSAMPLE): "the previous frame" of a record is the previous record of its run.
struct SbrRec {
    uint8_t L_E, lim_bands, flags;
    uint8_t no_noise;           // bit l: l == l_A || l == prevEnvIsShort  (delta = 0, no noise)
    uint16_t table;             // index into the context's SbrTab list (0: no header yet)
    uint8_t kx_prev, M_prev;
    uint16_t noise0;
    int8_t l_A;
    uint8_t first;              // first record of its run: previous-frame data comes from the slot state
    uint8_t t_E[6];
    uint8_t f[6];
    uint8_t tnb[5];             // current_t_noise_band of envelope l
    uint8_t gq0;                // GQ_ringbuf_index when the frame's first row is assembled
    uint8_t sine0;
    uint8_t blim;               // band limit of the record's run: QMF bands >= blim are zero in every
                                // row the SBR/PS stages hand on (X, X_left, all-pass output, mixed
                                // rows), so the kernels neither load nor store them (launch_sbr_stage)
    uint16_t ps_back;           // PS config: records back to the previous PS record of the run in this
                                // call (0: none, the PS state of the slot holds it)
    float lim_gain;             // limGain[bs_limiter_gains]
    uint32_t e_off;             // E_orig[l][band] at epool[e_off + sum_{l'<l} n[f[l']] + band]
    float bw[5];                // bwArray after calc_chirp_factors
    uint32_t slot;              // stream slot (state index)
    float q_div[2][5], q_div2[2][5];
    uint64_t s_index[5];        // bit m: S_index_mapped == 1
    uint64_t s_mapped[5];       // bit m: S_mapped == 1
};
static_assert(sizeof(SbrRec) == 232 && sizeof(SbrRec) <= 256, "SbrRec layout (copied by one wave, a dword per lane)");

// Per (slot, channel) state carried between calls, in global memory.  Read by the kernels of a
// call for the first frame of a run, rewritten by the last kernel of the call (sbr_state_kernel).
struct SbrChState {
    float tail[288];            // last 288 core samples of the previous frame (analysis ring)
    float xcarry[8][64][2];     // Xsbr rows 32..39 of the previous frame after HF adjustment
                                // (sbr_save_matrix: rows 0..7 of the next frame, every band)
    float xsyn[9][64][2];       // synthesis input rows 23..31 of the previous frame (v history)
    float gq[2][5][64];         // G/Q smoothing ring after the previous frame [ring position][m]
};
constexpr int kSbrCarryFloats = 8 * 64 * 2;  // per channel-frame in SbrArgs::xcarry

// Frame-parallel pipeline (one launch each, stream-ordered):
//   sbr_analysis_kernel  [ch-frame]  core time samples -> X_low  (AnalysisFilterbank)
//   sbr_hf_kernel        [ch-frame]  X_low -> synthesis input X, carry rows, gain ring
//                                    (HFGeneration, HFAdjustment); twice when smoothing is on
//   sbr_synthesis_kernel [chunk]     X -> PCM (SynthesisFilterbank64, SampleBuffer.accept)
//   sbr_state_kernel     [run, ch]   last frame of each run -> SbrChState
struct SbrChunk {
    uint32_t frame0;   // first frame (batch index)
    uint16_t n;        // frames
    uint8_t ch;
    uint8_t pad;
};

// Parametric stereo (A/ps/): device constants and per-slot state (PSImpl fields)
struct PsConst {
    float phi_qmf[64][2], phi_sub[12][2];
    float q_qmf[64][3][2], q_sub[12][3][2];
    float filter_a[3];
    float sf_iid[2][31];                 // [fine][num_steps + idx]
    float cos_alphas[8], sin_alphas[8];
    float cos_betas[2][16][8], sin_betas[2][16][8];
    float cos_gammas[2][16][8], sin_gammas[2][16][8];  // as IIDTables holds them (swapped, see PSImpl)
    float sincos_b[2][31][8];
    float p8[7], p2[7];
    float ipdopd_cos[9], ipdopd_sin[9];
};

// Rings are stored rotated so that index 0 is the next read position (the kernels run exactly
// 32 slots per frame, so every ring index inside a frame is a compile-time constant).
struct PsState {
    float2 ap[14][64];     // QMF bands <= 22 (lane = sb): [0..1] 2-slot delay, [2..4] link 0, [5..8] link 1,
                           // [9..13] link 2 (PSImpl delay_Qmf / delay_Qmf_ser)
    float2 dl[14][64];     // QMF bands 23..34: 14-slot delay; bands >= 35: dl[0] is the 1-slot delay
    float2 aph[14][16];    // hybrid groups 0..9 (delay_SubQmf / delay_SubQmf_ser), same layout as ap
    float hyb[3][12][2];   // Filterbank.buffer[band][0..11]
    float peak[20], smooth[20], pprev[20];
    float h_prev[22][8];   // h11, h12, h21, h22 real parts, then imaginary parts, per group
    float ipd_prev[20][2][2], opd_prev[20][2][2];  // PDData.prev per parameter band and phase slot
    int32_t phase_hist;
    int32_t init;
    int32_t pad[2];
};

struct SbrArgs {
    const float* time;          // [batch ch-frame][1024] core output (lc kernel, planar f32)
    const uint32_t* fmap;       // record frame -> batch frame (null: the same); the SBR stages index
                                // records, the core input and the PCM output batch frames
    const uint32_t* ups;        // batch frames output by upsampling the core (JAAD_SBR_UPSAMPLE)
    uint32_t n_ups;
    const SbrRec* recs;         // [record ch-frame]
    const float* epool;
    const SbrTab* tabs;
    float* xlow;                // [ch-frame][32 slots][32 bands][2]
    float* xsyn;                // [ch-frame][32 slots][64 bands][2] (not with PS: the HF kernel writes xps[f][0])
    float* xcarry;              // [ch-frame][8][64][2]: Xsbr rows 32..39 after HF adjustment
    float* gq;                  // [ch-frame][2][5][64] ring after the frame (smoothing / state)
    const SbrChunk* chunks;     // synthesis chunks
    const uint32_t* last_cf;    // ch-frame index of the last frame of each (run, channel)
    SbrChState* state;          // [slot][2]
    void* pcm;
    const uint32_t* fix;        // HF fix pass: the channel-frames it recomputes (kSbrDep chains)
    uint32_t n_fix;
    const uint32_t* chains;     // HF chain walker: (offset, count) per chain into the walker's part of
                                // `fix` (after the passes' lists), frames in order
    uint32_t n_chains;
    const float* noise;         // NOISE_TABLE [512][2]
    const float* qmf_c;         // [640]
    const float* dct;           // dct4_64_tab [192] + w_re [16] + w_im [16]
    // downsampled SBR (extension rate = core rate): 32-band synthesis, 1024 samples per frame
    int down;
    const float* tw32;          // qmf32_pre_twiddle [32][2] (A/sbr/SynthesisFilterbank32.java:5-38)
    uint32_t n_cf, n_chunks, n_last;
    int nch;
    uint32_t out_mode;          // JAAD_PCM_*
    int smoothing;              // some frame of the batch has bs_smoothing_mode == 0
    float* dbg;                 // debug dumps (internal, normally null)
    // parametric stereo (cfg.ps): the SBR stages run on the mono channel; the PS kernels turn
    // X_left into (X_left', X_right) in xps, the synthesis runs on xps with 2 output channels
    int ps;
    const float* zero;          // 32 rows x 64 bands x float2 of zeros: the rows all-pass lanes
                                // above their run's band limit read instead of X_left
    const jaad_ps_frame* psf;   // [frame]
    const PsConst* psc;
    PsState* pss;               // [slot]
    float* xps;                 // [frame][2][32][64][2]: X_left / raw all-pass output, then mixed
    float* xhl;                 // [frame][32][12][2] hybrid X_left
    float* xhr;                 // [frame][32][12][2] hybrid all-pass output
    float* pg;                  // [frame][32][20] P, then G_TransientRatio
    float* hb;                  // [frame][env 5][group 22][16]: H start (re 4, im 4), delta (re 4, im 4)
    const uint32_t* runs;       // [run] = (offset into ps_list, PS frame count)
    const uint32_t* ps_list;    // frames carrying PS data, run by run in time order
    uint32_t n_runs;
};

// HF fix passes launched one per chain link at most; deeper links go to the chain walker
constexpr uint32_t kSbrFixPasses = 8;
// fix_dev: channel-frames of the HF fix passes, pass after pass (fix_counts[p] in pass p), then
// the chain walker's lists (a.chains, relative to the end of the passes' lists)
hipError_t launch_sbr(const SbrArgs& a, hipStream_t stream, const uint32_t* fix_dev = nullptr,
                      const uint32_t* fix_counts = nullptr, int n_fix_passes = 0);
hipError_t launch_ps(const SbrArgs& a, hipStream_t stream);  // jaad_ps.hip, called by launch_sbr

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
struct SbrHostCh {
    float bwArray_prev[64];
    int invf_prev[5];
    uint64_t add_harmonic_prev;  // bit n = bs_add_harmonic_prev[n] (n < 49)
    int add_harmonic_flag_prev;
    int prevEnvIsShort;
    int index_noise_prev, psi_is_prev;
    int gq_index;
    int last_prev;  // t_E[L_E] of the previous frame (its HF adjusted rows up to last_prev + 1)
};

struct SbrHostSlot {
    int have_hdr;
    jaad_sbr_header hdr;
    int table;        // index into the context's table list, -1 before the first header
    int kx_prev, M_prev;
    SbrHostCh ch[2];
    // a header taken on a JAAD_SBR_UPSAMPLE frame: the frequency tables are hdr's, the patches
    // and limiter bands still those of phdr (the header of the last reset that ran
    // patch_construction / limiter_frequency_table, SbrHost::take_header)
    int mixed;
    jaad_sbr_header phdr;
    // highest band limit (SbrRec::blim) any frame of the stream has had since the last reset: PS
    // all-pass / delay state above it is zero, so above it every stage may skip the bands
    int blim_hw;
};

// Full derived tables of one header (host copy of the SBR object's table fields).
struct SbrFbt {
    int k0, k2, kx, M, N_master, N_high, N_low, N_Q, n[2];
    int f_master[65], f_table_res[2][65], f_table_noise[65], f_table_lim[4][65], N_L[4];
    int table_map_k_to_g[64];
    int noPatches, patchNoSubbands[64], patchStartSubband[64];
    int max_src;   // highest HF generation source band (-1: none)
    int gen_cnt;   // bands the patches generate (< M when patch_construction dropped one)
    // band counters of calculate_gain per limiter setting s, resolution f, band m
    int res_map[4][2][64], noise_map[4][64], hi_map[4][64];
    uint8_t visited[4][64];
};

// SBR.calc_sbr_tables for the bitstream parser (jaad_parse_sbr.cpp): band counts and f_table_res
bool sbr_tables_for_parse(int out_sf, const jaad_sbr_header& h, SbrFbt& t);

class SbrHost {
public:
    static constexpr size_t kMaxTables = 1024;  // distinct SBR headers per context
    static constexpr int kNoHeaderTable = 0;    // kx 32, M 0: the QMF banks on the low band only
    explicit SbrHost(int out_sf_index);
    static void reset_slot(SbrHostSlot& s);
    // Header.differs (A/sbr/Header.java:70-78): would this header reset the tables
    static bool header_changes(const jaad_sbr_header& a, const jaad_sbr_header& b);
    // Build the records of one frame of one stream (both channels) in stream order.
    // Returns 0 or a jaad_status; writes the E_orig values at epool[epos..] (epos advances; the
    // record's e_off is e_base + epos) -- room for kMaxEorig floats per channel is the caller's.
    // Thread-safe across slots.
    static constexpr int kMaxEorig = 5 * 49;
    int frame(SbrHostSlot& st, const jaad_sbr_frame& fr, int nch, bool first, uint32_t slot, SbrRec* rec_out,
              float* epool, uint32_t& epos, uint32_t e_base);
    const std::vector<SbrTab>& tabs() const { return tabs_; }
    // table index for a header (built on first use); -1 if its tables are invalid
    int table_index(const jaad_sbr_header& h) { return table_for(h); }
    // the table a slot's state uses (pure or mixed, see SbrHostSlot.mixed); -1 if invalid
    int table_index(const SbrHostSlot& s) { return s.mixed ? mixed_for(s.hdr, s.phdr) : table_for(s.hdr); }
    // The header of a JAAD_SBR_UPSAMPLE frame.  SBR.decode reads it into this.hdr and, when it
    // differs, recomputes the frequency tables (calc_sbr_tables, A/sbr/SBR.java:168-177,212-221)
    // even though the frame's SBR then does not run; patch_construction and
    // limiter_frequency_table run only inside a processed frame's HF generation with its own reset
    // flag (A/sbr/HFGeneration.java:27-28,95-97), so the next frames use the new frequency tables
    // with the old patches and limiter bands until a processed frame resets.  JAAD_ERR_UNSUPPORTED
    // where that mix would make the reference read outside its arrays or stale values (a different
    // M, a patch past band 63, a patch source at or above the new kx, no previous header).
    int take_header(SbrHostSlot& st, const jaad_sbr_header& h);

private:
    int out_sf_;
    std::mutex mu_;                                  // guards table creation
    std::vector<SbrTab> tabs_;                       // capacity fixed: elements never move
    std::vector<std::unique_ptr<SbrFbt>> fbt_;
    std::vector<jaad_sbr_header> keys_;
    std::vector<std::pair<jaad_sbr_header, jaad_sbr_header>> mixed_keys_;
    std::vector<int> mixed_idx_;
    int table_for(const jaad_sbr_header& h);
    int mixed_for(const jaad_sbr_header& h, const jaad_sbr_header& ph);
    int push_table(std::unique_ptr<SbrFbt> t, const jaad_sbr_header& key);
};

}  // namespace jaad
