/*
 * jaad_synth.h -- seeded synthetic "parsed frame" batches in the jaad_gpu.h SoA layout.
 *
 * Stands in for the host parser (the JVM's syntacticElements.decode) in benchmarks and tests:
 * it emits what ICStream/ICSInfo/CPE.decode would have produced for a plausible AAC-LC stream
 * (SURVEY.md 8(d) "Synthetic inputs").  SplitMix64-seeded, one independent generator per stream,
 * so any subset of streams can be regenerated on its own.
 */
#ifndef JAAD_SYNTH_H
#define JAAD_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#include "jaad_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct jaad_synth_params {
    uint64_t seed;
    uint32_t n_streams;
    uint32_t frames_per_stream;
    uint8_t sf_index;         /* 3 = 48 kHz                                                  */
    uint8_t channel_config;   /* 1 SCE, 2 CPE                                                */
    uint8_t window_switching; /* 0: ONLY_LONG (C2); 1: LONG/START/SHORT/STOP machine (C3)    */
    uint8_t tns_percent;      /* % of ch-frames with TNS data (C3: 50)                       */
    uint8_t pns_percent;      /* % of bands coded with NOISE_HCB (0 in C2-C5)                */
    uint8_t is_percent;       /* % of right-channel bands coded with INTENSITY_HCB(2)       */
    uint8_t ms_mode;          /* 0 none, 1 per-band ms_used ~ Bernoulli(1/2), 2 all ones    */
    uint8_t global_gain;      /* centre of the scalefactor random walk (130)                 */
    uint8_t escape_permille;  /* per-mille of bins replaced by escapes |q| in [16,1023]      */
    uint8_t common_window;    /* CPE: 1 = common_window (C2/C3)                              */
    uint8_t sbr;              /* 1: also emit SBR records (jaad_synth_sbr), C4; 2: SBR + PS, C5 */
    uint8_t sbr_level;        /* centre of the envelope-scalefactor walk, 3 dB units        */
    uint32_t pns_state0;      /* static ICStream.randomState before the first ch-frame       */
    uint8_t coupling_percent; /* SBR CPE: % of frames with bs_coupling (balance-coded channel 1) */
    uint8_t upsample_percent; /* SBR: % of frames without usable SBR data (JAAD_SBR_UPSAMPLE)   */
    uint8_t nohdr_frames;     /* SBR: leading frames of each stream before its first SBR header */
    uint8_t reserved;
    uint32_t first_stream;    /* global index of the first stream generated: the streams
                               * [first_stream, first_stream + n_streams) of a larger job (one
                               * rank's shard); 0 with pns_percent > 0 (the PNS LCG runs over the
                               * whole job in parse order) */
} jaad_synth_params;

/* defaults for a BASELINE.json config id (1..5: C1 mono 44.1k, C2, C3, C4 HE-AAC v1, C5 HE-AAC v2) */
void jaad_synth_default(int config_id, jaad_synth_params* p);

/* Fill caller-allocated arrays (sizes: ch = channel_config, F = n_streams*frames_per_stream):
 *   q[F*ch*1024] sf[F*ch*128] cb[F*ch*128] ics[F*ch] ms_used[F*2] (CPE, may be NULL for SCE)
 *   tns[F*ch] (may be NULL => no TNS emitted) stream_slot[n_streams] frame_begin[n_streams+1]
 * Frames are stream-major: stream s owns frames [s*fps, (s+1)*fps), slot s.  threads <= 0: all
 * cores.  Returns 0 or a jaad_status. */
int jaad_synth_generate(const jaad_synth_params* p, int16_t* q, uint8_t* sf, uint8_t* cb, jaad_ics_info* ics,
                        uint64_t* ms_used, jaad_tns* tns, uint32_t* stream_slot, uint32_t* frame_begin,
                        int threads);

/* SBR records (one jaad_sbr_frame per frame, stream-major like jaad_synth_generate) for the C4
 * workload: header every frame with the Header.java defaults, start_freq 5,
 * stop_freq 9, xover 0; FIXFIX grids with 1 or 2 envelopes; envelope/noise scalefactors as
 * bounded random walks; invf_mode uniform; sinusoids rare.  coupling_percent of the CPE frames
 * are coupled (channel 1 carries the coupled grid and even balance values 0..24, as
 * SBR2.sbr_data leaves them), upsample_percent of the frames are JAAD_SBR_UPSAMPLE and the first
 * nohdr_frames frames of a stream carry no header (none seen yet).  Every band of E[][64] and
 * Q[][8] is filled (the decoder reads only n[f] / N_Q of them). */
int jaad_synth_sbr(const jaad_synth_params* p, jaad_sbr_frame* out, int threads);

#ifdef __cplusplus
}
#endif
#endif
