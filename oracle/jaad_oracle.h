/*
 * jaad_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference decoder's DSP path (pucgenie/JAADec, Java), used as
 * the parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  It
 * is never linked into, loaded by or called from the product library (libjaadgpu.so).
 *
 * PARITY STATUS: the reference ships no golden vectors, known-answer tests or fixtures for
 * this path (its only test, src/test/java/PlayGoldDust.java, asserts nothing) and it cannot be
 * run here (Java; no JDK in this image).  Parity of this restatement with the Java code is
 * therefore "parity unpinned" by reference outputs; it is pinned instead by (i) op-for-op
 * restatement under strict binary32 semantics (-O2 -ffp-contract=off, no FMA -- Java >= 17 is
 * strict IEEE float without contraction), (ii) independent float64 closed-form checks in
 * tests/test_oracle.py, (iii) committed fixtures in tests/golden/.
 */
#ifndef JAAD_ORACLE_H
#define JAAD_ORACLE_H

#include "../include/jaad_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_sbr orc_sbr;
typedef struct orc_ps orc_ps;

/* per-stream state of the restated decoder: ICStream.overlap per channel (A/syntax/ICStream.java:47)
 * and the SBR object of the channel element (allocated on first use, freed by orc_streams_free) */
typedef struct orc_stream {
    float overlap[2][1024];
    orc_sbr* sbr;
} orc_stream;
size_t orc_stream_bytes(void);
void orc_streams_free(orc_stream* streams, int n);

/* FFT.process (A/filterbank/FFT.java:48-135), in place, n = 64 or 512 */
void orc_fft(float (*data)[2], int n, int forward);
/* MDCT.process (A/filterbank/MDCT.java:36-81), N = 2048 or 256 */
void orc_imdct(const float* in, float* out, int N);
/* FilterBank.process (A/filterbank/FilterBank.java:39-123) */
void orc_filterbank(int window_sequence, int shape, int shape_prev, const float* in, float* out,
                    float* overlap);
/* ICStream.decodeSpectralData inverse quantisation + PNS (A/syntax/ICStream.java:222-275).
 * *rand_state is the static ICStream.randomState, advanced in place. */
int orc_dequant(const jaad_ics_info* info, int sf_index, const int16_t* q, const uint8_t* sf,
                const uint8_t* cb, uint32_t* rand_state, float* iq);
/* MS.process (A/tools/MS.java:17-41) and IS.process (A/tools/IS.java:17-53) */
void orc_ms(const jaad_ics_info* infoL, int sf_index, const uint8_t* cbL, const uint8_t* cbR,
            const uint64_t* ms_used, float* L, float* R);
void orc_is(const jaad_ics_info* infoL, const jaad_ics_info* infoR, int sf_index, const uint8_t* cbR,
            const uint8_t* sfR, const uint64_t* ms_used, float* L, float* R);
/* ISO/IEC 14496-3 4.6.9 TNS synthesis filter ("spec" mode; the reference's TNS.process is a
 * no-op, so this is NOT reference behaviour and its parity is unpinned). */
void orc_tns_spec(const jaad_ics_info* info, int sf_index, const jaad_tns* tns, float* spec);

/* SampleBuffer.accept PCM packing of one frame (S/SampleBuffer.java:168-209): n_ch channel
 * arrays of `len` samples -> interleaved int16 (flags: JAAD_PCM_*) or f32; returns clip count */
int orc_pcm_pack(const float* const* ch, int n_ch, int len, uint32_t flags, void* out);

/* Decode a whole batch (host arrays), mirroring SyntacticElements.process + SampleBuffer.accept
 * for an SCE or CPE configuration.  streams[] is indexed by batch->stream_slot[]. */
int orc_decode_batch(const jaad_stream_cfg* cfg, orc_stream* streams, const jaad_batch* batch,
                     void* pcm_out, size_t pcm_bytes, uint32_t flags);

/* Same, multithreaded over runs (runs are independent streams); threads <= 0: all cores */
int orc_decode_batch_mt(const jaad_stream_cfg* cfg, orc_stream* streams, const jaad_batch* batch,
                        void* pcm_out, size_t pcm_bytes, uint32_t flags, int threads);

/* ---- SBR (jaad_oracle_sbr.c) ---- */
size_t orc_sbr_bytes(void);
void orc_sbr_init(orc_sbr* s, int out_sf_index);
/* SBR.decode for one frame's parsed SBR data (header handling, NoiseEnvelope dequantisation) */
int orc_sbr_decode(orc_sbr* s, const jaad_sbr_frame* fr, int nch);
int orc_sbr_take_header(orc_sbr* s, const jaad_sbr_header* h);
/* SBR2.process / SBR1.process (no PS): 2048-float channel buffers, first 1024 = core output */
void orc_sbr_process(orc_sbr* s, float* left, float* right, int nch);
/* SBR.downSampled (extension rate = core rate): 32-band synthesis, 1024 samples per channel */
void orc_sbr_set_downsampled(orc_sbr* s, int down);
/* SynthesisFilterbank32.synthesis over one frame: X[32][64][2] (bands < 32) -> 1024 samples */
void orc_qmf_synthesis32_frame(float* v1280, int* v_index, const float* X, float* output1024);
/* DCT.dct4_kernel (A/sbr/DCT.java:347-391) on copies of the inputs */
void orc_sbr_dct4(const float* in_re, const float* in_im, float* out_re, float* out_im);
/* AnalysisFilterbank.sbr_qmf_analysis_32 over one frame: X[32][64][2] */
void orc_qmf_analysis_frame(float* v1280, int* v_index, const float* input1024, float* X, int kx);
/* SynthesisFilterbank64.synthesis over one frame: X[32][64][2] -> 2048 samples */
void orc_qmf_synthesis_frame(float* v2560, int* v_index, const float* X, float* output2048);
void orc_sbr_free(orc_sbr* s);
/* ---- PS (jaad_oracle_ps.c) ---- */
size_t orc_ps_bytes(void);
void orc_ps_init(orc_ps* ps);
void orc_ps_set_frame(orc_ps* ps, const jaad_ps_frame* f);
/* PSImpl.process on X_left/X_right [38][64][2] (A/ps/PSImpl.java:685-707) */
void orc_ps_process(orc_ps* ps, float (*X_left)[64][2], float (*X_right)[64][2]);
void orc_ps_hybrid_analysis(const float* X, float* X_hybrid);
/* derived frequency tables for a header: info = k0 k2 kx M N_master N_high N_low N_Q noPatches N_L */
int orc_sbr_table_info(const jaad_sbr_header* h, int out_sf_index, int* info, int* f_master, int* f_table_lim);

#ifdef __cplusplus
}
#endif
#endif
