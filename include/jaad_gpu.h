/*
 * jaad_gpu.h -- C-ABI drop-in boundary for the DSP half of JAAD's decoder.
 *
 * The reference decoder (pucgenie/JAADec, pure Java) runs, per frame,
 *     Decoder.decode0                       A/Decoder.java:103-121
 *       syntacticElements.decode(in)        parse + Huffman        (stays on the host)
 *       syntacticElements.process()         DSP                    (REPLACED by this library)
 *       buffer.accept(channels, len, rate)  SampleBuffer PCM pack  (REPLACED by this library)
 * (A/ = aac/src/main/java/net/sourceforge/jaad/aac/).  The host parser emits, instead of
 * dequantised floats, the quantised spectrum plus the side information listed below, for
 * MANY frames of MANY streams at once; one call turns the batch into interleaved int16 PCM
 * byte-identical in layout to SampleBuffer.accept (S/SampleBuffer.java:168-209).
 *
 * Plain C types only: the JNI glue passes direct-ByteBuffer addresses.
 * Every entry point returns an int status (0 = ok, <0 = jaad_status); nothing throws.
 */
#ifndef JAAD_GPU_H
#define JAAD_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JAAD_ABI_VERSION 4u

/* ---- status codes (JNI maps every nonzero code to AACException, A/AACException.java) ---- */
typedef enum jaad_status {
    JAAD_OK = 0,
    JAAD_ERR_INVALID_ARG = -1,   /* NULL/short buffer, bad sizes                              */
    JAAD_ERR_NO_DEVICE = -2,     /* no usable gfx950 device / HIP runtime                    */
    JAAD_ERR_HIP = -3,           /* a HIP runtime call failed                                 */
    JAAD_ERR_UNSUPPORTED = -4,   /* profile/config not decodable (A/Decoder.java:115-116)     */
    JAAD_ERR_BITSTREAM = -5,     /* side info out of range, e.g. max_sfb > swb count          */
    JAAD_ERR_NOMEM = -6,
    JAAD_ERR_ABI = -7,           /* jaad_stream_cfg.abi_version mismatch                      */
    JAAD_ERR_EOS = -8            /* a frame's bitstream ended early (EOSException: the reference
                                    drops the frame, A/Decoder.java:96-100)                    */
} jaad_status;

/* ---- ICSInfo.WindowSequence ordinals (A/syntax/ICSInfo.java:26-53) ---- */
enum {
    JAAD_ONLY_LONG_SEQUENCE = 0,
    JAAD_LONG_START_SEQUENCE = 1,
    JAAD_EIGHT_SHORT_SEQUENCE = 2,
    JAAD_LONG_STOP_SEQUENCE = 3
};

/* ---- section codebooks with DSP meaning (A/huffman/HCB.java) ---- */
enum {
    JAAD_ZERO_HCB = 0,
    JAAD_FIRST_PAIR_HCB = 5,
    JAAD_ESCAPE_HCB = 11,
    JAAD_NOISE_HCB = 13,
    JAAD_INTENSITY_HCB2 = 14,
    JAAD_INTENSITY_HCB = 15
};

/* ---- TNS handling ---- */
enum {
    JAAD_TNS_COMPAT = 0,  /* reference behaviour: TNS.process is a no-op (A/tools/TNS.java:63-68)  */
    JAAD_TNS_SPEC = 1     /* ISO/IEC 14496-3 4.6.9 all-pole filtering (parity unpinned by the ref) */
};

/* ---- output format flags for jaad_decode_* ---- */
enum {
    JAAD_PCM_BIG_ENDIAN = 0u,     /* SampleBuffer default (S/SampleBuffer.java:28-30)            */
    JAAD_PCM_LITTLE_ENDIAN = 1u,  /* SampleBuffer.setBigEndian(false)                             */
    JAAD_PCM_FLOAT32 = 2u,        /* native-endian f32 samples BEFORE Math.round (tolerance checks) */
    /* jaad_decode_batch_device only (a performance hint, never a change of output): the batch holds
       EIGHT_SHORT_SEQUENCE frames -- the host parser saw their window_sequence -- so the kernel built
       for mixed windows runs (a CPE's two short-window transforms in lockstep).  Without it the
       long-window kernel decodes short frames too, one channel after the other.  jaad_decode_batch
       scans the side info itself and ignores the bit. */
    JAAD_HINT_SHORT_WINDOWS = 1u << 8
};

/*
 * Stream configuration: what DecoderConfig.decode (A/DecoderConfig.java:175-254) derives from
 * the AudioSpecificConfig.  One context serves any number of streams sharing one config.
 */
typedef struct jaad_stream_cfg {
    uint32_t abi_version;     /* = JAAD_ABI_VERSION                                             */
    uint8_t profile;          /* audio object type of the core: 2 = AAC LC (only one supported)  */
    uint8_t sf_index;         /* core SampleFrequency index 0..11 (A/SampleFrequency.java:15-26) */
    uint8_t channel_config;   /* 1 = one SCE (mono), 2 = one CPE (stereo)                        */
    uint8_t tns_mode;         /* JAAD_TNS_COMPAT | JAAD_TNS_SPEC                                  */
    uint8_t sbr;              /* 1 = explicit SBR (AOT 5): jaad_batch.sbr carries one record/frame  */
    uint8_t ps;               /* 1 = parametric stereo (AOT 29): SCE core + SBR + PS -> stereo;
                                 requires sbr = 1 and channel_config = 1                         */
    uint8_t ext_sf_index;     /* SBR output SampleFrequency index (extensionSampleFrequency of the
                                 ASC, A/DecoderConfig.java:184-198); must be the core index - 3,
                                 i.e. twice the core rate (bs_samplerate_mode = 1)                */
    uint8_t precision;        /* JAAD_PRECISION_EXACT (0, the default): PCM bit-identical to the
                                 reference's binary32 arithmetic; JAAD_PRECISION_LSB1: PCM within
                                 +-1 LSB of it (BASELINE.json's bar) -- the AAC-LC transforms use
                                 fused multiply-adds (fewer, shorter dependent operations).  Coupling,
                                 spec TNS and the SBR/PS stages stay exact in either mode.        */
} jaad_stream_cfg;

enum {
    JAAD_PRECISION_EXACT = 0,
    JAAD_PRECISION_LSB1 = 1
};

/*
 * Per channel-frame side information (16 bytes), one per ICStream per frame.
 * Filled by the host from ICSInfo.decode (A/syntax/ICSInfo.java:86-119) and ICStream.decode.
 */
typedef struct jaad_ics_info {
    uint8_t window_sequence;   /* JAAD_*_SEQUENCE                                                 */
    uint8_t window_shape;      /* ICSInfo.windowShape[CURRENT]: 0 sine, 1 KBD                      */
    uint8_t window_shape_prev; /* ICSInfo.windowShape[PREVIOUS]                                    */
    uint8_t max_sfb;           /* <= swb count of the window type                                  */
    uint8_t grouping;          /* EIGHT_SHORT only: bit i (i=0..6) set <=> window i+1 is in the same
                                  group as window i, i.e. the i-th scale_factor_grouping bit read by
                                  A/syntax/ICSInfo.java:97-104. 0 for long windows.               */
    uint8_t flags;             /* JAAD_ICS_* below                                                 */
    uint8_t reserved[2];
    uint32_t pns_state;        /* value of the static ICStream.randomState (A/syntax/ICStream.java:26)
                                  when this ICStream's decodeSpectralData started                 */
    uint32_t reserved2;
} jaad_ics_info;

enum {
    JAAD_ICS_HAS_PNS = 1u << 0,     /* some band uses NOISE_HCB                                  */
    JAAD_ICS_HAS_IS = 1u << 1,      /* some band uses INTENSITY_HCB(2) (right channel of a CPE)  */
    JAAD_ICS_TNS = 1u << 2,         /* tns_data_present (coefficients in jaad_batch.tns)         */
    JAAD_ICS_MS_PRESENT = 1u << 3,  /* left channel of a CPE: common_window && ms_mask != ALL_0
                                       (A/syntax/CPE.java:149-153, isMSMaskPresent)             */
    JAAD_ICS_COMMON_WINDOW = 1u << 4
};

/*
 * TNS side info per channel-frame (TNS.decode, A/tools/TNS.java:35-61).  Up to 8 filters in
 * total (long: <=3 in window 0; short: <=1 per window).  coef[] holds the 4-bit indices read
 * from the bitstream; the value is TNS_TABLES[2*compress+res][idx] (A/tools/TNSTables.java).
 */
typedef struct jaad_tns_filter {
    uint8_t window;    /* 0..7                                   */
    uint8_t length;    /* in scale factor bands                  */
    uint8_t order;     /* 0..20 (>20 rejected as the ref does)    */
    uint8_t flags;     /* bit0 direction, bit1 coef_res, bit2 coef_compress */
    uint8_t coef[20];
} jaad_tns_filter;

typedef struct jaad_tns {
    uint8_t n_filters; /* 0..8, filters ordered by (window, filt) as parsed */
    uint8_t reserved[3];
    jaad_tns_filter filt[8];
} jaad_tns;

/*
 * SBR side information of one frame, as the reference's parser leaves it after sbr_data
 * (A/sbr/SBR.java:161-245, SBR1.sbr_data :34-60, SBR2.sbr_data :35-135).  Host memory only.
 */
typedef struct jaad_sbr_header {   /* Header.decode (A/sbr/Header.java:24-62), defaults applied */
    uint8_t amp_res, start_freq, stop_freq, xover_band;
    uint8_t freq_scale, alter_scale, noise_bands, limiter_bands;
    uint8_t limiter_gains, interpol_freq, smoothing_mode, reserved;
} jaad_sbr_header;

typedef struct jaad_sbr_channel {  /* Channel fields after sbr_data (A/sbr/Channel.java) */
    uint64_t add_harmonic;         /* bit n = bs_add_harmonic[n], n < N_high (sinusoidal_coding)     */
    int16_t E[5][64];              /* [env][band] envelope scalefactors after extract_envelope_data  */
    int16_t Q[2][8];               /* [noise env][band] after extract_noise_floor_data (N_Q <= 5)   */
    uint8_t frame_class;           /* FrameClass ordinal: FIXFIX, FIXVAR, VARFIX, VARVAR            */
    uint8_t L_E, L_Q, bs_pointer;  /* envelopes (1..5), noise envelopes (1..2), pointer             */
    uint8_t t_E[6];                /* envelope time borders (envelope_time_border_vector, :455-542) */
    uint8_t t_Q[3];                /* noise time borders (noise_floor_time_border_vector, :544-556) */
    uint8_t f[6];                  /* frequency resolution per envelope (0 = LO_RES, 1 = HI_RES)    */
    uint8_t invf_mode[5];          /* bs_invf_mode per noise band                                   */
    uint8_t add_harmonic_flag;
    uint8_t reserved[7];
} jaad_sbr_channel;                /* 712 bytes */

/*
 * Parametric stereo parameters of one frame as PSImpl.ps_data_decode leaves them
 * (A/ps/PSImpl.java:137-199): envelope borders and delta-decoded IID/ICC (and IPD/OPD) indices
 * per parameter band.
 */
typedef struct jaad_ps_frame {
    uint8_t iid_mode, icc_mode;    /* IIDMode / ICCMode ids 0..5 (A/ps/IIDMode.java:48-55)           */
    uint8_t num_env;               /* 1..5 after ps_data_decode                                      */
    uint8_t nr_ipdopd_par;         /* Extension.nr_par(): 0 without the IPD/OPD extension, else 11
                                      or 17 (A/ps/Extension.java:81-86, A/ps/ExtData.java:55-60)     */
    uint8_t border[6];             /* border_position[0..num_env]                                     */
    uint8_t reserved[2];
    int8_t iid[5][34];             /* iid_index[env][bk]  (|.| <= 7 normal, <= 15 fine)              */
    int8_t icc[5][34];             /* icc_index[env][bk]  (0..7)                                     */
    int8_t ipd[5][17];             /* ipd_index[env][bk]  (0..7, PDMode.clip)                        */
    int8_t opd[5][17];             /* opd_index[env][bk]; carried as parsed, but the reference's
                                      mixing reads the IPD index for both (A/ps/PSImpl.java:502-503) */
    uint8_t pad[6];
} jaad_ps_frame;                   /* 528 bytes */

/* jaad_sbr_frame.status */
enum {
    /* sbr_data decoded (SBR.decode sets valid, A/sbr/SBR.java:179-184).  Before the stream's first
       SBR header the reference marks the element valid too and runs the QMF banks on the low band
       only (Channel.process_channel with hdr == null, A/sbr/Channel.java:589-617): the library
       does the same for such frames (header_present = 0 and no header seen yet on the slot).  */
    JAAD_SBR_OK = 0,
    /* the element has no usable SBR data this frame: no SBR payload followed it, or sbr_data
       failed (a grid whose borders do not fit, A/sbr/Channel.java:418-432).  The reference then
       skips SBR entirely -- its state stays as the last processed frame left it -- and outputs
       the core upsampled by sample repetition (SBR.upsample, A/sbr/SBR.java:302-309, which never
       writes index 1; A/syntax/CPE.java:196-204, SCE.java:123-132).  With a downsampled-SBR
       configuration (output rate = core rate) the core is output as it is.                     */
    JAAD_SBR_UPSAMPLE = 1
};

typedef struct jaad_sbr_frame {
    uint8_t header_present;        /* bs_header_flag: hdr below is this frame's sbr_header           */
    uint8_t coupling;              /* bs_coupling (CPE only)                                         */
    uint8_t ps_present;            /* PS data decoded for this frame (SBR1.isPSUsed, A/sbr/SBR1.java:136) */
    uint8_t status;                /* JAAD_SBR_OK / JAAD_SBR_UPSAMPLE (the rest of the record is then
                                      ignored except header_present/hdr, which must not change the
                                      slot's tables: the reference would lose that reset)         */
    jaad_sbr_header hdr;
    jaad_sbr_channel ch[2];        /* ch[1] unused for an SCE                                        */
    jaad_ps_frame ps;              /* valid when ps_present                                          */
} jaad_sbr_frame;                  /* 1968 bytes */

/*
 * Dependent coupling (coupling_channel_element, A/syntax/CCE.java).  A CCE's ICStream is carried
 * as a record in jaad_batch.cce_q/cce_sf/cce_cb/cce_ics (the same layouts as the channel records;
 * its spectrum is ICStream.decodeSpectralData's, PNS from cce_ics.pns_state).  Each application
 * of CCE.applyDependentCoupling (:188-215) to a target channel, as
 * ChannelElement.processDependentCoupling (A/syntax/ChannelElement.java:105-130) makes them, is one
 * term: target[k] += gain[idx] * cce_spectrum[k] over the CCE's bands idx = g*max_sfb+sfb whose
 * sfbCB != ZERO_HCB (all windows of the group).  Terms of a frame are listed in the reference's
 * order (CCEs in bitstream order, then coupled targets in order).  The reference applies them
 * after M/S and I/S in two passes, every point-0 (BEFORE_TNS) term, TNS, then every point-1
 * (AFTER_TNS) term; the library does the same.  The reference's TNS is a no-op, so only the order
 * of the additions tells the points apart in JAAD_TNS_COMPAT mode; in JAAD_TNS_SPEC mode the
 * point-1 terms are added after the spec filters (channel configurations 1 and 2; JAAD_TNS_SPEC
 * batches with terms in configurations 3..7 are refused).  Independent switching
 * CCEs (ind_sw_cce_flag) never apply in the reference (couplingPoint becomes 3, matching neither
 * BEFORE_TNS, AFTER_TNS nor AFTER_IMDCT: CCE.java:113-129), so they produce no terms.
 * Limits (JAAD_ERR_UNSUPPORTED): a gain that is not finite or whose magnitude exceeds
 * JAAD_CCE_GAIN_MAX (the reference's (float)Math.pow(scale, -t) of a long gain walk, where its
 * spectrum and IMDCT overflow to inf/NaN), and more than 65536 CCE records in one batch (the
 * 16-bit jaad_cce_term.cce).
 */
#define JAAD_CCE_GAIN_MAX 1.152921504606846976e18f /* 2^60 */
#define JAAD_CCE_MAX_RECORDS 65536u
typedef struct jaad_cce_term {
    uint32_t frame;    /* batch frame (terms sorted by frame)                                  */
    uint8_t channel;   /* target channel within the frame (0 .. channels-1)                      */
    uint8_t point;     /* 0 BEFORE_TNS, 1 AFTER_TNS                                               */
    uint16_t cce;      /* CCE record (index into cce_q / cce_sf / cce_cb / cce_ics)               */
    float gain[120];   /* CCE.gain[index][idx] for idx < groups * max_sfb of the CCE's ICS       */
} jaad_cce_term;       /* 488 bytes */

/*
 * A batch: n_frames frames (raw_data_blocks) of one channel configuration.  Frames are grouped
 * in runs: run r holds consecutive-in-time frames [frame_begin[r], frame_begin[r+1]) of the
 * stream whose persistent DSP state (IMDCT overlap, ...) lives in context slot stream_slot[r].
 * A run continues its slot's stream exactly where the previous call left it.
 *
 * ch-frame index = frame * channels + ch  (channels = 1 for an SCE config, 2 for a CPE config).
 * Arrays marked [dev] live in device memory for jaad_decode_batch_device and in host memory
 * for jaad_decode_batch; the run arrays are always host memory.
 */
typedef struct jaad_batch {
    uint32_t n_frames;
    uint32_t n_runs;
    const uint32_t* stream_slot;  /* [n_runs]   host                                             */
    const uint32_t* frame_begin;  /* [n_runs+1] host, frame_begin[0] = 0, frame_begin[n_runs] = n_frames */
    const int16_t* q;             /* [dev] [ch-frame][1024] quantised coefficients, ICStream iqData order
                                     (window-major for EIGHT_SHORT, A/syntax/ICStream.java:229-274);
                                     bins >= swb_offset[max_sfb] of each window must be 0          */
    const uint8_t* sf;            /* [dev] [ch-frame][128]: per (group, sfb) band, idx = g*max_sfb+sfb:
                                     scalefactor-table index minus 100, i.e. the gain is
                                     SCALEFACTOR_TABLE[sf+100] (negated for NOISE_HCB);
                                     spectral: global-gain sum; noise: clip(off1,-100,155)+100;
                                     intensity: 100-clip(off2,-155,100) (A/syntax/ICStream.java:172-220) */
    const uint8_t* cb;            /* [dev] [ch-frame][128] section codebook per band (sfbCB)       */
    const jaad_ics_info* ics;     /* [dev] [ch-frame]                                              */
    const uint64_t* ms_used;      /* [dev] [frame][2] bit idx = g*max_sfb+sfb (CPE only, else NULL) */
    const jaad_tns* tns;          /* [dev] [ch-frame] or NULL when no ch-frame sets JAAD_ICS_TNS    */
    const jaad_sbr_frame* sbr;    /* host [frame] when cfg.sbr ([frame][channel element] for channel
                                     configurations 3..7), else NULL                             */
    /* dependent coupling (jaad_cce_term above); all zero / NULL for a batch without CCEs.  JAAD_TNS_SPEC
       mode: channel configurations 1 and 2 only (JAAD_ERR_UNSUPPORTED otherwise). */
    uint32_t n_cce;               /* CCE records                                                    */
    uint32_t n_cce_terms;
    const int16_t* cce_q;         /* [dev] [n_cce][1024]                                            */
    const uint8_t* cce_sf;        /* [dev] [n_cce][128]                                             */
    const uint8_t* cce_cb;        /* [dev] [n_cce][128]                                             */
    const jaad_ics_info* cce_ics; /* [dev] [n_cce]                                                  */
    const jaad_cce_term* cce_terms; /* host [n_cce_terms]                                           */
    /* per-frame status (ABI 4): host [n_frames] of JAAD_FRAME_*, or NULL = every frame decodes.  A
       frame marked JAAD_FRAME_EOS is dropped as Decoder.decodeFrame drops a frame whose bitstream
       ended early (it catches the EOSException and skips process() and buffer.accept,
       A/Decoder.java:89-101): no DSP runs for it, its PCM slot in the output is left as it is, and
       its stream's state is the one the previous decoded frame left, so the run's next frame
       continues from there.  Its records are not read (they may be zero).  The other frames of the
       batch decode as usual. */
    const uint8_t* frame_status;
} jaad_batch;

/* jaad_batch.frame_status values */
enum {
    JAAD_FRAME_DECODE = 0,
    JAAD_FRAME_EOS = 1     /* dropped: the parser hit the end of this frame's bitstream (EOSException) */
};

typedef struct jaad_ctx jaad_ctx;

/* DecoderConfig.getSampleLength (A/DecoderConfig.java:83-86) and getChannelCount (:108-115).
 * Note: a mono (SCE) stream is emitted as 2 identical channels, as SyntacticElements.process
 * does (A/syntax/SyntacticElements.java:243-245).                                          */
int jaad_cfg_sample_length(const jaad_stream_cfg* cfg);
int jaad_cfg_channel_count(const jaad_stream_cfg* cfg);
/* bytes of PCM one frame produces for the given output flags */
size_t jaad_frame_pcm_bytes(const jaad_stream_cfg* cfg, uint32_t flags);

/* Create a context bound to HIP device `device` with `n_slots` independent stream states
 * (each as freshly created by Decoder.create: overlap zero, window shapes sine).            */
int jaad_ctx_create(const jaad_stream_cfg* cfg, uint32_t n_slots, int device, jaad_ctx** out);
void jaad_ctx_destroy(jaad_ctx* ctx);
/* channels per ch-frame record of the context's batches: 1 (SCE core) or 2 (CPE core); this,
 * not jaad_cfg_channel_count (the PCM channel count), sizes q/sf/cb/ics/tns.  Used by the JNI
 * glue to check the Java side's buffers against the context.                               */
int jaad_ctx_core_channels(const jaad_ctx* ctx);

/* Synchronous host-buffer entry: copies the batch to the device, runs the DSP, copies
 * n_frames * jaad_frame_pcm_bytes(flags) bytes of PCM back to pcm_out (frame-major; the slots of
 * frames marked JAAD_FRAME_EOS are not written).
 * Replaces the per-frame Decoder.decodeFrame(byte[], SampleBuffer) (A/Decoder.java:131-150)
 * for a batch of already parsed frames.  The side info is range-checked first
 * (JAAD_ERR_BITSTREAM, every slot's state left as before the call).  Dropped frames (ABI 4
 * frame_status) are left out of the call's plan: one launch sequence decodes every run's kept
 * frames as consecutive ones (the SBR header of a dropped frame whose payload was parsed whole is
 * still taken, as for a JAAD_SBR_UPSAMPLE frame).  An AAC-LC batch of >= 4096 frames without
 * dropped frames is cut into run-aligned pieces whose copies and kernels overlap; caller
 * buffers registered with jaad_host_register are copied by DMA directly, others through
 * page-locked staging.                                                                      */
int jaad_decode_batch(jaad_ctx* ctx, const jaad_batch* batch, void* pcm_out, size_t pcm_bytes,
                      uint32_t flags);

/* On an error status the PCM buffer's contents are unspecified (pieces decoded before a later piece
 * failed its checks may have been written); the stream states are as before the call.        */

/* Page-lock [p, p + bytes) (hipHostRegister) for the context's host-buffer entry: batch arrays
 * and PCM buffers that lie inside a registered range skip the staging copy.  Register buffers
 * that are reused call after call (a JNI caller: its direct ByteBuffers, once per stream);
 * unregister before freeing them.  jaad_ctx_destroy unregisters what is left.  Memory that is
 * page-locked already (hipHostMalloc) is accepted and only recorded.  Registering the same start
 * address again is a no-op (JAAD_ERR_INVALID_ARG if it asks for a longer range).             */
int jaad_host_register(jaad_ctx* ctx, void* p, size_t bytes);
int jaad_host_unregister(jaad_ctx* ctx, void* p);
/* Page-locked host memory owned by the context (hipHostMalloc), counted as registered: batch
 * arrays and PCM buffers placed in it are copied by DMA directly.  A JNI caller wraps it in a
 * direct ByteBuffer.  jaad_host_free releases it (after the context's work
 * that may read it); jaad_ctx_destroy frees what is left.                                    */
int jaad_host_alloc(jaad_ctx* ctx, size_t bytes, void** p);
int jaad_host_free(jaad_ctx* ctx, void* p);

/* Device-resident entry: all [dev] arrays and pcm_dev are device pointers; work is queued on
 * `hip_stream` (a hipStream_t, NULL = the context's stream) and the call returns without
 * waiting.  Calls on one context must not overlap in time on the host; on the device every
 * call is ordered after the context's previous call whatever stream either was queued on,
 * and jaad_wait / jaad_state_* wait for all of them.
 * The side info is NOT range-checked on the host here (that would read device memory): the
 * kernels clamp it instead (window_sequence & 3, window shapes & 1, max_sfb to the window's
 * swb count, |q| to 8190, TNS window & 7 / order <= 20), so a malformed batch decodes to
 * garbage PCM but never reads or writes outside its buffers.  jaad_decode_batch rejects the
 * same batch with JAAD_ERR_BITSTREAM.                                                     */
int jaad_decode_batch_device(jaad_ctx* ctx, const jaad_batch* batch, void* pcm_dev, size_t pcm_bytes,
                             uint32_t flags, void* hip_stream);
int jaad_wait(jaad_ctx* ctx);

/* Per-slot persistent DSP state (seek/resume, A/syntax/ICStream.java:47,56 overlap, ...).
 * The blob is opaque and specific to the library build that wrote it (its layout follows the
 * kernels' state records): resume within one deployment, do not persist it across upgrades. */
size_t jaad_state_bytes(const jaad_ctx* ctx);
int jaad_state_export(jaad_ctx* ctx, uint32_t slot, void* buf, size_t bytes);
int jaad_state_import(jaad_ctx* ctx, uint32_t slot, const void* buf, size_t bytes);
int jaad_state_reset(jaad_ctx* ctx, uint32_t slot);

const char* jaad_strerror(int status);
/* last HIP error string recorded by the context (diagnostics) */
const char* jaad_last_error(const jaad_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* JAAD_GPU_H */
