/*
 * jaad_parse.h -- host-side bitstream front end feeding the jaad_gpu.h batch layout.
 *
 * The reference parses on the JVM: Decoder.decode0 (A/Decoder.java:103-121)
 * calls syntacticElements.decode(in) (A/syntax/SyntacticElements.java:57-132) and then the DSP.
 * In the drop-in the DSP is jaad_decode_batch*; this library is the parse half for hosts that
 * have no JVM parser: it turns raw_data_blocks (ADTS payloads, MP4 samples) into exactly the
 * records the JVM-side emitter would write -- quantised spectra, scalefactor/codebook rows,
 * jaad_ics_info, M/S masks, TNS records -- with the reference's parse semantics:
 *
 *   element loop / FIL / DSE / PCE   A/syntax/SyntacticElements.java:57-203, DSE.java, PCE.java
 *   CPE / SCE                        A/syntax/CPE.java:85-123, SCE.java
 *   ics_info                         A/syntax/ICSInfo.java:86-119
 *   section data, scalefactors       A/syntax/ICStream.java:113-146, 172-220
 *   pulse data (parsed, not applied) A/syntax/ICStream.java:148-170
 *   TNS data                         A/tools/TNS.java:35-61
 *   spectral Huffman + escapes       A/syntax/ICStream.java:222-275, A/huffman/Huffman.java:15-84
 *   static PNS LCG state             A/syntax/ICStream.java:26,247 (one LCG per parser)
 *   AudioSpecificConfig              A/DecoderConfig.java:175-291
 *   ADTS header / sync search        S/adts/ADTSFrame.java, S/adts/ADTSDemultiplexer.java:25-58
 *   SBR / PS extension payloads      A/sbr/SBR.java:161-284, SBR1.java, SBR2.java, Channel.java:85-583,
 *                                    A/ps/PSImpl.java:103-199, EnvData.java, Envelope.java
 *
 * Plain C types only; every entry point returns 0 or a negative jaad_status.
 */
#ifndef JAAD_PARSE_H
#define JAAD_PARSE_H

#include <stddef.h>
#include <stdint.h>

#include "jaad_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* AudioSpecificConfig -> stream configuration (DecoderConfig.decode).  AOT 2 (LC), 5 (SBR) and
 * 29 (PS) with an LC core; frameLengthFlag = 1 (960-sample frames) is rejected as the
 * reference rejects it (JAAD_ERR_UNSUPPORTED).  A mono AOT 5 stream gets ps = 1: the reference
 * has PS enabled by default (A/DecoderConfig.java:36, A/sbr/SBR1.java:62-73), so PS data it
 * meets is applied, and frames without it duplicate the SBR channel as ps = 0 would.  An AOT 2
 * config with the backward-compatible sync extension (0x2B7, sbrPresent, extension rate;
 * readSyncExtension A/DecoderConfig.java:260-291) is explicit SBR as well.  Without it the
 * output rate is the core rate (A/DecoderConfig.java:180): SBR found later in the frames
 * (implicit signalling) runs downsampled for such a decoder, unlike one created from an ADTS
 * header (AudioDecoderInfo), whose output rate is doubled (DecoderConfig.setSBRPresent :124-135).
 * channelConfiguration 0 reads the program_config_element that follows (PCE.read/decode,
 * A/syntax/PCE.java:47-52,133-188); its profile and sample rate replace the ASC's and its channel
 * count selects the configuration (setAudioDecoderInfo, PCE.getChannelConfiguration :221-223).
 * Accepted when the PCE's elements (front, side, back, LFE) carry the channel counts of that
 * configuration's element list, which is the list the frames are parsed against;
 * JAAD_ERR_UNSUPPORTED otherwise (e.g. two SCEs as "dual mono", a 7-channel count). */
int jaad_asc_parse(const uint8_t* asc, size_t bytes, jaad_stream_cfg* cfg);

/* ADTS fixed + variable header (S/adts/ADTSFrame.java:48-111) */
typedef struct jaad_adts_header {
    uint8_t profile;            /* audio object type = profile_ObjectType + 1 (2 = LC)          */
    uint8_t sf_index;
    uint8_t channel_config;
    uint8_t protection_absent;
    uint8_t n_raw_blocks;       /* number_of_raw_data_blocks_in_frame + 1                         */
    uint8_t reserved[3];
    uint32_t frame_length;      /* aac_frame_length: header + payload bytes                      */
    uint32_t header_bytes;      /* 7, or 9 with the CRC word                                      */
} jaad_adts_header;

/* Find the next ADTS sync word (0xFFF, layer 0) at or after buf[0] within the reference's
 * search window (ADTSDemultiplexer.MAXIMUM_FRAME_SIZE = 6144 bytes) and decode its header.
 * *offset = byte offset of the header.  JAAD_ERR_EOS when no complete header is found. */
int jaad_adts_find(const uint8_t* buf, size_t bytes, size_t* offset, jaad_adts_header* h);
/* The stream configuration a raw_data_block's leading program_config_element declares (an ADTS
 * stream with channel_configuration 0: the reference decodes the PCE as an element and applies it
 * with DecoderConfig.setAudioDecoderInfo, A/syntax/SyntacticElements.java:153-156); the same layout
 * rule as jaad_asc_parse.  JAAD_ERR_BITSTREAM when the frame does not start with a PCE. */
int jaad_raw_pce_cfg(const uint8_t* raw, size_t bytes, jaad_stream_cfg* cfg);

/* stream configuration implied by an ADTS header (AAC LC only); channel_configuration 0 gives
 * channel_config 0, the layout then comes from the first frame (jaad_raw_pce_cfg) */
int jaad_adts_cfg(const jaad_adts_header* h, jaad_stream_cfg* cfg);

typedef struct jaad_parser jaad_parser;

int jaad_parser_create(const jaad_stream_cfg* cfg, jaad_parser** out);
void jaad_parser_destroy(jaad_parser* p);
/* Snapshot / rollback of a parser's whole state (window shapes, PNS LCG, SBR/PS history): a
 * host that parses a batch ahead of its decode copies the state first and restores it when the
 * decode is rejected, so the parser never runs ahead of the DSP state.  `dst` of copy must have
 * been created for the same configuration. */
int jaad_parser_clone(const jaad_parser* src, jaad_parser** out);
int jaad_parser_copy(jaad_parser* dst, const jaad_parser* src);
/* the static ICStream.randomState (PNS) the next ch-frame starts from; 0x1F2E3D4C initially */
uint32_t jaad_parser_pns_state(const jaad_parser* p);
void jaad_parser_set_pns_state(jaad_parser* p, uint32_t state);

/* Where one frame's records go: this frame's slot in each jaad_batch array (nch = 1 for an
 * SCE config, 2 for a CPE config).  tns may be NULL (TNS data is then parsed and dropped:
 * the reference does not apply it either); sbr is required when cfg.sbr is set. */
typedef struct jaad_frame_out {
    int16_t* q;            /* [nch][1024] */
    uint8_t* sf;           /* [nch][128]  */
    uint8_t* cb;           /* [nch][128]  */
    jaad_ics_info* ics;    /* [nch]       */
    uint64_t* ms_used;     /* [2], CPE only */
    jaad_tns* tns;         /* [nch] or NULL */
    jaad_sbr_frame* sbr;   /* when cfg.sbr: [1], or one per channel element (in bitstream order,
                              LFE included: always JAAD_SBR_UPSAMPLE) for configurations 3..7 */
    /* coupling channel elements (CCE.decode, A/syntax/CCE.java:112-175): NULL cce_q makes a frame
       with a CCE JAAD_ERR_UNSUPPORTED.  Records go to cce_q/sf/cb/ics (up to cce_cap), the terms
       the frame's CCEs apply (jaad_gpu.h jaad_cce_term; frame 0, cce relative to this frame's
       records, in the reference's order) to cce_terms (up to term_cap). */
    int16_t* cce_q;        /* [cce_cap][1024] */
    uint8_t* cce_sf;       /* [cce_cap][128]  */
    uint8_t* cce_cb;       /* [cce_cap][128]  */
    jaad_ics_info* cce_ics; /* [cce_cap]      */
    jaad_cce_term* cce_terms; /* [term_cap]   */
    uint32_t cce_cap, term_cap;
    uint32_t n_cce, n_cce_terms; /* out */
} jaad_frame_out;

/* Parse one raw_data_block (SyntacticElements.decode) into *out.  JAAD_ERR_EOS (the bitstream
 * ended early: the reference's EOSException, which Decoder.decodeFrame swallows, dropping the
 * frame, A/Decoder.java:96-100) leaves the state where the reference's reads left it: the window
 * shape of every ICSInfo whose shape bit was read, the PNS LCG advanced over the noise bands
 * decodeSpectralData reached, the SBR/PS state of payloads parsed whole -- and out->sbr keeps
 * those payloads' records (header included: the reference swapped it in before the exception,
 * A/sbr/SBR.java:162-184; jaad_decode_batch applies it for a frame marked JAAD_FRAME_EOS).  An
 * SBR payload that ends inside its fill element's bytes is JAAD_ERR_UNSUPPORTED: the reference
 * would have applied part of it.  Any error other than JAAD_ERR_EOS changes nothing of the
 * parser's state. */
int jaad_parse_frame(jaad_parser* p, const uint8_t* data, size_t bytes, jaad_frame_out* out);

/* Implicit SBR signalling (ADTS, LC-only AudioSpecificConfig): the reference opens SBR when it
 * meets an SBR extension payload (A/syntax/ChannelElement.java:63-74) and doubles the output
 * rate when it can (DecoderConfig.setSBRPresent, A/DecoderConfig.java:124-135).  This tells a
 * host whether a raw_data_block of a core configuration carries one (*found bit 0), so it can
 * re-open the stream with sbr = 1, ext_sf_index = sf_index - 3 (and ps = 1 for a mono core);
 * sf_index < 3 has no doubled rate (the reference's downsampled SBR, not supported).
 * jaad_parse_frame itself refuses an SBR payload in a core configuration (UNSUPPORTED). */
int jaad_probe_sbr(const jaad_stream_cfg* cfg, const uint8_t* data, size_t bytes, uint32_t* found);

#ifdef __cplusplus
}
#endif
#endif /* JAAD_PARSE_H */
