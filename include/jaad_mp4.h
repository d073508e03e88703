/*
 * jaad_mp4.h -- MP4 (ISO base media file) transport feeder for the host front end.
 *
 * Replaces the part of the reference's MP4 API a decoder needs (M/ = mp4/src/main/java/net/
 * sourceforge/jaad/mp4/): MP4Container -> Movie.getTracks (M/api/Movie.java:15-62), the sound
 * track's sample entry and its esds DecoderSpecificInfo (M/api/AudioTrack.java:46-77,
 * M/api/Track.java:158-173), and the frame table Track.parseSampleTable builds from stsz, stco /
 * co64, stsc and stts, sorted by time stamp (M/api/Track.java:90-155).  Track.readNextFrame
 * (:320-349) then is "bytes [offset, offset + size) of the file"; the DecoderSpecificInfo is the
 * AudioSpecificConfig for jaad_asc_parse (include/jaad_parse.h), as in S/Main.java:49-80.
 *
 * The file image is read in place (mmap or a buffer); the handle keeps pointers into it, so it
 * must outlive the handle.  Plain C types only; entry points return 0 or a negative jaad_status.
 */
#ifndef JAAD_MP4_H
#define JAAD_MP4_H

#include <stddef.h>
#include <stdint.h>

#include "jaad_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct jaad_mp4 jaad_mp4;

typedef struct jaad_mp4_track {
    uint32_t track_id;       /* tkhd track_ID                                                      */
    uint32_t sample_entry;   /* four-cc of the first sample entry ('mp4a' = AudioCodec.AAC)        */
    uint32_t channel_count;  /* AudioSampleEntry.getChannelCount                                   */
    uint32_t sample_size;    /* AudioSampleEntry.getSampleSize (bits)                              */
    uint32_t sample_rate;    /* AudioSampleEntry.getSampleRate (integer part of the 16.16 value)   */
    uint32_t timescale;      /* mdhd timescale                                                     */
    uint32_t n_frames;       /* samples in the track                                               */
    uint32_t dsi_bytes;      /* DecoderSpecificInfo length (0 without an esds)                     */
} jaad_mp4_track;

/* Parse the movie box of a file image (the top-level boxes are walked to find 'moov').  Sound
 * tracks (handler 'soun') are kept in file order; other tracks are skipped as Movie.createTrack
 * skips non-audio/video ones.  JAAD_ERR_BITSTREAM for a malformed box tree, JAAD_ERR_EOS when the
 * image ends inside a box the parse needs. */
int jaad_mp4_open(const uint8_t* file, size_t bytes, jaad_mp4** out);
void jaad_mp4_close(jaad_mp4* m);

int jaad_mp4_track_count(const jaad_mp4* m);
int jaad_mp4_track_info(const jaad_mp4* m, int track, jaad_mp4_track* info);
/* esds DecoderSpecificInfo bytes (the AudioSpecificConfig); *bytes = 0 when absent */
int jaad_mp4_decoder_specific_info(const jaad_mp4* m, int track, const uint8_t** dsi, size_t* bytes);
/* frame i of the track in time-stamp order: file offset, size, time stamp in seconds */
int jaad_mp4_frame(const jaad_mp4* m, int track, uint32_t i, uint64_t* offset, uint32_t* size, double* time);

#ifdef __cplusplus
}
#endif
#endif /* JAAD_MP4_H */
