"""Host-side mirror of the reference's decoder API for the DSP path (Python over the C-ABI).

Names and behaviour follow the Java classes a caller of the reference uses:

* ``DecoderConfig.decode(asc)``   -- A/DecoderConfig.java:175-254 (AudioSpecificConfig)
* ``Decoder.create(asc|config)``  -- A/Decoder.java:36-54
* ``Decoder.decodeFrame(frame, buffer)`` -- A/Decoder.java:89-101 (one parsed frame)
* ``Decoder.decodeFrames(batch, buffers)`` -- the batched entry the drop-in adds
* ``SampleBuffer`` -- S/SampleBuffer.java (big-endian by default, setBigEndian swaps in place)

* ``ADTSDemultiplexer``           -- S/adts/ADTSDemultiplexer.java (readNextFrame)

A frame is either a raw_data_block (bytes: parsed by the native host front end,
include/jaad_parse.h, as ``syntacticElements.decode(in)`` parses it) or an already parsed
frame in the jaad_gpu.h layout (a ``native.Batch``, what a JVM-side emitter hands over).
Errors surface as ``AACException`` (the JNI glue maps every nonzero jaad_status the same way).
"""
from __future__ import annotations

import logging
from collections import namedtuple

import numpy as np

from . import native as N

LOGGER = logging.getLogger("jaad.aac.Decoder")


_FRESH = object()  # decodeFrames: the batch created the stream's parser

class AACException(RuntimeError):
    """A/AACException.java"""


class EOSException(AACException):
    """A/EOSException.java: the frame ended inside a syntax element."""


# javax.sound.sampled.AudioFormat fields the reference sets (A/Decoder.java:123-147)
AudioFormat = namedtuple("AudioFormat", "encoding sample_rate bits channels frame_size frame_rate big_endian")


# A/SampleFrequency.java:15-26
SAMPLE_FREQUENCIES = [96000, 88200, 64000, 48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000]


class DecoderConfig:
    """DecoderConfig (A/DecoderConfig.java) for the DSP path: AAC LC core, optionally with
    explicit SBR (AOT 5) or SBR + PS (AOT 29)."""

    def __init__(self, profile: int = 2, sf_index: int = 3, channel_config: int = 2, tns_mode: int = N.TNS_COMPAT,
                 sbr: bool = False, ps: bool = False, ext_sf_index: int | None = None, from_asc: bool = False):
        self.profile, self.sf_index, self.channel_config, self.tns_mode = profile, sf_index, channel_config, tns_mode
        self.sbr, self.ps = bool(sbr), bool(ps)
        self.ext_sf_index = (sf_index - 3) if ext_sf_index is None and sbr else (ext_sf_index or 0)
        # decoded from an AudioSpecificConfig: outputFrequency is set to the core rate there
        # (A/DecoderConfig.java:180), so implicit SBR does not double it (setSBRPresent :124-135)
        self.from_asc = bool(from_asc)

    @classmethod
    def decode(cls, asc: bytes) -> "DecoderConfig":
        """AudioSpecificConfig (A/DecoderConfig.java:175-254) through the native front end
        (include/jaad_parse.h: jaad_asc_parse); errors as the reference words them."""
        asc = bytes(asc)
        aot = asc[0] >> 3 if asc else -1
        try:
            c = N.asc_parse(asc)
        except N.JaadError as e:
            if e.status == N.ERR_EOS or not asc:
                raise AACException("unexpected end of AudioSpecificConfig") from e
            if aot not in (2, 5, 29):
                raise AACException(f"profile not supported: {aot}") from e
            if aot == 2 and len(asc) > 1 and (asc[1] >> 2) & 1:
                raise AACException("config uses 960-sample frames, not yet supported") from e  # :206-207
            raise AACException(f"unsupported configuration ({e})") from e
        return cls(c.profile, c.sf_index, c.channel_config, N.TNS_COMPAT, bool(c.sbr), bool(c.ps), c.ext_sf_index,
                   from_asc=True)

    def getChannelCount(self) -> int:  # noqa: N802  (Java name)
        # mono -> stereo while sbrEnabled (A/DecoderConfig.java:108-115); otherwise the
        # configuration's speakers (ChannelConfiguration.forInt: 7 -> 7.1, 8 channels)
        if self.channel_config in N.MC_ELEMENTS:
            return 8 if self.channel_config == 7 else self.channel_config
        if self.channel_config == 0:
            return 0  # ChannelConfiguration.NONE until a PCE arrives
        return 2

    def getSampleLength(self) -> int:  # noqa: N802
        # A/DecoderConfig.java:83-86: doubled only by upsampling SBR (not downsampled SBR)
        return 2048 if self.sbr and self.ext_sf_index != self.sf_index else 1024

    def getSampleFrequency(self) -> int:  # noqa: N802
        return SAMPLE_FREQUENCIES[self.sf_index]

    def getOutputFrequency(self) -> int:  # noqa: N802
        return SAMPLE_FREQUENCIES[self.ext_sf_index] if self.sbr else self.getSampleFrequency()

    def cfg(self) -> N.StreamCfg:
        return N.make_cfg(self.sf_index, self.channel_config, self.tns_mode, sbr=self.sbr, ps=self.ps,
                          down=self.sbr and self.ext_sf_index == self.sf_index)


class SampleBuffer:
    """S/SampleBuffer.java: int16 PCM, interleaved, big-endian unless setBigEndian(False).

    The fields set per frame follow ``accept`` (S/SampleBuffer.java:167-209): sampleRate,
    channels = 2, bitsPerSample = 16, length = sampleLength / sampleRate and the reference's
    bitrate expression ``sampleLength*bitsPerSample*channels/bytes`` (:186, kept as is).
    """

    def __init__(self, big_endian: bool = True):
        self.big_endian = big_endian
        self.data = b""
        self.sample_rate = self.channels = self.bits_per_sample = 0
        self.length = self.bitrate = 0.0

    def isBigEndian(self) -> bool:  # noqa: N802
        return self.big_endian

    def setBigEndian(self, big_endian: bool) -> None:  # noqa: N802
        """Swaps the bytes of the data already held, as S/SampleBuffer.java:128-139 does."""
        if big_endian != self.big_endian:
            a = np.frombuffer(self.data, np.uint16).byteswap()
            self.data = a.tobytes()
            self.big_endian = big_endian

    def getBB(self) -> memoryview:  # noqa: N802
        """S/SampleBuffer.java:48-50 (read-only view of this frame's PCM bytes)."""
        return memoryview(self.data)

    def getData(self, primitive: bytearray | None = None) -> bytes:  # noqa: N802
        """S/SampleBuffer.java:59-68 (deprecated there): copy into `primitive` when it is big enough."""
        if primitive is not None and len(primitive) >= len(self.data):
            primitive[:len(self.data)] = self.data
            return primitive
        return self.data

    def getSampleRate(self) -> int:  # noqa: N802
        return self.sample_rate

    def getChannels(self) -> int:  # noqa: N802
        return self.channels

    def getBitsPerSample(self) -> int:  # noqa: N802
        return self.bits_per_sample

    def getLength(self) -> float:  # noqa: N802
        return self.length

    def getBitrate(self) -> float:  # noqa: N802
        return self.bitrate

    def _set(self, pcm: bytes, rate: int, sample_length: int = 1024, channels: int = 2) -> None:
        self.data, self.sample_rate, self.channels, self.bits_per_sample = pcm, rate, channels, 16
        self.length = sample_length / rate
        self.bitrate = sample_length * 16 * channels / len(pcm)


class Decoder:
    """A/Decoder.java facade: one decoder = one stream slot of a (shared) GPU context."""

    def __init__(self, config: DecoderConfig, context: N.Context | None = None, slot: int = 0):
        if config.profile != 2:
            raise AACException(f"unsupported profile: {config.profile}")
        self.config = config
        # channel_configuration 0 (an ADTS header's): the layout arrives with the first frame's
        # PCE (SyntacticElements.decode -> setAudioDecoderInfo, A/syntax/SyntacticElements.java:
        # 153-156), the context is opened then (_pce_layout)
        self._ctx = context or (N.Context(config.cfg(), 1) if config.channel_config else None)
        self._own = context is None
        self.slot = slot
        self.frames = 0
        self._parser = None  # host bitstream front end, created on the first raw frame

    @classmethod
    def create(cls, data) -> "Decoder":
        cfg = data if isinstance(data, DecoderConfig) else DecoderConfig.decode(data)
        try:
            return cls(cfg)
        except N.JaadError as e:
            raise AACException(str(e)) from e

    def getConfig(self) -> DecoderConfig:  # noqa: N802
        return self.config

    def _flags(self, buf: SampleBuffer) -> int:
        return N.PCM_BIG_ENDIAN if buf.big_endian else N.PCM_LITTLE_ENDIAN

    def _implicit_sbr(self, first: bytes) -> None:
        """A core configuration whose first frame carries SBR data is upgraded as the reference
        upgrades its DecoderConfig (A/syntax/ChannelElement.java:63-74, SBR.java:100): stereo
        output, PS applied if present; the output rate doubled for an ADTS-created decoder, kept
        (downsampled SBR) for one created from an AudioSpecificConfig (native.implicit_sbr_cfg)."""
        c = self.config
        try:
            if c.sbr or not N.probe_sbr(c.cfg(), first):
                return
            up = N.implicit_sbr_cfg(c.cfg(), from_asc=c.from_asc)
        except N.JaadError as e:
            raise AACException(str(e)) from e
        if not self._own:
            raise AACException("implicit SBR in a stream decoded on a shared core-only context")
        self._ctx.close()
        self.config = DecoderConfig(c.profile, c.sf_index, c.channel_config, c.tns_mode, True, bool(up.ps),
                                    up.ext_sf_index, from_asc=c.from_asc)
        self._ctx = N.Context(self.config.cfg(), 1)

    def _pce_layout(self, first: bytes) -> None:
        """Channel configuration 0: the configuration of the first frame's program_config_element
        (its profile, rate and channel count, DecoderConfig.setAudioDecoderInfo :60-65)."""
        if not self._own:
            raise AACException("a PCE-defined layout needs its own context")
        try:
            c = N.raw_pce_cfg(first)
            self.config = DecoderConfig(c.profile, c.sf_index, c.channel_config, self.config.tns_mode,
                                        from_asc=self.config.from_asc)
            self._ctx = N.Context(self.config.cfg(), 1)
        except N.JaadError as e:
            raise AACException(str(e)) from e

    def _parse(self, frames: list, drop_eos: bool = False) -> N.Batch:
        if self._parser is None:
            if self._ctx is None:
                if not frames:
                    raise AACException("channel configuration 0: the first frame must carry the PCE")
                self._pce_layout(bytes(frames[0]))
            if frames and self.frames == 0:
                self._implicit_sbr(bytes(frames[0]))
            self._parser = N.Parser(self.config.cfg())
        try:
            return self._parser.parse(frames, self.slot, drop_eos=drop_eos)
        except N.JaadError as e:
            raise (EOSException if e.status == N.ERR_EOS else AACException)(str(e)) from e

    def decodeFrames(self, batch, buffers: list[SampleBuffer], _drop_eos: bool = True) -> None:  # noqa: N802
        """Decode consecutive frames of this stream -- a list of raw_data_blocks or a parsed
        ``native.Batch`` -- buffer i receives frame i's PCM.

        Per frame as Decoder.decodeFrame (A/Decoder.java:89-101): a frame whose bitstream ends
        early is logged and dropped -- its buffer is left as it is, the stream continues from the
        previous frame's state -- and still counts as a frame; the rest of the batch decodes
        (jaad_batch.frame_status).  Any other error rejects the whole batch (AACException) and
        leaves the decoder as it was."""
        snap = None
        if isinstance(batch, (list, tuple)):
            # the parser commits frame by frame: roll it back if this batch is not decoded, so
            # it never runs ahead of the DSP state (a failed parse restores nothing else)
            snap = self._parser.snapshot() if self._parser is not None else _FRESH
            try:
                batch = self._parse(list(batch), drop_eos=_drop_eos)
            except AACException:
                self._rollback(snap)
                raise
        if self._ctx is None:  # channel configuration 0 and no raw frame (with its PCE) seen yet
            raise AACException("channel configuration 0: decode the raw frames (the first carries the PCE)")
        if len(buffers) != batch.n_frames:
            self._rollback(snap)
            raise AACException("one SampleBuffer per frame expected")
        b = N.Batch(batch.q, batch.sf, batch.cb, batch.ics, batch.ms_used, batch.tns,
                    np.array([self.slot], np.uint32), np.array([0, batch.n_frames], np.uint32), batch.nch,
                    batch.sbr, batch.cce_q, batch.cce_sf, batch.cce_cb, batch.cce_ics, batch.cce_terms,
                    batch.frame_status)
        flags = self._flags(buffers[0]) if buffers else 0
        try:
            pcm = self._ctx.decode(b, flags)
        except N.JaadError as e:
            self._rollback(snap)
            raise AACException(str(e)) from e
        if snap is not None and snap is not _FRESH:
            snap.close()
        rate = self.config.getOutputFrequency()
        st = b.frame_status
        for i, buf in enumerate(buffers):
            if st is not None and st[i] != N.FRAME_DECODE:
                LOGGER.warning("unexpected end of frame: frame %d dropped", self.frames + i)
                continue  # the reference swallows the EOSException: this buffer keeps what it had
            want = buf.big_endian
            buf._set(pcm[i].tobytes(), rate, self.config.getSampleLength(), N.out_channels(self.config.cfg()))
            buf.big_endian = flags == N.PCM_BIG_ENDIAN
            buf.setBigEndian(want)  # no-op unless this buffer asked for the other byte order
        self.frames += batch.n_frames

    def _rollback(self, snap) -> None:
        if snap is None:  # a pre-parsed batch: no parser state was touched
            return
        if snap is _FRESH:  # the parser was created by this batch: start over at the next one
            if self._parser is not None:
                self._parser.close()
                self._parser = None
            return
        self._parser.restore(snap)
        snap.close()

    def decode0(self, frame, buffer: SampleBuffer) -> None:
        """A/Decoder.java:103-121: one frame; an EOSException propagates."""
        self.decodeFrames([frame] if isinstance(frame, (bytes, bytearray, memoryview)) else frame, [buffer],
                          _drop_eos=False)

    def decodeFrame(self, frame, buffer: SampleBuffer) -> None:  # noqa: N802
        """A/Decoder.java:89-101 for one frame (raw_data_block bytes or a parsed Batch): a frame that
        ends early is logged and dropped -- the buffer keeps the previous frame's PCM -- and still
        counts as a frame.  (The parser is atomic: unlike the JVM, nothing of its state moved.)"""
        try:
            self.decode0(frame, buffer)
        except EOSException as e:
            LOGGER.warning("unexpected end of frame: %s", e)
            self.frames += 1

    def getAudioFormat(self) -> AudioFormat:  # noqa: N802
        """A/Decoder.java:123-134: 16-bit signed little-endian; a mono core below 24 kHz is assumed
        to carry SBR/PS (rate doubled), whatever the configuration says."""
        freq = self.config.getSampleFrequency()
        if self.config.channel_config == 1 and freq < 24000:
            freq *= 2
        ch = self.config.getChannelCount()
        return AudioFormat("PCM_SIGNED", freq, 16, ch, 2 * ch, freq, False)

    def getAudioFormatFloat(self) -> AudioFormat:  # noqa: N802
        """A/Decoder.java:136-147"""
        freq = self.config.getSampleFrequency()
        if self.config.channel_config == 1 and freq < 24000:
            freq *= 2
        ch = self.config.getChannelCount()
        return AudioFormat("PCM_FLOAT", freq, 32, ch, 4 * ch, freq, False)

    def close(self) -> None:
        if self._own and self._ctx is not None:
            self._ctx.close()
        if self._parser is not None:
            self._parser.close()


class ADTSDemultiplexer:
    """S/adts/ADTSDemultiplexer.java over a byte string: readNextFrame() returns the next
    raw_data_block (EOFError at the end), the stream parameters come from the ADTS header."""

    def __init__(self, data: bytes):
        self._frames = N.adts_frames(bytes(data))
        try:
            self._first = next(self._frames)
        except StopIteration:
            raise OSError("no ADTS header found") from None  # ADTSDemultiplexer.java:21-22
        self._next = self._first

    def readNextFrame(self) -> bytes:  # noqa: N802
        if self._next is None:
            try:
                self._next = next(self._frames)
            except StopIteration:
                raise EOFError() from None
        h, payload = self._next
        self._next = None
        return payload

    def getSampleFrequency(self) -> int:  # noqa: N802
        return SAMPLE_FREQUENCIES[self._first[0].sf_index]

    def getChannelCount(self) -> int:  # noqa: N802
        return self._first[0].channel_config

    def getDecoderInfo(self) -> DecoderConfig:  # noqa: N802
        c = N.adts_cfg(self._first[0])
        return DecoderConfig(c.profile, c.sf_index, c.channel_config)
