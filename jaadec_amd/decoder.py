"""Host-side mirror of the reference's decoder API for the DSP path (Python over the C-ABI).

Names and behaviour follow the Java classes a caller of the reference uses:

* ``DecoderConfig.decode(asc)``   -- A/DecoderConfig.java:175-254 (AudioSpecificConfig, LC only)
* ``Decoder.create(asc|config)``  -- A/Decoder.java:36-54
* ``Decoder.decodeFrame(frame, buffer)`` -- A/Decoder.java:89-101 (one parsed frame)
* ``Decoder.decodeFrames(batch, buffers)`` -- the batched entry the drop-in adds
* ``SampleBuffer`` -- S/SampleBuffer.java (big-endian by default, setBigEndian swaps in place)

A "parsed frame" is what the reference's ``syntacticElements.decode(in)`` leaves behind, in the
jaad_gpu.h layout: this module does not parse bitstreams.
Errors surface as ``AACException`` (the JNI glue maps every nonzero jaad_status the same way).
"""
from __future__ import annotations

import numpy as np

from . import native as N


class AACException(RuntimeError):
    """A/AACException.java"""


# A/SampleFrequency.java:15-26
SAMPLE_FREQUENCIES = [96000, 88200, 64000, 48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000]


class _Bits:
    def __init__(self, data: bytes):
        self.data, self.pos = data, 0

    def read(self, n: int) -> int:
        v = 0
        for _ in range(n):
            if self.pos >= 8 * len(self.data):
                raise AACException("unexpected end of AudioSpecificConfig")
            v = (v << 1) | ((self.data[self.pos >> 3] >> (7 - (self.pos & 7))) & 1)
            self.pos += 1
        return v


class DecoderConfig:
    """The subset of A/DecoderConfig.java the DSP path needs."""

    def __init__(self, profile: int = 2, sf_index: int = 3, channel_config: int = 2, tns_mode: int = N.TNS_COMPAT):
        self.profile, self.sf_index, self.channel_config, self.tns_mode = profile, sf_index, channel_config, tns_mode

    @classmethod
    def decode(cls, asc: bytes) -> "DecoderConfig":
        """AudioSpecificConfig (A/DecoderConfig.java:175-254): AOT, sampling frequency, channels."""
        b = _Bits(bytes(asc))
        aot = b.read(5)
        if aot == 31:
            aot = 32 + b.read(6)
        sfi = b.read(4)
        if sfi == 15:  # explicit frequency
            freq = b.read(24)
            sfi = min(range(12), key=lambda i: abs(SAMPLE_FREQUENCIES[i] - freq))
        ch = b.read(4)
        if aot != 2:
            raise AACException(f"profile not supported: {aot}")
        frame_length_flag = b.read(1)
        if frame_length_flag:
            raise AACException("config uses 960-sample frames, not yet supported")  # DecoderConfig.java:206-207
        if b.read(1):  # dependsOnCoreCoder
            b.read(14)
        b.read(1)  # extensionFlag
        return cls(aot, sfi, ch)

    def getChannelCount(self) -> int:  # noqa: N802  (Java name)
        return 2  # mono -> stereo while sbrEnabled (A/DecoderConfig.java:108-115)

    def getSampleLength(self) -> int:  # noqa: N802
        return 1024

    def getSampleFrequency(self) -> int:  # noqa: N802
        return SAMPLE_FREQUENCIES[self.sf_index]

    def cfg(self) -> N.StreamCfg:
        return N.make_cfg(self.sf_index, self.channel_config, self.tns_mode)


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

    def _set(self, pcm: bytes, rate: int, sample_length: int = 1024) -> None:
        self.data, self.sample_rate, self.channels, self.bits_per_sample = pcm, rate, 2, 16
        self.length = sample_length / rate
        self.bitrate = sample_length * 16 * 2 / len(pcm)


class Decoder:
    """A/Decoder.java facade: one decoder = one stream slot of a (shared) GPU context."""

    def __init__(self, config: DecoderConfig, context: N.Context | None = None, slot: int = 0):
        if config.profile != 2:
            raise AACException(f"unsupported profile: {config.profile}")
        self.config = config
        self._ctx = context or N.Context(config.cfg(), 1)
        self._own = context is None
        self.slot = slot
        self.frames = 0

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

    def decodeFrames(self, batch: N.Batch, buffers: list[SampleBuffer]) -> None:  # noqa: N802
        """Decode consecutive parsed frames of this stream; buffer i receives frame i's PCM."""
        if len(buffers) != batch.n_frames:
            raise AACException("one SampleBuffer per frame expected")
        b = N.Batch(batch.q, batch.sf, batch.cb, batch.ics, batch.ms_used, batch.tns,
                    np.array([self.slot], np.uint32), np.array([0, batch.n_frames], np.uint32), batch.nch)
        flags = self._flags(buffers[0]) if buffers else 0
        try:
            pcm = self._ctx.decode(b, flags)
        except N.JaadError as e:
            raise AACException(str(e)) from e
        rate = self.config.getSampleFrequency()
        for i, buf in enumerate(buffers):
            want = buf.big_endian
            buf._set(pcm[i].tobytes(), rate)
            buf.big_endian = flags == N.PCM_BIG_ENDIAN
            buf.setBigEndian(want)  # no-op unless this buffer asked for the other byte order
        self.frames += batch.n_frames

    def decodeFrame(self, frame: N.Batch, buffer: SampleBuffer) -> None:  # noqa: N802
        """A/Decoder.java:89-101 for one parsed frame."""
        self.decodeFrames(frame, [buffer])

    def close(self) -> None:
        if self._own:
            self._ctx.close()
