"""MP4 transport over the native feeder (include/jaad_mp4.h): the reference's MP4 API as far as
a decoder uses it -- MP4Container(data).getMovie().getTracks(AudioCodec.AAC), the track's
DecoderSpecificInfo and Track.readNextFrame (M/ = mp4/src/main/java/net/sourceforge/jaad/mp4/:
MP4Container.java, api/Movie.java, api/Track.java, api/AudioTrack.java, api/Frame.java), as
S/Main.java:49-80 drives them.  The box walk and the frame table are native; this module holds
the file image and the read cursor.
"""
from __future__ import annotations

import ctypes as C
import enum

from . import native as N


class _TrackInfo(C.Structure):
    _fields_ = [("track_id", C.c_uint32), ("sample_entry", C.c_uint32), ("channel_count", C.c_uint32),
                ("sample_size", C.c_uint32), ("sample_rate", C.c_uint32), ("timescale", C.c_uint32),
                ("n_frames", C.c_uint32), ("dsi_bytes", C.c_uint32)]


MP4_EXPORTS = ["jaad_mp4_open", "jaad_mp4_close", "jaad_mp4_track_count", "jaad_mp4_track_info",
               "jaad_mp4_decoder_specific_info", "jaad_mp4_frame"]
_bound = False


def _lib():
    global _bound
    L = N.lib()
    if not _bound:
        L.jaad_mp4_open.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p)]
        L.jaad_mp4_close.argtypes = [C.c_void_p]
        L.jaad_mp4_close.restype = None
        L.jaad_mp4_track_count.argtypes = [C.c_void_p]
        L.jaad_mp4_track_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(_TrackInfo)]
        L.jaad_mp4_decoder_specific_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p),
                                                     C.POINTER(C.c_size_t)]
        L.jaad_mp4_frame.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_double)]
        _bound = True
    return L


class AudioCodec(enum.Enum):
    """AudioTrack.AudioCodec.forType (M/api/AudioTrack.java:24-44) for the sample entry four-cc."""
    AAC = b"mp4a"
    AC3 = b"ac-3"
    AMR = b"samr"
    AMR_WIDE_BAND = b"sawb"
    EVRC = b"sevc"
    EXTENDED_AC3 = b"ec-3"
    QCELP = b"sqcp"
    SMV = b"ssmv"
    UNKNOWN_AUDIO_CODEC = b""

    @classmethod
    def for_type(cls, fourcc: int) -> "AudioCodec":
        b = fourcc.to_bytes(4, "big")
        for c in cls:
            if c.value == b:
                return c
        return cls.UNKNOWN_AUDIO_CODEC


class DecoderSpecificInfo:
    def __init__(self, data: bytes):
        self._data = data

    def getData(self) -> bytes:  # noqa: N802
        return self._data


class Frame:
    """M/api/Frame.java: offset, size, time stamp and (after reading) the sample bytes."""

    def __init__(self, offset: int, size: int, time: float):
        self._offset, self._size, self._time, self._data = offset, size, time, None

    def getOffset(self) -> int:  # noqa: N802
        return self._offset

    def getSize(self) -> int:  # noqa: N802
        return self._size

    def getTime(self) -> float:  # noqa: N802
        return self._time

    def getData(self) -> bytes | None:  # noqa: N802
        return self._data


class AudioTrack:
    def __init__(self, container: "MP4Container", index: int):
        self._c, self._i = container, index
        info = _TrackInfo()
        rc = _lib().jaad_mp4_track_info(container._h, index, C.byref(info))
        if rc:
            raise N.JaadError(rc, "jaad_mp4_track_info")
        self._info = info
        p, n = C.c_void_p(), C.c_size_t()
        _lib().jaad_mp4_decoder_specific_info(container._h, index, C.byref(p), C.byref(n))
        self._dsi = C.string_at(p.value, n.value) if n.value else None
        self._frames = []
        off, size, t = C.c_uint64(), C.c_uint32(), C.c_double()
        for i in range(info.n_frames):
            _lib().jaad_mp4_frame(container._h, index, i, C.byref(off), C.byref(size), C.byref(t))
            self._frames.append(Frame(off.value, size.value, t.value))
        self._current = 0

    def getCodec(self) -> AudioCodec:  # noqa: N802
        return AudioCodec.for_type(self._info.sample_entry)

    def getChannelCount(self) -> int:  # noqa: N802
        return self._info.channel_count

    def getSampleRate(self) -> int:  # noqa: N802
        return self._info.sample_rate

    def getSampleSize(self) -> int:  # noqa: N802
        return self._info.sample_size

    def getDecoderSpecificInfo(self) -> DecoderSpecificInfo | None:  # noqa: N802
        return DecoderSpecificInfo(self._dsi) if self._dsi is not None else None

    def getFrameCount(self) -> int:  # noqa: N802
        return len(self._frames)

    def hasMoreFrames(self) -> bool:  # noqa: N802
        return self._current < len(self._frames)

    def readNextFrame(self) -> Frame:  # noqa: N802
        """Track.readNextFrame (M/api/Track.java:320-349): EOFError past the last frame or when the
        sample lies beyond the end of the file image."""
        if not self.hasMoreFrames():
            raise EOFError()
        f = self._frames[self._current]
        end = f.getOffset() + f.getSize()
        if end > len(self._c._data):
            raise EOFError(f"readNextFrame failed: tried to read {f.getSize()} bytes at {f.getOffset()}")
        f._data = self._c._data[f.getOffset():end]
        self._current += 1
        return f

    def seek(self, timestamp: float) -> float:
        """Track.seek as the reference has it (M/api/Track.java:359-370): the loop advances its index
        twice per step, so it tests frames 0, 2, 4, ... and leaves the cursor one past the frame it
        found; -1 only for an empty track."""
        frame = None
        i = 0
        while i < len(self._frames):
            frame = self._frames[i]
            i += 1
            if frame.getTime() > timestamp:
                self._current = i
                break
            i += 1
        return -1 if frame is None else frame.getTime()


class Movie:
    def __init__(self, container: "MP4Container"):
        self._tracks = [AudioTrack(container, i) for i in range(_lib().jaad_mp4_track_count(container._h))]

    def getTracks(self, codec: AudioCodec | None = None) -> list:  # noqa: N802
        return [t for t in self._tracks if codec is None or t.getCodec() == codec]


class MP4Container:
    """MP4Container over a file image (bytes / mmap); sound tracks only."""

    def __init__(self, data):
        self._data = data
        h = C.c_void_p()
        buf = bytes(data[:]) if not isinstance(data, bytes) else data
        self._buf = buf
        rc = _lib().jaad_mp4_open(buf, len(buf), C.byref(h))
        if rc:
            raise N.JaadError(rc, "jaad_mp4_open")
        self._h = h
        self._movie = Movie(self)

    def getMovie(self) -> Movie:  # noqa: N802
        return self._movie

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            _lib().jaad_mp4_close(h)

    def __del__(self):
        try:
            self.close()
        except TypeError:  # interpreter shutdown: the module's globals are already gone
            pass
