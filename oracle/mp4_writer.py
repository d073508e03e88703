"""TEST INFRASTRUCTURE ONLY: a minimal MP4 (ISO base media) file WRITER for the transport
feeder's tests (include/jaad_mp4.h).  It lays out what the reference's MP4 reader consumes
(M/api/Movie.java, Track.java, AudioTrack.java; M/boxes/impl/*; M/od/*): ftyp, moov with one
sound track (tkhd, mdia: mdhd, hdlr 'soun', minf: smhd, dinf/dref/url, stbl: stsd/mp4a/esds,
stts, stsc, stsz, stco or co64) and optionally a video track to be skipped, then mdat.
"""
from __future__ import annotations

import struct


def box(t: bytes, body: bytes) -> bytes:
    return struct.pack(">I", 8 + len(body)) + t + body


def full(t: bytes, body: bytes, version: int = 0, flags: int = 0) -> bytes:
    return box(t, struct.pack(">I", version << 24 | flags) + body)


def desc(tag: int, body: bytes, long_size: bool = False) -> bytes:
    n = len(body)
    if long_size:  # 4-byte size field, as many encoders write it
        sz = bytes([0x80 | (n >> 21) & 0x7F, 0x80 | (n >> 14) & 0x7F, 0x80 | (n >> 7) & 0x7F, n & 0x7F])
    else:
        assert n < 128
        sz = bytes([n])
    return bytes([tag]) + sz + body


def esds(asc: bytes, long_size: bool = False, url: bytes | None = None) -> bytes:
    dsi = desc(5, asc, long_size)
    dcd = desc(4, bytes([0x40, 0x15]) + b"\x00\x18\x00" + struct.pack(">II", 128000, 128000) + dsi, long_size)
    slc = desc(6, b"\x02", long_size)
    flags = 0x40 if url is not None else 0
    es_body = struct.pack(">HB", 1, flags) + (bytes([len(url)]) + url if url is not None else b"") + dcd + slc
    return full(b"esds", desc(3, es_body, long_size))


def sample_table(sizes, chunk_layout, chunk_offsets, deltas, co64=False, stsz_fixed=None):
    """chunk_layout: stsc entries (first_chunk, samples_per_chunk); deltas: stts (count, delta)."""
    stts = full(b"stts", struct.pack(">I", len(deltas)) + b"".join(struct.pack(">II", c, d) for c, d in deltas))
    stsc = full(b"stsc", struct.pack(">I", len(chunk_layout)) +
                b"".join(struct.pack(">III", f, n, 1) for f, n in chunk_layout))
    if stsz_fixed is not None:
        stsz = full(b"stsz", struct.pack(">II", stsz_fixed, len(sizes)))
    else:
        stsz = full(b"stsz", struct.pack(">II", 0, len(sizes)) + b"".join(struct.pack(">I", s) for s in sizes))
    if co64:
        stco = full(b"co64", struct.pack(">I", len(chunk_offsets)) + b"".join(struct.pack(">Q", o) for o in chunk_offsets))
    else:
        stco = full(b"stco", struct.pack(">I", len(chunk_offsets)) + b"".join(struct.pack(">I", o) for o in chunk_offsets))
    return stts, stsc, stsz, stco


def write_mp4(frames: list[bytes], asc: bytes, sample_rate: int, channels: int, samples_per_frame: int = 1024,
              chunk_sizes=(3, 5, 1), co64: bool = False, video_track: bool = False, long_desc: bool = False,
              mdat_first: bool = False, esds_url: bytes | None = None) -> bytes:
    """An MP4 file holding `frames` as one AAC track.  Chunks take chunk_sizes[i % len] samples."""
    # chunk plan
    per_chunk, i = [], 0
    while i < len(frames):
        n = min(chunk_sizes[len(per_chunk) % len(chunk_sizes)], len(frames) - i)
        per_chunk.append(n)
        i += n
    layout = []
    for c, n in enumerate(per_chunk):
        if not layout or layout[-1][1] != n:
            layout.append((c + 1, n))
    mdat_body = b"".join(frames)
    # two passes: build moov with placeholder offsets, then with the real ones
    def build(mdat_start: int) -> bytes:
        offs, pos, k = [], mdat_start, 0
        for n in per_chunk:
            offs.append(pos)
            pos += sum(len(f) for f in frames[k:k + n])
            k += n
        deltas = [(len(frames) - 1, samples_per_frame), (1, samples_per_frame)] if len(frames) > 1 else \
            [(len(frames), samples_per_frame)]
        stts, stsc, stsz, stco = sample_table([len(f) for f in frames], layout, offs, deltas, co64)
        mp4a_body = (b"\x00" * 6 + struct.pack(">H", 1) + b"\x00" * 8 + struct.pack(">HH", channels, 16) +
                     b"\x00" * 4 + struct.pack(">HH", sample_rate & 0xFFFF, 0) + esds(asc, long_desc, esds_url))
        stsd = full(b"stsd", struct.pack(">I", 1) + box(b"mp4a", mp4a_body))
        stbl = box(b"stbl", stsd + stts + stsc + stsz + stco)
        dinf = box(b"dinf", full(b"dref", struct.pack(">I", 1) + full(b"url ", b"", flags=1)))
        minf = box(b"minf", full(b"smhd", b"\x00" * 4) + dinf + stbl)
        hdlr = full(b"hdlr", b"\x00" * 4 + b"soun" + b"\x00" * 12 + b"SoundHandler\x00")
        mdhd = full(b"mdhd", struct.pack(">IIII", 0, 0, sample_rate, len(frames) * samples_per_frame) + b"\x55\xc4\x00\x00")
        tkhd = full(b"tkhd", struct.pack(">IIII", 0, 0, 2, 0) + b"\x00" * 64, flags=7)
        trak = box(b"trak", tkhd + box(b"mdia", mdhd + hdlr + minf))
        vtrak = b""
        if video_track:
            vh = full(b"hdlr", b"\x00" * 4 + b"vide" + b"\x00" * 12 + b"VideoHandler\x00")
            vmdhd = full(b"mdhd", struct.pack(">IIII", 0, 0, 90000, 0) + b"\x00" * 4)
            vstbl = box(b"stbl", full(b"stsd", struct.pack(">I", 0)))
            vtrak = box(b"trak", full(b"tkhd", struct.pack(">IIII", 0, 0, 1, 0) + b"\x00" * 64) +
                        box(b"mdia", vmdhd + vh + box(b"minf", vstbl)))
        mvhd = full(b"mvhd", struct.pack(">IIII", 0, 0, 1000, 0) + b"\x00" * 80)
        return box(b"moov", mvhd + vtrak + trak)

    ftyp = box(b"ftyp", b"M4A \x00\x00\x02\x00isomM4A mp42")
    if mdat_first:
        moov = build(len(ftyp) + 8)
        return ftyp + box(b"mdat", mdat_body) + moov
    moov = build(0)
    moov = build(len(ftyp) + len(moov) + 8)
    return ftyp + moov + box(b"mdat", mdat_body)
