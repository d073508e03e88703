"""MP4 transport feeder (include/jaad_mp4.h, jaadec_amd/mp4.py): the reference's
MP4Container -> Movie -> AudioTrack -> readNextFrame chain (M/api/*.java) as S/Main.java:49-80
uses it.  Files come from the test writer (oracle/mp4_writer.py) over frames written by the
bitstream writer, so every layer is checked against known contents: box tree, esds
DecoderSpecificInfo, the stsc/stco/stsz frame table, and the records the frames parse to."""
import numpy as np
import pytest

from jaadec_amd import mp4 as M
from jaadec_amd import native as N
from oracle import mp4_writer as W
from oracle import oracle as O


def _lc_stream(frames=14):
    p = N.synth_params(3, n_streams=1, frames_per_stream=frames)
    b = N.synth_batch(p)
    return p, b, O.write_frames(b, p.sf_index)


@pytest.mark.parametrize("opts", [
    {},
    dict(co64=True),
    dict(video_track=True, long_desc=True),
    dict(mdat_first=True, chunk_sizes=(1,)),
    dict(esds_url=b"http://x", chunk_sizes=(4, 4, 2, 7)),
], ids=["plain", "co64", "video_longdesc", "mdat_first", "url_mixed_chunks"])
def test_mp4_round_trip(opts):
    p, b, frames = _lc_stream()
    asc = bytes([0x11, 0x90])  # AAC LC, 48 kHz, stereo
    data = W.write_mp4(frames, asc, 48000, 2, **opts)
    movie = M.MP4Container(data).getMovie()
    tracks = movie.getTracks(M.AudioCodec.AAC)
    assert len(tracks) == 1 and len(movie.getTracks()) == 1  # the video track is not an audio track
    t = tracks[0]
    assert (t.getSampleRate(), t.getChannelCount(), t.getSampleSize()) == (48000, 2, 16)
    assert t.getDecoderSpecificInfo().getData() == asc
    got = []
    while t.hasMoreFrames():
        f = t.readNextFrame()
        assert abs(f.getTime() - len(got) * 1024 / 48000) < 1e-12
        got.append(f.getData())
    assert got == frames
    with pytest.raises(EOFError):
        t.readNextFrame()
    # the frames parse to the records they were written from
    P = N.Parser(N.asc_parse(t.getDecoderSpecificInfo().getData()))
    P.pns_state = int(b.ics["pns_state"][0])
    rec = P.parse(got)
    assert np.array_equal(rec.q, b.q) and np.array_equal(rec.ics, b.ics)


def test_mp4_he_aac_track():
    p = N.synth_params(4, n_streams=1, frames_per_stream=10)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 2))
    asc = bytes([0x2B, 0x11, 0x88, 0x00])  # AOT 5, 24 kHz core, 48 kHz output, stereo
    t = M.MP4Container(W.write_mp4(frames, asc, 48000, 2, samples_per_frame=2048)).getMovie().getTracks()[0]
    c = N.asc_parse(t.getDecoderSpecificInfo().getData())
    assert (c.sbr, c.sf_index, c.ext_sf_index) == (1, 6, 3)
    P = N.Parser(c)
    got = P.parse([t.readNextFrame().getData() for _ in range(t.getFrameCount())])
    assert np.array_equal(got.q, b.q)


def test_mp4_seek_follows_the_reference_loop():
    """Track.seek steps its index twice per iteration (M/api/Track.java:359-370): it tests frames
    0, 2, 4, ... and leaves the cursor one past the frame it reports."""
    _, _, frames = _lc_stream(10)
    t = M.MP4Container(W.write_mp4(frames, bytes([0x11, 0x90]), 48000, 2)).getMovie().getTracks()[0]
    dt = 1024 / 48000
    assert t.seek(2.5 * dt) == pytest.approx(4 * dt)   # frame 3 is never tested
    assert t.readNextFrame().getData() == frames[5]
    assert t.seek(100.0) == pytest.approx(8 * dt)     # last frame tested; the cursor stays
    assert t.readNextFrame().getData() == frames[6]


def test_mp4_errors():
    _, _, frames = _lc_stream(6)
    data = W.write_mp4(frames, bytes([0x11, 0x90]), 48000, 2)
    with pytest.raises(N.JaadError) as e:
        M.MP4Container(data[:60])  # the image ends inside moov
    assert e.value.status == N.ERR_EOS
    with pytest.raises(N.JaadError) as e:
        M.MP4Container(b"\x00\x00\x00\x10free" + b"\x00" * 8)  # no moov
    assert e.value.status == N.ERR_BITSTREAM
    # mdat cut short: the table is intact, the last frames cannot be read
    cut = data[:-len(frames[-1]) // 2]
    t = M.MP4Container(cut).getMovie().getTracks()[0]
    for _ in range(5):
        t.readNextFrame()
    with pytest.raises(EOFError):
        t.readNextFrame()


def test_mp4_huge_sample_count_is_rejected():
    """A fixed-size stsz claiming 2^28 samples in a ~1 KB file is corrupt: rejected before any
    table is sized from it (no allocation from the claimed count)."""
    _, _, frames = _lc_stream(4)
    data = bytearray(W.write_mp4(frames, bytes([0x11, 0x90]), 48000, 2))
    i = data.find(b"stsz")
    assert i > 0
    # version/flags(4) | sample_size(4) | sample_count(4): make it fixed-size with 2^28 samples
    data[i + 8:i + 12] = (64).to_bytes(4, "big")
    data[i + 12:i + 16] = (1 << 28).to_bytes(4, "big")
    with pytest.raises(N.JaadError) as e:
        M.MP4Container(bytes(data))
    assert e.value.status == N.ERR_BITSTREAM
    # per-sample sizes: a count beyond the box's bytes ends the box early
    data[i + 8:i + 12] = (0).to_bytes(4, "big")
    data[i + 12:i + 16] = (1 << 27).to_bytes(4, "big")
    with pytest.raises(N.JaadError) as e:
        M.MP4Container(bytes(data))
    assert e.value.status == N.ERR_EOS


def test_adts_split_is_linear():
    """adts_frames searches one buffer at an offset (no per-frame copy of the rest of the file)."""
    import time
    _, _, frames = _lc_stream(6)
    one = O.adts_wrap(frames, 3, 2)
    t0 = time.perf_counter()
    n = sum(1 for _ in N.adts_frames(one * 2000))  # 12 000 frames, ~6 MB
    dt = time.perf_counter() - t0
    assert n == 12000
    assert dt < 5.0, dt


def test_mp4_exports():
    L = N.lib()
    for name in M.MP4_EXPORTS:
        assert hasattr(L, name), name


@pytest.mark.gpu
@pytest.mark.parametrize("cfgid", [3, 4])
def test_mp4_file_decodes_on_the_gpu(cfgid):
    """S/Main.java decodeMP4: MP4 -> AudioTrack frames -> Decoder.create(DSI) -> decodeFrame, PCM
    equal to the restatement's decode of the records, byte for byte."""
    from jaadec_amd.decoder import Decoder, SampleBuffer
    p = N.synth_params(cfgid, n_streams=1, frames_per_stream=16)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    sw = O.SbrWriter(cfg.ext_sf_index, 4) if cfg.sbr else None
    frames = O.write_frames(b, p.sf_index, sbr_writer=sw)
    asc = bytes([0x11, 0x90]) if cfgid == 3 else bytes([0x2B, 0x11, 0x88, 0x00])
    track = M.MP4Container(W.write_mp4(frames, asc, 48000, 2)).getMovie().getTracks(M.AudioCodec.AAC)[0]
    dec = Decoder.create(track.getDecoderSpecificInfo().getData())
    out = []
    while track.hasMoreFrames():
        buf = SampleBuffer()
        dec.decodeFrame(track.readNextFrame().getData(), buf)
        out.append(buf.data)
    want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    assert b"".join(out) == want.tobytes()
    dec.close()
