"""Multichannel HE-AAC (SBR per channel element), channel configurations 3..7.

The reference gives every channel element its own SBR (ChannelElement.decodeSBR, the payload of an
EXT_SBR_DATA fill element belonging to the last audio element, A/syntax/SyntacticElements.java:
207-211).  SCE.process with SBR outputs dataL and dataR -- two channels (A/syntax/SCE.java:
115-132); CPE.process runs SBR2 on its pair (A/syntax/CPE.java:195-204); an LFE carries no SBR
data and is upsampled (one channel).  SyntacticElements.process collects them in element order
(:235-248), so a 5.1 HE-AAC stream gives 7 output channels.

CPU: writer -> parser round trips of the per-element SBR records; refusals (an SCE without SBR
data would change the channel count; SBR on the LFE).  GPU: byte-exact against the restatement
(oracle.decode_batch_mc with sbr), host and device entry, int16 and float32."""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

IDS = N.MC_ELEMENTS


def mc_sbr_synth(cc: int, n_streams: int = 2, fps: int = 12, seed: int = 0, down: bool = False):
    """A multichannel HE-AAC batch: SCEs from mono SBR streams (no upsample frames: an SCE must
    carry SBR data), CPEs from stereo SBR streams (some upsample frames), the LFE from a mono LC
    stream (upsampled); 24 kHz core, SBR to 48 kHz (or downsampled)."""
    els = []
    for k, i in enumerate(IDS[cc]):
        p = N.synth_params(4, n_streams=n_streams, frames_per_stream=fps, channel_config=2 if i == 1 else 1,
                           pns_percent=0)
        p.seed = p.seed + 0x1000 * (k + 1) + seed
        if i == 3:
            p.sbr = 0
            p.window_switching = 0
        elif i == 0:
            p.upsample_percent = 0
        else:
            p.upsample_percent = 10
        els.append(N.synth_batch(p))
    return N.mc_batch(els, IDS[cc])


def writers(cc: int, seed: int, down: bool = False):
    out = 3 + (3 if down else 0)
    return [None if i == 3 else O.SbrWriter(out, seed + k) for k, i in enumerate(IDS[cc])]


@pytest.mark.parametrize("cc", [3, 4, 5, 6, 7])
def test_out_channels(cc):
    cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
    assert N.out_channels(cfg) == {3: 4, 4: 6, 5: 6, 6: 7, 7: 9}[cc]
    assert N.out_channels(N.make_cfg(channel_config=cc)) == N.core_channels(N.make_cfg(channel_config=cc))


@pytest.mark.parametrize("cc", [3, 6, 7])
def test_write_parse_round_trip(cc):
    from tests.test_parse_sbr import _assert_sbr_equal
    b = mc_sbr_synth(cc, n_streams=1, fps=10, seed=cc)
    frames = O.write_frames_mc(b, 6, IDS[cc], sbr_writers=writers(cc, cc))
    cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    got = P.parse(frames)
    for k in ("q", "sf", "cb", "ics", "ms_used"):
        assert getattr(got, k).tobytes() == getattr(b, k).tobytes(), k
    assert got.sbr.shape == (b.n_frames, len(IDS[cc]))
    for e, i in enumerate(IDS[cc]):
        if i == 3:
            assert (got.sbr[:, e]["status"] == N.SBR_UPSAMPLE).all()
        else:
            _assert_sbr_equal(got.sbr[:, e], b.sbr[:, e], 2 if i == 1 else 1, 3)


def test_parse_refusals():
    b = mc_sbr_synth(6, n_streams=1, fps=3, seed=1)
    cfg = N.make_cfg(sf_index=6, channel_config=6, sbr=True)
    # an SCE without SBR data: the reference's channel list would shrink (SCE.java:122-132)
    sbr = b.sbr.copy()
    sbr[1, 0]["status"] = N.SBR_UPSAMPLE  # frame 1: no FIL after the SCE
    b.sbr = sbr
    frames = O.write_frames_mc(b, 6, IDS[6], sbr_writers=writers(6, 1))
    P = N.Parser(cfg)
    P.parse(frames[:1])
    with pytest.raises(N.JaadError) as e:
        P.parse(frames[1:2])
    assert e.value.status == N.ERR_UNSUPPORTED
    # SBR data after the LFE
    b = mc_sbr_synth(6, n_streams=1, fps=2, seed=2)
    sbr = b.sbr.copy()
    sbr[:, 3] = sbr[:, 0]
    b.sbr = sbr
    w = writers(6, 2)
    w[3] = O.SbrWriter(3, 99)
    frames = O.write_frames_mc(b, 6, IDS[6], sbr_writers=w)
    with pytest.raises(N.JaadError) as e:
        N.Parser(cfg).parse(frames[:1])
    assert e.value.status == N.ERR_UNSUPPORTED


def test_oracle_channel_layout():
    """5.1 HE-AAC: 7 channels of 2048 samples; the SCE's two channels are equal (SBR1 without PS
    copies left to right), the LFE is the upsampled core of its element."""
    b = mc_sbr_synth(6, n_streams=1, fps=4, seed=3)
    pcm = O.decode_batch_mc(6, b, IDS[6], N.PCM_BIG_ENDIAN, sbr=True)
    assert pcm.shape == (4, 2048 * 7 * 2)
    s = pcm.view(">i2").reshape(4, 2048, 7)
    assert (s[:, :, 0] == s[:, :, 1]).all()
    c = b.nch - 1  # the LFE's core channel (5.1: SCE, CPE, CPE, LFE = 6 records per frame)
    lfe = O.decode_batch(N.make_cfg(sf_index=6, channel_config=1, sbr=True),
                         N.Batch(np.ascontiguousarray(b.q[c::b.nch]), np.ascontiguousarray(b.sf[c::b.nch]),
                                 np.ascontiguousarray(b.cb[c::b.nch]), np.ascontiguousarray(b.ics[c::b.nch]), None, None,
                                 b.stream_slot.copy(), b.frame_begin.copy(), 1, np.ascontiguousarray(b.sbr[:, 3])),
                         O.Streams(1), N.PCM_BIG_ENDIAN)
    assert (s[:, :, 6] == lfe.view(">i2").reshape(4, 2048, 2)[:, :, 0]).all()


# ------------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("cc", [3, 4, 5, 6, 7])
@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_FLOAT32])
def test_gpu_mc_sbr_matches_oracle(cc, flags):
    b = mc_sbr_synth(cc, n_streams=4, fps=24, seed=cc)
    cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
    want = O.decode_batch_mc(6, b, IDS[cc], flags, threads=8, sbr=True)
    with N.Context(cfg, 4) as ctx:
        got = ctx.decode(b, flags)
    assert got.shape == want.shape
    assert (got == want).all(), np.flatnonzero((got != want).any(1))[:8]


@pytest.mark.gpu
def test_gpu_mc_sbr_calls_device_entry_drops_and_state():
    """Two calls continue the streams (per-element SBR state), the device entry gives the same PCM,
    dropped frames skip every element, and state export/import round-trips a slot."""
    import torch
    cc = 6
    b = mc_sbr_synth(cc, n_streams=3, fps=20, seed=9)
    cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
    want = O.decode_batch_mc(6, b, IDS[cc], N.PCM_BIG_ENDIAN, threads=8, sbr=True)
    a1, a2 = b.split_frames(8)
    with N.Context(cfg, 3) as ctx:
        p1 = ctx.decode(a1, N.PCM_BIG_ENDIAN)
        blob = ctx.state_export(1)
        ctx.state_reset(1)
        ctx.state_import(1, blob)
        p2 = ctx.decode(a2, N.PCM_BIG_ENDIAN)
    fb = b.frame_begin
    for r in range(3):
        assert (p1[8 * r:8 * r + 8] == want[fb[r]:fb[r] + 8]).all()
        assert (p2[12 * r:12 * r + 12] == want[fb[r] + 8:fb[r + 1]]).all()
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).reshape(-1).view(np.uint8)).to(dev)
    d = {k: t(getattr(b, k)) for k in ("q", "sf", "cb", "ics", "ms_used")}
    ptr = {k: v.data_ptr() for k, v in d.items()}
    pcm = torch.empty(want.size, dtype=torch.uint8, device=dev)
    with N.Context(cfg, 3) as ctx:
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), N.PCM_BIG_ENDIAN)
        ctx.wait()
    assert (pcm.cpu().numpy().reshape(want.shape) == want).all()
    st = np.zeros(b.n_frames, np.uint8)
    st[[0, 7, 8, 30, 59]] = N.FRAME_EOS
    b.frame_status = st
    from tests.test_frame_status import no_header_before_first_sbr
    no_header_before_first_sbr(b, st)
    want2 = O.decode_batch_mc(6, b, IDS[cc], N.PCM_BIG_ENDIAN, threads=8, sbr=True)
    out = np.full(want2.shape, 0x11, np.uint8)
    with N.Context(cfg, 3) as ctx:
        ctx.decode(b, N.PCM_BIG_ENDIAN, out=out)
    assert (out[st == 1] == 0x11).all() and (out[st == 0] == want2[st == 0]).all()


@pytest.mark.gpu
def test_gpu_mc_sbr_bitstream_through_the_decoder_facade():
    """ADTS 5.1 HE-AAC frames -> Decoder.decodeFrame: 7 channels per SampleBuffer, equal to the
    restatement on the parsed records."""
    from jaadec_amd.decoder import Decoder, DecoderConfig, SampleBuffer
    cc = 6
    b = mc_sbr_synth(cc, n_streams=1, fps=8, seed=4)
    frames = O.write_frames_mc(b, 6, IDS[cc], sbr_writers=writers(cc, 4))
    P = N.Parser(N.make_cfg(sf_index=6, channel_config=cc, sbr=True))
    P.pns_state = int(b.ics["pns_state"][0])
    pb = P.parse(frames)
    want = O.decode_batch_mc(6, pb, IDS[cc], N.PCM_BIG_ENDIAN, sbr=True)
    conf = DecoderConfig(2, 6, cc, sbr=True, ext_sf_index=3)
    dec = Decoder(conf)
    dec._parse([])
    dec._parser.pns_state = int(b.ics["pns_state"][0])
    for i, fr in enumerate(frames):
        buf = SampleBuffer()
        dec.decodeFrame(fr, buf)
        assert buf.getChannels() == 7 and buf.getData() == want[i].tobytes(), i
    dec.close()


@pytest.mark.gpu
def test_gpu_mc_sbr_rejected_element_leaves_every_element_as_it_was():
    """element 2 of a 5.1 HE-AAC batch carries SBR data the stage refuses (a PS payload
    with borders out of order is not what ps_data_decode produces; here: an unknown SBR status);
    the call fails before any element launches, every element's slot state (core overlap, SBR
    rings, host SBR state) is as before, and the same stream then decodes as if the call had not
    happened.  And a state blob whose last element is bad is refused whole."""
    cc = 6
    b = mc_sbr_synth(cc, n_streams=2, fps=16, seed=9)
    cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
    want = O.decode_batch_mc(6, b, IDS[cc], N.PCM_BIG_ENDIAN, threads=8, sbr=True)
    a1, a2 = b.split_frames(6)
    bad = N.Batch(a2.q, a2.sf, a2.cb, a2.ics, a2.ms_used, a2.tns, a2.stream_slot, a2.frame_begin, a2.nch,
                  a2.sbr.copy(), **a2._cce_for(np.arange(a2.n_frames)))
    bad.sbr["status"][3, 2] = 7  # element 2 (a CPE), frame 3 of the first run
    with N.Context(cfg, 2) as ctx:
        p1 = ctx.decode(a1, N.PCM_BIG_ENDIAN)
        before = [ctx.state_export(s) for s in range(2)]
        with pytest.raises(N.JaadError) as e:
            ctx.decode(bad, N.PCM_BIG_ENDIAN)
        assert e.value.status in (N.ERR_INVALID_ARG, N.ERR_BITSTREAM)
        for s in range(2):
            assert (ctx.state_export(s) == before[s]).all(), s
        p2 = ctx.decode(a2, N.PCM_BIG_ENDIAN)
        # a blob whose last element's overlap is not finite: refused before any element is written
        blob = ctx.state_export(0)
        broken = blob.copy()
        n = len(broken)
        last = 3 * n // 4  # four elements with blobs of one size: the LFE's overlap starts here
        broken[last:last + 4] = np.frombuffer(np.float32(np.inf).tobytes(), np.uint8)
        ctx.state_reset(0)
        reset = ctx.state_export(0)
        with pytest.raises(N.JaadError):
            ctx.state_import(0, broken)
        assert (ctx.state_export(0) == reset).all()
    fb = b.frame_begin
    for r in range(2):
        assert (p1[6 * r:6 * r + 6] == want[fb[r]:fb[r] + 6]).all()
        assert (p2[10 * r:10 * r + 10] == want[fb[r] + 6:fb[r + 1]]).all()
