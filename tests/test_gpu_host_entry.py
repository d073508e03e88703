"""The host-buffer entry (jaad_decode_batch): the pieces pipelines for large batches (AAC-LC: the
LC kernel per piece; HE-AAC v1/v2 and batches with dropped frames: whole launches per piece), with
pageable and registered (jaad_host_register) caller buffers, against the device-resident entry
and the C restatement; validation failures leave every slot's state untouched."""
import numpy as np
import pytest
import torch

from jaadec_amd import native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _device_decode(cfg, b, n_slots, flags):
    dev = torch.device("cuda", 0)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
    d = {k: t(getattr(b, k)) for k in ("q", "sf", "cb", "ics", "ms_used", "tns")}
    ptr = {k: (v.data_ptr() if v is not None else None) for k, v in d.items()}
    nb = N.pcm_frame_bytes(flags, bool(cfg.sbr), N.sbr_downsampled(cfg))
    pcm = torch.empty(b.n_frames * nb, dtype=torch.uint8, device=dev)
    with N.Context(cfg, n_slots) as ctx:
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), flags)
        ctx.wait()
    return pcm.cpu().numpy().reshape(b.n_frames, nb)


def _ragged(b, lens):
    """Runs of the given lengths (prefixes of b's runs)."""
    fb = b.frame_begin
    frames = np.concatenate([np.arange(fb[r], fb[r] + L) for r, L in enumerate(lens)])
    cfr = (frames[:, None] * b.nch + np.arange(b.nch)).reshape(-1)
    begin = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
    return N.Batch(b.q[cfr].copy(), b.sf[cfr].copy(), b.cb[cfr].copy(), b.ics[cfr].copy(),
                   None if b.ms_used is None else b.ms_used[frames].copy(),
                   None if b.tns is None else b.tns[cfr].copy(), b.stream_slot[:len(lens)].copy(), begin, b.nch)


@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_FLOAT32])
def test_pieces_pipeline_matches_device_entry_and_oracle(flags):
    p = N.synth_params(3, n_streams=24, frames_per_stream=700)  # 16 800 frames: 4 pieces
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    with N.Context(cfg, 24) as ctx:
        got = ctx.decode(b, flags)
    want_dev = _device_decode(cfg, b, 24, flags)
    assert (got == want_dev).all()
    sub = b.select_runs([0, 11, 23])
    want = O.decode_batch(cfg, sub, O.Streams(24), flags, threads=8)
    fb = b.frame_begin
    g = np.concatenate([got[fb[r]:fb[r + 1]] for r in (0, 11, 23)])
    assert (g == want).all()


def test_registered_buffers_and_continuation():
    p = N.synth_params(2, n_streams=12, frames_per_stream=1400)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    first, second = b.split_frames(900)  # 10 800 frames, then 6 000 frames: both piecewise
    want = np.concatenate(
        [_device_decode(cfg, b, 12, N.PCM_BIG_ENDIAN)[b.frame_begin[r]:b.frame_begin[r + 1]] for r in range(12)])
    with N.Context(cfg, 12) as ctx:
        out1 = np.empty((first.n_frames, 4096), np.uint8)
        out2 = np.empty((second.n_frames, 4096), np.uint8)
        arrays = [first.q, first.sf, first.cb, first.ics, first.ms_used, out1]
        ctx.register(*arrays)
        g1 = ctx.decode(first, out=out1)
        g2 = ctx.decode(second, out=out2)  # pageable
        ctx.unregister(*arrays)
    got = np.empty_like(want)
    i1 = i2 = 0
    for r in range(12):
        got[r * 1400:r * 1400 + 900] = g1[i1:i1 + 900]
        got[r * 1400 + 900:(r + 1) * 1400] = g2[i2:i2 + 500]
        i1 += 900
        i2 += 500
    assert (got == want).all()


def test_ragged_runs_and_few_runs():
    p = N.synth_params(2, n_streams=3, frames_per_stream=9000)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    rag = _ragged(b, [9000, 17, 5000])  # 3 runs, pieces of unequal size
    with N.Context(cfg, 3) as ctx:
        got = ctx.decode(rag, N.PCM_FLOAT32)
    assert (got == _device_decode(cfg, rag, 3, N.PCM_FLOAT32)).all()


def test_bad_piece_leaves_state_untouched():
    p = N.synth_params(2, n_streams=16, frames_per_stream=1024)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    with N.Context(cfg, 16) as ctx:
        half, rest = b.split_frames(512)
        ctx.decode(half)
        before = [ctx.state_export(s) for s in range(16)]
        bad = rest.select_runs(range(16))
        bad.q[-1, 5] = 9000  # |q| > 8190 in the last piece
        with pytest.raises(N.JaadError) as e:
            ctx.decode(bad)
        assert e.value.status == N.ERR_BITSTREAM
        assert all((ctx.state_export(s) == before[s]).all() for s in range(16))
        # the good batch still continues every stream exactly
        g2 = ctx.decode(rest)
    want = _device_decode(cfg, b, 16, N.PCM_BIG_ENDIAN)
    fb = b.frame_begin
    i = 0
    for r in range(16):
        assert (g2[i:i + 512] == want[fb[r] + 512:fb[r + 1]]).all()
        i += 512


def test_host_alloc_buffers_and_foreign_pinned_memory():
    """Batch and PCM in jaad_host_alloc memory (DMA straight from it), then the same batch in
    memory page-locked by someone else (torch's pinned allocator) passed to jaad_host_register,
    which records it without registering it again; both equal the device entry."""
    p = N.synth_params(2, n_streams=10, frames_per_stream=1000)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    want = _device_decode(cfg, b, 10, N.PCM_BIG_ENDIAN)
    with N.Context(cfg, 10) as ctx:
        hb = ctx.host_batch(b)
        out = ctx.host_array((b.n_frames, 4096))
        ctx.decode(hb, out=out)
        assert (out == want).all()
        ctx.free_host(hb.q, hb.sf, hb.cb, hb.ics, hb.ms_used, out)
        with pytest.raises(N.JaadError):
            ctx.free_host(hb.q)  # freed already
    with N.Context(cfg, 10) as ctx:
        def pin(a):
            raw = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
            return torch.from_numpy(raw).pin_memory().numpy().view(a.dtype).reshape(a.shape)
        tb = N.Batch(pin(b.q), pin(b.sf), pin(b.cb), pin(b.ics), pin(b.ms_used), None, b.stream_slot, b.frame_begin,
                     b.nch)
        out2 = torch.empty(b.n_frames * 4096, dtype=torch.uint8).pin_memory().numpy().reshape(b.n_frames, 4096)
        arrays = [tb.q, tb.sf, tb.cb, tb.ics, tb.ms_used, out2]
        ctx.register(*arrays)
        ctx.decode(tb, out=out2)
        ctx.unregister(*arrays)
    assert (out2 == want).all()


@pytest.mark.gpu
def test_registering_a_range_twice_is_idempotent():
    """a second jaad_host_register of the same range keeps one entry, so one unregister
    releases it and a second one is refused; a longer range at the same address is refused."""
    p = N.synth_params(2, n_streams=2, frames_per_stream=8)
    b = N.synth_batch(p)
    with N.Context(N.cfg_for(p), 2) as ctx:
        want = ctx.decode(b, N.PCM_BIG_ENDIAN)
        ctx.register(b.q)
        ctx.register(b.q)
        import ctypes as C
        assert N.lib().jaad_host_register(ctx.h, C.c_void_p(b.q.ctypes.data), C.c_size_t(b.q.nbytes + 4096)) == \
            N.ERR_INVALID_ARG
        for s in range(2):
            ctx.state_reset(s)
        assert (ctx.decode(b, N.PCM_BIG_ENDIAN) == want).all()
        ctx.unregister(b.q)
        with pytest.raises(N.JaadError) as e:
            ctx.unregister(b.q)
        assert e.value.status == N.ERR_INVALID_ARG


def _runs_of(pcm_a, pcm_b, fb_a, fb_b, runs):
    return all((pcm_a[fb_a[r]:fb_a[r + 1]] == pcm_b[fb_b[r]:fb_b[r + 1]]).all() for r in runs)


@pytest.mark.parametrize("cfgid,flags", [(4, N.PCM_BIG_ENDIAN), (5, N.PCM_LITTLE_ENDIAN), (5, N.PCM_FLOAT32)])
def test_sbr_ps_pieces_pipeline_matches_device_entry(cfgid, flags):
    """HE-AAC v1 / v2 batches through the host-buffer entry run as pieces of whole
    launches whose copies overlap; two calls (the second continuing every stream) == the device
    entry over the whole streams, and == the restatement on a sample of streams."""
    p = N.synth_params(cfgid, n_streams=64, frames_per_stream=160)  # 10 240 frames: 5 pieces
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    first, second = b.split_frames(100)
    with N.Context(cfg, 64) as ctx:
        g1 = ctx.decode(first, flags)
        g2 = ctx.decode(second, flags)
    want = _device_decode(cfg, b, 64, flags)
    fb = b.frame_begin
    for r in range(64):
        assert (g1[100 * r:100 * (r + 1)] == want[fb[r]:fb[r] + 100]).all(), r
        assert (g2[60 * r:60 * (r + 1)] == want[fb[r] + 100:fb[r + 1]]).all(), r
    sub = b.select_runs([0, 63])
    o = O.decode_batch(cfg, sub, O.Streams(64), flags, threads=8)
    assert (np.concatenate([want[fb[r]:fb[r + 1]] for r in (0, 63)]) == o).all()


def test_sbr_pieces_registered_buffers_and_dropped_frames():
    """The same pipeline with registered caller buffers, and with a dropped frame in every stream
    (their PCM rows keep the caller's bytes)."""
    p = N.synth_params(4, n_streams=48, frames_per_stream=128)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    rng = np.random.default_rng(3)
    st = np.zeros(b.n_frames, np.uint8)
    for r in range(48):
        st[int(b.frame_begin[r]) + int(rng.integers(1, 128))] = N.FRAME_EOS
    b.frame_status = st
    want = O.decode_batch(cfg, b.select_runs([5, 40]), O.Streams(48), N.PCM_BIG_ENDIAN, threads=8)
    want_dev = _device_decode(cfg, b, 48, N.PCM_BIG_ENDIAN)
    for registered in (False, True):
        out = np.full((b.n_frames, 8192), 0x5A, np.uint8)
        with N.Context(cfg, 48) as ctx:
            arrays = [b.q, b.sf, b.cb, b.ics, b.ms_used, out]
            if registered:
                ctx.register(*arrays)
            ctx.decode(b, N.PCM_BIG_ENDIAN, out=out)
            if registered:
                ctx.unregister(*arrays)
        assert (out[st == 1] == 0x5A).all(), registered
        assert (out[st == 0] == want_dev[st == 0]).all(), registered
        fb = b.frame_begin
        got = np.concatenate([out[fb[r]:fb[r + 1]] for r in (5, 40)])
        keep = np.concatenate([st[fb[r]:fb[r + 1]] for r in (5, 40)]) == 0
        assert (got[keep] == want[keep]).all()


@pytest.mark.parametrize("what", ["q", "sbr"])
def test_sbr_bad_piece_rolls_the_call_back(what):
    """A bad record in the last piece (|q| > 8190, or an SBR envelope count the reference cannot
    have parsed) fails the call after earlier pieces' kernels ran: every slot's core, SBR and PS
    state is put back, and the good batch then continues every stream exactly."""
    p = N.synth_params(5, n_streams=64, frames_per_stream=160)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    want = _device_decode(cfg, b, 64, N.PCM_BIG_ENDIAN)
    half, rest = b.split_frames(80)
    with N.Context(cfg, 64) as ctx:
        ctx.decode(half)
        before = [ctx.state_export(s) for s in range(64)]
        bad = rest.select_runs(range(64))
        if what == "q":
            bad.q[-1, 7] = 9000
        else:
            s = bad.sbr.copy()
            s["ch"]["L_E"][-3, 0] = 7
            bad = N.Batch(bad.q, bad.sf, bad.cb, bad.ics, bad.ms_used, bad.tns, bad.stream_slot, bad.frame_begin,
                          bad.nch, s)
        with pytest.raises(N.JaadError) as e:
            ctx.decode(bad)
        assert e.value.status == N.ERR_BITSTREAM
        assert all((ctx.state_export(s) == before[s]).all() for s in range(64))
        g2 = ctx.decode(rest)
    fb = b.frame_begin
    for r in range(64):
        assert (g2[80 * r:80 * (r + 1)] == want[fb[r] + 80:fb[r + 1]]).all(), r


# ------------------------------------------------------------------------------------------------
# multichannel AAC-LC and coupling batches through the pipelined host entry (VERDICT r4 missing #4)
# ------------------------------------------------------------------------------------------------

def _mc_device_decode(cfg, b, n_slots, flags):
    """The device entry for a multichannel batch (PCM: out_channels(cfg) channels a sample)."""
    dev = torch.device("cuda", 0)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
    d = {k: t(getattr(b, k)) for k in ("q", "sf", "cb", "ics", "ms_used", "tns")}
    ptr = {k: (v.data_ptr() if v is not None else None) for k, v in d.items()}
    nb = 1024 * N.out_channels(cfg) * (4 if flags & N.PCM_FLOAT32 else 2)
    pcm = torch.empty(b.n_frames * nb, dtype=torch.uint8, device=dev)
    with N.Context(cfg, n_slots) as ctx:
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), flags)
        ctx.wait()
    return pcm.cpu().numpy().reshape(b.n_frames, nb)


@pytest.mark.parametrize("cc", [6, 7])
def test_multichannel_pieces_pipeline(cc):
    """5.1 / 7.1 AAC-LC batches large enough for pieces: the pipelined host entry == the device
    entry over the whole batch and == the restatement on a sample of streams; a second call
    continues every stream."""
    from tests.test_multichannel import mc_synth, IDS
    b = mc_synth(cc, n_streams=16, fps=320, seed=4)  # 5 120 frames: 2 pieces
    cfg = N.make_cfg(channel_config=cc)
    first, second = b.split_frames(200)
    with N.Context(cfg, 16) as ctx:
        g1 = ctx.decode(first)
        g2 = ctx.decode(second)
    want = _mc_device_decode(cfg, b, 16, N.PCM_BIG_ENDIAN)
    fb = b.frame_begin
    for r in range(16):
        assert (g1[200 * r:200 * (r + 1)] == want[fb[r]:fb[r] + 200]).all(), r
        assert (g2[120 * r:120 * (r + 1)] == want[fb[r] + 200:fb[r + 1]]).all(), r
    sub = b.select_runs([0, 15])
    o = O.decode_batch_mc(3, sub, IDS[cc], N.PCM_BIG_ENDIAN, threads=8)
    assert (np.concatenate([want[fb[r]:fb[r + 1]] for r in (0, 15)]) == o).all()


def test_multichannel_bad_piece_rolls_back():
    from tests.test_multichannel import mc_synth
    b = mc_synth(6, n_streams=16, fps=320, seed=5)
    cfg = N.make_cfg(channel_config=6)
    half, rest = b.split_frames(160)
    with N.Context(cfg, 16) as ctx:
        ctx.decode(half)
        before = [ctx.state_export(s) for s in range(16)]
        bad = rest.select_runs(range(16))
        bad.q[-1, 3] = 9000  # the last piece
        with pytest.raises(N.JaadError) as e:
            ctx.decode(bad)
        assert e.value.status == N.ERR_BITSTREAM
        assert all((ctx.state_export(s) == before[s]).all() for s in range(16))


@pytest.mark.parametrize("cc,sbr", [(2, False), (2, True), (6, False)])
def test_coupling_pieces_pipeline(cc, sbr):
    """Coupling batches as run-aligned pieces: each piece gets its frames' terms, renumbered; the
    CCE records are uploaded once.  == the restatement (stereo LC over the whole batch; HE-AAC and
    5.1 on a sample of streams)."""
    from tests.test_cce import coupled_batch, coupled_sbr_batch
    from tests.test_multichannel import IDS
    if sbr:
        b = coupled_sbr_batch(cc, n_streams=16, fps=300, seed=61)
        cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
    else:
        b = coupled_batch(cc, n_streams=16, fps=300, seed=62)
        cfg = N.make_cfg(channel_config=cc)
    assert len(b.cce_terms) > 1000
    with N.Context(cfg, 16) as ctx:
        got = ctx.decode(b, N.PCM_BIG_ENDIAN)
    runs = (0, 7, 15)
    sub = b.select_runs(list(runs))
    if cc in N.MC_ELEMENTS:
        want = O.decode_batch_mc(3, sub, IDS[cc], N.PCM_BIG_ENDIAN, threads=8)
    else:
        want = O.decode_batch(cfg, sub, O.Streams(16), N.PCM_BIG_ENDIAN, threads=8)
    fb = b.frame_begin
    assert (np.concatenate([got[fb[r]:fb[r + 1]] for r in runs]) == want).all()


def test_multichannel_he_aac_pieces_and_roll_back():
    """5.1 HE-AAC (one SBR child context per element) through the pipelined entry: two calls ==
    the restatement on every stream; then a call whose last piece fails puts every element's core
    and SBR state back (the good call after it continues the streams exactly)."""
    from tests.test_mc_sbr import mc_sbr_synth, IDS
    b = mc_sbr_synth(6, n_streams=24, fps=300, seed=21)
    cfg = N.make_cfg(sf_index=6, channel_config=6, sbr=True)
    want = O.decode_batch_mc(6, b, IDS[6], N.PCM_BIG_ENDIAN, threads=8, sbr=True)
    first, second = b.split_frames(120)  # 2 880 frames (one launch), then 4 320 (2 pieces)
    fb = b.frame_begin
    with N.Context(cfg, 24) as ctx:
        g1 = ctx.decode(first)
        before = [ctx.state_export(s) for s in range(24)]
        bad = second.select_runs(range(24))
        bad.q[-1, 5] = 9000  # in the last piece
        with pytest.raises(N.JaadError) as e:
            ctx.decode(bad)
        assert e.value.status == N.ERR_BITSTREAM
        assert all((ctx.state_export(s) == before[s]).all() for s in range(24))
        g2 = ctx.decode(second)
    for r in range(24):
        assert (g1[120 * r:120 * (r + 1)] == want[fb[r]:fb[r] + 120]).all(), r
        assert (g2[180 * r:180 * (r + 1)] == want[fb[r] + 120:fb[r + 1]]).all(), r


def test_coupling_with_ps_time_slices():
    """An HE-AAC v2 batch with coupling terms through the time-sliced pipeline: each slice gets its
    runs' terms, renumbered; == the restatement on a sample of streams."""
    from tests.test_cce import cce_records
    p = N.synth_params(5, n_streams=16, frames_per_stream=300)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    rng = np.random.default_rng(71)
    n_rec = 64
    b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics = cce_records(n_rec, 71, pns=10, sf_index=p.sf_index)
    terms = []
    for f in range(b.n_frames):
        if rng.integers(3):
            continue
        t = np.zeros((), N.CCE_TERM_DTYPE)
        t["frame"], t["channel"], t["point"], t["cce"] = f, 0, rng.integers(2), rng.integers(n_rec)
        t["gain"] = rng.choice([0.0, 1.0, -0.5, 2.0, 1.0905077], 120).astype(np.float32)
        terms.append(t)
    b.cce_terms = np.array(terms, N.CCE_TERM_DTYPE)
    with N.Context(cfg, 16) as ctx:
        got = ctx.decode(b, N.PCM_BIG_ENDIAN)
    runs = (0, 9, 15)
    want = O.decode_batch(cfg, b.select_runs(list(runs)), O.Streams(16), N.PCM_BIG_ENDIAN, threads=8)
    fb = b.frame_begin
    assert (np.concatenate([got[fb[r]:fb[r + 1]] for r in runs]) == want).all()


@pytest.mark.parametrize("fps,pieces", [(3, 8), (4, 6)])
def test_ps_time_slices_with_runs_shorter_than_the_slice_count(fps, pieces, monkeypatch):
    """HE-AAC v2 time slices of runs shorter than P frames -- some slices then hold
    no frame at all.  Every non-empty slice's PCM goes through the two page-locked staging slots
    (pageable output) and must reach the caller: == the device entry over the whole batch, and ==
    the restatement on a sample of streams.  (Before round 6 the staging slot was picked by piece
    index, so the PCM of the piece two before an empty one was never copied out.)"""
    n_streams = (2048 * pieces + fps - 1) // fps  # P = min(JAAD_SBR_PIECES, frames / 2048) slices
    p = N.synth_params(5, n_streams=n_streams, frames_per_stream=fps)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    monkeypatch.setenv("JAAD_SBR_PIECES", str(pieces))
    with N.Context(cfg, n_streams) as ctx:
        got = ctx.decode(b, N.PCM_BIG_ENDIAN)
    want = _device_decode(cfg, b, n_streams, N.PCM_BIG_ENDIAN)
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, f"{bad.size} frames differ, first {bad[:8]}"
    runs = [0, n_streams // 2, n_streams - 1]
    o = O.decode_batch(cfg, b.select_runs(runs), O.Streams(n_streams), N.PCM_BIG_ENDIAN, threads=8)
    fb = b.frame_begin
    assert (np.concatenate([got[fb[r]:fb[r + 1]] for r in runs]) == o).all()
