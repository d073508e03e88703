"""Per-frame status in the batch ABI (jaad_batch.frame_status): a frame whose
bitstream ended early is dropped as Decoder.decodeFrame drops it (A/Decoder.java:89-101: the
EOSException is caught, process() and buffer.accept are skipped, the frame still counts) -- no DSP
for it, its PCM slot untouched, its stream continuing from the previous frame's state -- while
the rest of the batch decodes.

CPU: Parser.parse(drop_eos=True) marks the truncated frame and parses the next ones as if it were
absent; the restatement with a status array equals the restatement of the batch without those
frames.  GPU: every path (AAC-LC stereo/mono, window switching, HE-AAC v1/v2, multichannel,
coupling, host and device entry, the Decoder facade, the JNI glue) against the restatement."""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O


def without_frames(b: N.Batch, drop) -> N.Batch:
    """b with the given frames removed (runs shortened, slots kept): what the stream sees when the
    dropped frames never happened."""
    drop = set(int(f) for f in drop)
    fb = b.frame_begin
    keep, lens = [], []
    for r in range(len(b.stream_slot)):
        fr = [f for f in range(int(fb[r]), int(fb[r + 1])) if f not in drop]
        keep += fr
        lens.append(len(fr))
    frames = np.array(keep, np.int64)
    cfr = (frames[:, None] * b.nch + np.arange(b.nch)[None, :]).reshape(-1)
    begin = np.zeros(len(lens) + 1, np.uint32)
    begin[1:] = np.cumsum(lens)
    return N.Batch(np.ascontiguousarray(b.q[cfr]), np.ascontiguousarray(b.sf[cfr]), np.ascontiguousarray(b.cb[cfr]),
                   np.ascontiguousarray(b.ics[cfr]),
                   None if b.ms_used is None else np.ascontiguousarray(b.ms_used[frames]),
                   None if b.tns is None else np.ascontiguousarray(b.tns[cfr]),
                   b.stream_slot.copy(), begin, b.nch,
                   None if b.sbr is None else np.ascontiguousarray(b.sbr[frames]), **b._cce_for(frames))


def drop_pattern(b: N.Batch) -> np.ndarray:
    """Dropped frames at a run's first frame, in the middle, two in a row, and a run's last frame."""
    fb = b.frame_begin
    st = np.zeros(b.n_frames, np.uint8)
    st[int(fb[0])] = N.FRAME_EOS
    r = len(b.stream_slot) // 2
    mid = (int(fb[r]) + int(fb[r + 1])) // 2
    st[mid] = st[mid + 1] = N.FRAME_EOS
    st[int(fb[-1]) - 1] = N.FRAME_EOS
    st[int(fb[1]) + 5] = N.FRAME_EOS
    return st


def no_header_before_first_sbr(b: N.Batch, st: np.ndarray) -> None:
    """The SBR records of dropped frames that come before their run's first decoded frame lose their
    header: a frame dropped after its SBR payload hands its header to the SBR state (the reference's
    SBR.decode swapped it in before the EOSException), which needs a processed frame before it
    (SbrHost::take_header; the restatement refuses the same case).  The synthetic batches carry a
    header in every frame; here a run's leading dropped frames stand for frames cut before their
    SBR payload."""
    if b.sbr is None:
        return
    s = b.sbr.reshape(b.n_frames, -1)
    fb = b.frame_begin
    for r in range(len(b.stream_slot)):
        for f in range(int(fb[r]), int(fb[r + 1])):
            if not st[f]:
                break
            s["header_present"][f] = 0


def oracle_pcm(cfg, b, flags, threads=4):
    nsl = int(b.stream_slot.max()) + 1
    return O.decode_batch(cfg, b, O.Streams(nsl), flags, threads=threads)


def test_oracle_status_equals_the_batch_without_the_frames():
    p = N.synth_params(3, n_streams=3, frames_per_stream=16)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    st = drop_pattern(b)
    b.frame_status = st
    got = oracle_pcm(cfg, b, N.PCM_BIG_ENDIAN)
    assert not got[st == 1].any()  # dropped rows untouched (zero)
    b.frame_status = None
    want = oracle_pcm(cfg, without_frames(b, np.flatnonzero(st)), N.PCM_BIG_ENDIAN)
    assert (got[st == 0] == want).all()


LCG_A, LCG_C = 1664525, 1013904223  # ICStream.randomState (A/syntax/ICStream.java:247)


def noise_prefix(b: N.Batch, f: int) -> list:
    """Noise bins that decodeSpectralData has consumed at each band boundary of frame f, channels in
    bitstream order (A/syntax/ICStream.java:222-275: groups, bands, windows; a noise band takes
    width x group-length LCG steps)."""
    from test_tables import table
    swl = table("JAAD_SWB_OFFSET_1024_48").astype(int)
    sws = table("JAAD_SWB_OFFSET_128_48").astype(int)
    out, n = [0], 0
    for c in range(b.nch):
        ic = b.ics[f * b.nch + c]
        short = int(ic["window_sequence"]) == 2
        glen = [1]
        if short:
            for i in range(7):
                if (int(ic["grouping"]) >> i) & 1:
                    glen[-1] += 1
                else:
                    glen.append(1)
        sw, msfb = (sws if short else swl), int(ic["max_sfb"])
        cb = b.cb[f * b.nch + c]
        for g, gl in enumerate(glen):
            for s in range(msfb):
                if cb[g * msfb + s] == 13:
                    n += gl * int(sw[s + 1] - sw[s])
                out.append(n)
    return out


def test_parser_truncated_frame_moves_state_as_far_as_the_reference_read():
    """A frame cut short anywhere: it is marked FRAME_EOS, the next frame parses to the same records,
    and the state that frame sees is the reference's after its EOSException -- every window shape
    whose bit was read (A/syntax/ICSInfo.java:90-91, CPE setCommonData :193-197) and the static PNS
    LCG advanced over the noise bands decodeSpectralData reached (A/syntax/ICStream.java:222-275):
    for every cut length, the next frame's first pns_state is the start state advanced by one of
    the frame's band-boundary noise prefix sums, never decreasing with the cut length; a shape
    switches from the previous frame's to this frame's once and stays."""
    p = N.synth_params(3, n_streams=1, frames_per_stream=8, pns_percent=35, sf_index=3)
    b = N.synth_batch(p)
    frames = O.write_frames(b, p.sf_index)
    cfg = N.make_cfg(sf_index=p.sf_index)
    k = next(f for f in range(2, 7) if noise_prefix(b, f)[-1] > 0 and
             (b.ics["window_shape"][2 * f:2 * f + 2] != b.ics["window_shape"][2 * f - 2:2 * f]).any())
    prefix = noise_prefix(b, k)
    s0 = int(b.ics["pns_state"][2 * k])
    states = {}
    x = s0
    for n in range(prefix[-1] + 1):
        states.setdefault(x, n)
        if n < prefix[-1]:
            x = (LCG_A * x + LCG_C) & 0xFFFFFFFF
    assert int(b.ics["pns_state"][2 * k + 2]) == x  # the synthetic chain: frame k consumed whole
    full = N.Parser(cfg)
    full.pns_state = int(b.ics["pns_state"][0])
    ref = full.parse(frames[:k + 2])
    last_n, switched, seen = 0, [False, False], set()
    for cut in range(1, len(frames[k])):
        P = N.Parser(cfg)
        P.pns_state = int(b.ics["pns_state"][0])
        got = P.parse(frames[:k] + [frames[k][:cut], frames[k + 1]], drop_eos=True)
        assert np.flatnonzero(got.frame_status).tolist() == [k], cut
        assert not got.q[2 * k:2 * k + 2].any()
        for f in ("q", "sf", "cb"):
            assert (getattr(got, f)[2 * k + 2:] == getattr(ref, f)[2 * k + 2:]).all(), (cut, f)
        st = int(got.ics["pns_state"][2 * k + 2])
        assert st in states and states[st] in prefix, (cut, st)
        assert states[st] >= last_n, cut
        last_n = states[st]
        seen.add(last_n)
        for c in range(2):
            sp = int(got.ics["window_shape_prev"][2 * k + 2 + c])
            old, new = int(b.ics["window_shape"][2 * k - 2 + c]), int(b.ics["window_shape"][2 * k + c])
            assert sp in (old, new), (cut, c)
            if old != new:
                if switched[c]:
                    assert sp == new, (cut, c)
                switched[c] = sp == new
    assert len(seen) > 2, "no cut ended between noise bands"
    # a one-byte frame ends before any ICSInfo: nothing moved
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    got = P.parse(frames[:k] + [frames[k][:1], frames[k + 1]], drop_eos=True)
    assert int(got.ics["pns_state"][2 * k + 2]) == s0
    assert (got.ics["window_shape_prev"][2 * k + 2:2 * k + 4] == b.ics["window_shape"][2 * k - 2:2 * k]).all()
    # the last cut before the full frame has read every band
    assert last_n == prefix[-1] and all(switched[c] or b.ics["window_shape"][2 * k - 2 + c] == b.ics["window_shape"][2 * k + c]
                                        for c in range(2))


# ------------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------------

def _gpu_vs_oracle(cfg, b, flags, decode_batch=None):
    st = b.frame_status
    want = (decode_batch or oracle_pcm)(cfg, b, flags)
    nsl = int(b.stream_slot.max()) + 1
    out = np.full(want.shape, 0xA5, np.uint8)  # sentinel: dropped rows must keep it
    with N.Context(cfg, nsl) as ctx:
        ctx.decode(b, flags, out=out)
    assert (out[st == 1] == 0xA5).all(), "a dropped frame's PCM slot was written"
    assert (out[st == 0] == want[st == 0]).all(), np.flatnonzero((out != want).any(1) & (st == 0))[:8]


@pytest.mark.gpu
@pytest.mark.parametrize("config,streams,fps", [(2, 6, 40), (3, 6, 40), (4, 4, 24), (5, 4, 24)])
def test_gpu_dropped_frames_match_the_restatement(config, streams, fps):
    p = N.synth_params(config, n_streams=streams, frames_per_stream=fps)
    b = N.synth_batch(p)
    b.frame_status = drop_pattern(b)
    no_header_before_first_sbr(b, b.frame_status)
    _gpu_vs_oracle(N.cfg_for(p), b, N.PCM_BIG_ENDIAN)


@pytest.mark.gpu
def test_gpu_dropped_frames_mono_and_float32():
    p = N.synth_params(3, n_streams=3, frames_per_stream=30, channel_config=1)
    b = N.synth_batch(p)
    b.frame_status = drop_pattern(b)
    _gpu_vs_oracle(N.cfg_for(p), b, N.PCM_FLOAT32)


@pytest.mark.gpu
def test_gpu_dropped_frames_multichannel_and_coupling():
    from tests.test_cce import coupled_batch
    from tests.test_multichannel import mc_synth
    b = mc_synth(6, n_streams=3, fps=20, seed=4)
    b.frame_status = drop_pattern(b)
    cfg = N.make_cfg(channel_config=6)

    def mc_oracle(cfg, b, flags):
        return O.decode_batch_mc(3, b, N.MC_ELEMENTS[6], flags, threads=4)
    _gpu_vs_oracle(cfg, b, N.PCM_BIG_ENDIAN, mc_oracle)
    c = coupled_batch(2, n_streams=4, fps=20, seed=8)
    c.frame_status = drop_pattern(c)
    _gpu_vs_oracle(N.make_cfg(channel_config=2), c, N.PCM_BIG_ENDIAN)


@pytest.mark.gpu
def test_gpu_large_batch_dropped_frames_host_pieces():
    """A batch big enough for the piece pipeline of the host entry (>= 8192 frames)."""
    p = N.synth_params(2, n_streams=64, frames_per_stream=160)
    b = N.synth_batch(p)
    st = np.zeros(b.n_frames, np.uint8)
    st[np.random.default_rng(3).choice(b.n_frames, 40, replace=False)] = N.FRAME_EOS
    b.frame_status = st
    cfg = N.cfg_for(p)
    want = oracle_pcm(cfg, b, N.PCM_BIG_ENDIAN, threads=16)
    out = np.full((b.n_frames, N.pcm_frame_bytes(0)), 0x5A, np.uint8)
    with N.Context(cfg, 64) as ctx:
        ctx.decode(b, N.PCM_BIG_ENDIAN, out=out)
    assert (out[st == 1] == 0x5A).all()
    assert (out[st == 0] == want[st == 0]).all()


@pytest.mark.gpu
def test_gpu_dropped_frames_device_entry_and_errors():
    import torch
    p = N.synth_params(2, n_streams=4, frames_per_stream=30)
    b = N.synth_batch(p)
    b.frame_status = drop_pattern(b)
    cfg = N.cfg_for(p)
    want = oracle_pcm(cfg, b, N.PCM_BIG_ENDIAN)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).reshape(-1).view(np.uint8)).to(dev)
    d = {k: t(getattr(b, k)) for k in ("q", "sf", "cb", "ics", "ms_used")}
    ptr = {k: v.data_ptr() for k, v in d.items()}
    nb = N.pcm_frame_bytes(0)
    pcm = torch.full((b.n_frames * nb,), 0x33, dtype=torch.uint8, device=dev)
    st = b.frame_status
    with N.Context(cfg, 4) as ctx:
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), N.PCM_BIG_ENDIAN)
        ctx.wait()
        got = pcm.cpu().numpy().reshape(b.n_frames, nb)
        assert (got[st == 1] == 0x33).all() and (got[st == 0] == want[st == 0]).all()
        # every frame dropped: nothing written, no state moved
        b2 = N.synth_batch(p)
        b2.frame_status = np.ones(b2.n_frames, np.uint8)
        out = np.full((b2.n_frames, nb), 7, np.uint8)
        ctx.decode(b2, N.PCM_BIG_ENDIAN, out=out)
        assert (out == 7).all()
        # an unknown status value is refused
        b2.frame_status = np.full(b2.n_frames, 2, np.uint8)
        with pytest.raises(N.JaadError) as e:
            ctx.decode(b2, N.PCM_BIG_ENDIAN)
        assert e.value.status == N.ERR_INVALID_ARG
        # a bad side-info record in a later segment: refused before anything decodes
        b3 = N.synth_batch(p)
        st3 = np.zeros(b3.n_frames, np.uint8)
        st3[10] = N.FRAME_EOS
        b3.frame_status = st3
        b3.ics["max_sfb"][2 * 50] = 60
        before = ctx.state_export(0)
        with pytest.raises(N.JaadError) as e:
            ctx.decode(b3, N.PCM_BIG_ENDIAN)
        assert e.value.status == N.ERR_BITSTREAM
        assert (ctx.state_export(0) == before).all()


@pytest.mark.gpu
def test_decode_frames_drops_a_truncated_frame_per_frame():
    """frame k of a 40-frame decodeFrames batch is truncated; the other 39 equal the
    per-frame decode with frame k dropped, and buffer k keeps what it held (here: frame k-1's PCM,
    as a reused SampleBuffer would)."""
    from jaadec_amd.decoder import Decoder, SampleBuffer
    p = N.synth_params(3, n_streams=1, frames_per_stream=40, pns_percent=10)
    b = N.synth_batch(p)
    frames = O.write_frames(b, p.sf_index)
    k = 17
    bad = list(frames)
    bad[k] = frames[k][:len(frames[k]) // 2]
    # the records and the state the frames after k see (the parser moves the window shapes and
    # the PNS LCG as far as the reference's reads got: test_parser_truncated_frame_moves_state_...)
    P = N.Parser(N.make_cfg(sf_index=p.sf_index))
    P.pns_state = int(b.ics["pns_state"][0])
    pb = P.parse(bad, drop_eos=True)
    P.close()
    assert np.flatnonzero(pb.frame_status).tolist() == [k]
    want = oracle_pcm(N.make_cfg(sf_index=p.sf_index), pb, N.PCM_BIG_ENDIAN)
    dec = Decoder.create(bytes([0x11, 0x90]))
    dec._parse([])
    dec._parser.pns_state = int(b.ics["pns_state"][0])
    bufs = [SampleBuffer() for _ in range(40)]
    bufs[k]._set(want[k - 1].tobytes(), 48000)
    dec.decodeFrames(bad, bufs)
    assert dec.frames == 40
    for i, buf in enumerate(bufs):
        assert buf.getData() == (want[k - 1] if i == k else want[i]).tobytes(), i
    # the stream goes on from frame k+1's state: frame k re-sent whole is the next frame
    dec.close()


@pytest.mark.gpu
def test_jni_frame_status_and_state_export_import():
    """nativeDecode's frameStatus buffer, and nativeStateExport/Import (seek/resume) through the
    mock JNIEnv: a stream decoded in two calls with its state exported, the slot reset and the
    state imported in between equals one call."""
    import ctypes as C
    from tests.test_jni_glue import AAC_EXC, PFX, _buf, _exception, _lib
    L = _lib()
    env = L.jni_mock_env()
    p = N.synth_params(2, n_streams=2, frames_per_stream=24)
    b = N.synth_batch(p)
    st = drop_pattern(b)
    b.frame_status = st
    cfg = N.cfg_for(p)
    want = oracle_pcm(cfg, b, N.PCM_BIG_ENDIAN)
    h = getattr(L, PFX + "nativeCreate")(env, None, 3, 2, 0, 0, 0, 0, 2, 0)
    assert h and _exception(L) is None
    decode = getattr(L, PFX + "nativeDecode")
    try:
        keep = []
        out = np.zeros_like(want)
        args = [_buf(x, keep) for x in (b.stream_slot, b.frame_begin, b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, None,
                                         out)]
        decode(env, None, h, b.n_frames, 2, 2, *args, N.PCM_BIG_ENDIAN, _buf(st, keep))
        assert _exception(L) is None
        assert (out[st == 0] == want[st == 0]).all() and not out[st == 1].any()
        # a status buffer shorter than the batch is refused
        short = st[:-1].copy()
        decode(env, None, h, b.n_frames, 2, 2, *args, N.PCM_BIG_ENDIAN, _buf(short, keep))
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
        # seek/resume: frames [0, 12) of both streams, export, reset, import, frames [12, 24)
        b.frame_status = None
        full = oracle_pcm(cfg, b, N.PCM_BIG_ENDIAN)
        a1, a2 = b.split_frames(12)
        n = getattr(L, PFX + "nativeStateBytes")(env, None, h)
        assert n > 0 and _exception(L) is None
        for slot in range(2):
            getattr(L, PFX + "nativeReset")(env, None, h, slot)
        o1 = np.zeros((a1.n_frames, want.shape[1]), np.uint8)
        decode(env, None, h, a1.n_frames, 2, 2, *[_buf(x, keep) for x in (a1.stream_slot, a1.frame_begin, a1.q, a1.sf,
                                                                         a1.cb, a1.ics, a1.ms_used, a1.tns, None, o1)],
               N.PCM_BIG_ENDIAN, None)
        assert _exception(L) is None
        blobs = [np.zeros(n, np.uint8) for _ in range(2)]
        for slot in range(2):
            getattr(L, PFX + "nativeStateExport")(env, None, h, slot, _buf(blobs[slot], keep))
            assert _exception(L) is None
            getattr(L, PFX + "nativeReset")(env, None, h, slot)
        small = np.zeros(n - 1, np.uint8)
        getattr(L, PFX + "nativeStateImport")(env, None, h, 0, _buf(small, keep))
        cls, msg = _exception(L)
        assert cls == AAC_EXC and N.strerror(N.ERR_INVALID_ARG) in msg
        for slot in range(2):
            getattr(L, PFX + "nativeStateImport")(env, None, h, slot, _buf(blobs[slot], keep))
            assert _exception(L) is None
        o2 = np.zeros((a2.n_frames, want.shape[1]), np.uint8)
        decode(env, None, h, a2.n_frames, 2, 2, *[_buf(x, keep) for x in (a2.stream_slot, a2.frame_begin, a2.q, a2.sf,
                                                                         a2.cb, a2.ics, a2.ms_used, a2.tns, None, o2)],
               N.PCM_BIG_ENDIAN, None)
        assert _exception(L) is None
        fb = b.frame_begin
        for r in range(2):
            assert (o1[12 * r:12 * r + 12] == full[fb[r]:fb[r] + 12]).all()
            assert (o2[12 * r:12 * r + 12] == full[fb[r] + 12:fb[r + 1]]).all()
        del C
    finally:
        getattr(L, PFX + "nativeDestroy")(env, None, h)


@pytest.mark.gpu
def test_gpu_c2_batch_with_one_dropped_frame_per_stream_in_one_call():
    """the whole 65 536-frame C2 batch with one frame of every stream dropped decodes
    in ONE call (the planner walks the kept frames; no sub-batches), bit-exact against the
    restatement through the host and the device entry, and the device entry takes no more than
    1.1x the clean batch's time (same inputs, alternating blocks after a warm-up)."""
    import time
    import torch
    p = N.synth_params(2)
    b = N.synth_batch(p)
    rng = np.random.default_rng(11)
    fb = b.frame_begin
    st = np.zeros(b.n_frames, np.uint8)
    for r in range(len(b.stream_slot)):
        st[int(fb[r]) + int(rng.integers(0, int(fb[r + 1] - fb[r])))] = N.FRAME_EOS
    cfg = N.cfg_for(p)
    nsl = int(b.stream_slot.max()) + 1
    b.frame_status = st
    want = oracle_pcm(cfg, b, N.PCM_BIG_ENDIAN, threads=16)
    out = np.full(want.shape, 0x3C, np.uint8)
    with N.Context(cfg, nsl) as ctx:
        ctx.decode(b, N.PCM_BIG_ENDIAN, out=out)
    assert (out[st == 1] == 0x3C).all()
    assert (out[st == 0] == want[st == 0]).all()
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).reshape(-1).view(np.uint8)).to(dev)
    d = {k: t(getattr(b, k)) for k in ("q", "sf", "cb", "ics", "ms_used")}
    ptr = {k: v.data_ptr() for k, v in d.items()}
    ptr["tns"] = None
    nb = N.pcm_frame_bytes(0)
    pcm = torch.full((b.n_frames * nb,), 0x3C, dtype=torch.uint8, device=dev)
    clean = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch)
    s = torch.cuda.Stream(dev)
    with N.Context(cfg, nsl) as ctx_d, N.Context(cfg, nsl) as ctx_c:
        ctx_d.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), N.PCM_BIG_ENDIAN, s.cuda_stream)
        torch.cuda.synchronize()
        got = pcm.cpu().numpy().reshape(b.n_frames, nb)
        assert (got[st == 1] == 0x3C).all() and (got[st == 0] == want[st == 0]).all()
        scratch = torch.empty_like(pcm)
        t_end = time.perf_counter() + 0.4  # past the GPU clock's load-onset transient
        while time.perf_counter() < t_end:
            for c, bb in ((ctx_d, b), (ctx_c, clean)):
                c.decode_device(ptr, bb, scratch.data_ptr(), scratch.numel(), N.PCM_BIG_ENDIAN, s.cuda_stream)
            torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        times = {"drop": [], "clean": []}
        for blk in range(6):
            for name, c, bb in (("drop", ctx_d, b), ("clean", ctx_c, clean))[::1 if blk % 2 == 0 else -1]:
                ev[0].record(s)
                for _ in range(10):
                    c.decode_device(ptr, bb, scratch.data_ptr(), scratch.numel(), N.PCM_BIG_ENDIAN, s.cuda_stream)
                ev[1].record(s)
                torch.cuda.synchronize()
                times[name].append(ev[0].elapsed_time(ev[1]) / 10)
    ratio = float(np.median(times["drop"]) / np.median(times["clean"]))
    print(f"dropped/clean device-entry time: {np.median(times['drop']):.4f} / {np.median(times['clean']):.4f} ms"
          f" = {ratio:.3f}")
    assert ratio <= 1.1, times
