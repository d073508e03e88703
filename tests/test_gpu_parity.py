"""GPU parity: the HIP path (through the C-ABI) against the C restatement of the reference.

The bar is bit-exact PCM (|delta| = 0, stricter than the +-1 LSB of BASELINE.json): the kernels
evaluate the reference's binary32 arithmetic in the same order without contraction.  Float32
output mode (samples before Math.round) is compared bit-exactly as well.
"""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _run_both(p, cfg, flags=N.PCM_BIG_ENDIAN, threads=8):
    b = N.synth_batch(p)
    n_slots = int(b.stream_slot.max()) + 1
    with N.Context(cfg, n_slots) as ctx:
        got = ctx.decode(b, flags)
    want = O.decode_batch(cfg, b, O.Streams(n_slots), flags, threads=threads)
    return b, got, want


def _assert_pcm_equal(got, want, flags=N.PCM_BIG_ENDIAN):
    if flags & N.PCM_FLOAT32:
        g, w = got.view(np.float32), want.view(np.float32)
        bad = np.flatnonzero(g.view(np.uint32) != w.view(np.uint32))
        assert bad.size == 0, f"{bad.size} float samples differ, first at {bad[:5]}: {g.reshape(-1)[bad[:5]]} vs {w.reshape(-1)[bad[:5]]}"
        return
    dt = ">i2" if not (flags & N.PCM_LITTLE_ENDIAN) else "<i2"
    g = got.view(dt).astype(np.int32)
    w = want.view(dt).astype(np.int32)
    d = np.abs(g - w)
    assert d.max() <= 1, f"max |delta| {d.max()} LSB"
    assert (d != 0).sum() == 0, f"{(d != 0).sum()} samples off by one"


@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_LITTLE_ENDIAN, N.PCM_FLOAT32])
def test_c2_long_windows(flags):
    p = N.synth_params(2, n_streams=6, frames_per_stream=21)  # 21 frames: 3 chunks, ragged tail
    _, got, want = _run_both(p, N.make_cfg(), flags)
    _assert_pcm_equal(got, want, flags)


def test_c3_window_switching_tns_compat():
    p = N.synth_params(3, n_streams=8, frames_per_stream=40)
    b, got, want = _run_both(p, N.make_cfg(), N.PCM_FLOAT32)
    seqs = np.bincount(b.ics["window_sequence"], minlength=4)
    assert (seqs > 0).all(), seqs  # every window sequence exercised
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)


def test_c3_tns_spec_mode():
    p = N.synth_params(3, n_streams=6, frames_per_stream=24)
    cfg = N.make_cfg(tns_mode=N.TNS_SPEC)
    _, got, want = _run_both(p, cfg, N.PCM_FLOAT32)
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)


@pytest.mark.parametrize("cfg_id", [2, 3])
def test_escaped_values_beyond_the_lds_iq_head(cfg_id):
    """|q| in [1024, 8191] (IQ_TABLE entries past the kernel's 2 x 1024-entry LDS head, read from
    the global table; A/syntax/ICStream.java:258-271), scattered over every band -- spectral,
    zero, noise and intensity bands and bins past max_sfb, where the reference never reads q."""
    p = N.synth_params(cfg_id, n_streams=4, frames_per_stream=20, pns_percent=6, is_percent=10)
    b = N.synth_batch(p)
    rng = np.random.default_rng(11)
    flat = b.q.reshape(-1)
    pick = rng.choice(flat.size, flat.size // 200, replace=False)
    mag = rng.integers(1024, 8192, pick.size)
    flat[pick] = np.where(rng.integers(0, 2, pick.size) == 1, mag, -mag).astype(np.int16)
    n_slots = int(b.stream_slot.max()) + 1
    with N.Context(N.make_cfg(), n_slots) as ctx:
        got = ctx.decode(b, N.PCM_FLOAT32)
    want = O.decode_batch(N.make_cfg(), b, O.Streams(n_slots), N.PCM_FLOAT32)
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)


def test_pns_and_intensity():
    p = N.synth_params(3, n_streams=5, frames_per_stream=20, pns_percent=8, is_percent=15)
    b, got, want = _run_both(p, N.make_cfg(), N.PCM_FLOAT32)
    assert (b.ics["flags"] & N.ICS_HAS_PNS).any() and (b.ics["flags"] & N.ICS_HAS_IS).any()
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)


def test_ms_all_ones_and_independent_windows():
    p = N.synth_params(3, n_streams=4, frames_per_stream=18, ms_mode=2)
    _, got, want = _run_both(p, N.make_cfg(), N.PCM_FLOAT32)
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)
    p = N.synth_params(3, n_streams=4, frames_per_stream=18, common_window=0, ms_mode=0, is_percent=10)
    _, got, want = _run_both(p, N.make_cfg(), N.PCM_FLOAT32)
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)


def test_mono_sce_duplicated_to_stereo():
    p = N.synth_params(1, n_streams=3, frames_per_stream=19, window_switching=1, pns_percent=5)
    cfg = N.make_cfg(sf_index=4, channel_config=1)
    _, got, want = _run_both(p, cfg, N.PCM_BIG_ENDIAN)
    _assert_pcm_equal(got, want)
    s = got.view(">i2").reshape(got.shape[0], 1024, 2)
    assert (s[..., 0] == s[..., 1]).all()


@pytest.mark.parametrize("sf_index", [0, 5, 6, 8, 11])
def test_other_sample_rates(sf_index):
    p = N.synth_params(3, n_streams=3, frames_per_stream=12, sf_index=sf_index)
    _, got, want = _run_both(p, N.make_cfg(sf_index=sf_index), N.PCM_FLOAT32)
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)


def test_continuation_across_calls_and_state_roundtrip():
    p = N.synth_params(3, n_streams=4, frames_per_stream=30)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    want = O.decode_batch(cfg, b, O.Streams(4), N.PCM_FLOAT32)
    first, second = b.split_frames(13)
    with N.Context(cfg, 4) as ctx:
        g1 = ctx.decode(first, N.PCM_FLOAT32)
        saved = [ctx.state_export(s) for s in range(4)]
        g2 = ctx.decode(second, N.PCM_FLOAT32)
        # rewind: import the saved state and decode the second half again
        for s in range(4):
            ctx.state_import(s, saved[s])
        g2b = ctx.decode(second, N.PCM_FLOAT32)
    got = np.empty_like(want)
    fb = b.frame_begin
    i1 = i2 = 0
    for r in range(4):
        n = int(fb[r + 1] - fb[r])
        a = min(13, n)
        got[fb[r]:fb[r] + a] = g1[i1:i1 + a]
        got[fb[r] + a:fb[r + 1]] = g2[i2:i2 + n - a]
        i1 += a
        i2 += n - a
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)
    assert (g2 == g2b).all()


def test_ragged_runs_and_subset_of_slots():
    p = N.synth_params(2, n_streams=6, frames_per_stream=17)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    sub = b.select_runs([4, 1, 3])  # slots 4,1,3 only; others untouched
    lens = [1, 9, 17]
    frames, begin = [], [0]
    for r, L in zip(range(3), lens):
        f0 = int(sub.frame_begin[r])
        frames.append(np.arange(f0, f0 + L))
        begin.append(begin[-1] + L)
    frames = np.concatenate(frames)
    cfr = (frames[:, None] * 2 + np.arange(2)).reshape(-1)
    rag = N.Batch(sub.q[cfr].copy(), sub.sf[cfr].copy(), sub.cb[cfr].copy(), sub.ics[cfr].copy(),
                  sub.ms_used[frames].copy(), None, sub.stream_slot.copy(), np.array(begin, np.uint32), 2)
    with N.Context(cfg, 6) as ctx:
        got = ctx.decode(rag, N.PCM_FLOAT32)
        st_other = ctx.state_export(0)
    want = O.decode_batch(cfg, rag, O.Streams(6), N.PCM_FLOAT32)
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)
    assert (st_other[:-16] == 0).all()  # (the blob's 16-byte trailer names its layout)


def test_bitstream_errors_are_reported():
    p = N.synth_params(2, n_streams=1, frames_per_stream=2)
    b = N.synth_batch(p)
    b.ics["max_sfb"][0] = 60  # > 49 bands at 48 kHz
    with N.Context(N.make_cfg(), 1) as ctx:
        with pytest.raises(N.JaadError) as e:
            ctx.decode(b)
        assert e.value.status == N.ERR_BITSTREAM


@pytest.mark.slow
def test_c2_full_batch_bitexact():
    """The whole 65 536-frame C2 batch (the bench workload) against the restatement."""
    p = N.synth_params(2)
    _, got, want = _run_both(p, N.make_cfg(), N.PCM_BIG_ENDIAN, threads=16)
    _assert_pcm_equal(got, want)


@pytest.mark.slow
def test_c3_full_batch_bitexact():
    """The whole 65 536-frame C3 batch (LONG/START/SHORT/STOP + TNS data, compat mode) in float32
    output (samples before Math.round) against the restatement."""
    p = N.synth_params(3)
    b, got, want = _run_both(p, N.make_cfg(), N.PCM_FLOAT32, threads=16)
    seqs = np.bincount(b.ics["window_sequence"], minlength=4)
    assert (seqs > 0).all(), seqs
    assert b.tns is not None and (b.tns["n_filters"] > 0).mean() > 0.3  # TNS data in ~50 % of ch-frames
    _assert_pcm_equal(got, want, N.PCM_FLOAT32)


@pytest.mark.parametrize("cfg_id", [2, 3])
def test_float32_output_stays_inside_its_frames(cfg_id, monkeypatch):
    """the float32 PCM form goes through a buffer resource over exactly its frame, as
    the int16 form does.  Device entry into a buffer with guard frames on both sides: chunks that
    re-decode a prefix frame (runs of 40 frames: several chunks each) leave the guards untouched,
    and the rows equal the host entry's."""
    import torch
    p = N.synth_params(cfg_id, n_streams=8, frames_per_stream=40)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    with N.Context(cfg, 8) as ctx:
        want = ctx.decode(b, N.PCM_FLOAT32)
    dev = torch.device("cuda", 0)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
    d = {k: t(getattr(b, k)) for k in ("q", "sf", "cb", "ics", "ms_used", "tns")}
    ptr = {k: (v.data_ptr() if v is not None else None) for k, v in d.items()}
    nb = 8192
    guard = 2
    pcm = torch.full(((b.n_frames + 2 * guard) * nb,), 0x7F, dtype=torch.uint8, device=dev)
    monkeypatch.setenv("JAAD_CHUNK_FRAMES", "9")  # (read at context creation) prefix frames in every run
    with N.Context(cfg, 8) as ctx:
        ctx.decode_device(ptr, b, pcm.data_ptr() + guard * nb, b.n_frames * nb, N.PCM_FLOAT32)
        ctx.wait()
    host = pcm.cpu().numpy().reshape(-1, nb)
    assert (host[:guard] == 0x7F).all() and (host[-guard:] == 0x7F).all()
    assert (host[guard:-guard] == want).all()


def test_state_blob_names_its_layout():
    """a state blob ends with a trailer (magic, layout version, context kind, payload
    bytes); an import checks it, so a blob with another version or written by another kind of
    context (here: HE-AAC with a downsampled vs an upsampled synthesis, same size) is refused and
    the slot keeps its state."""
    p = N.synth_params(2, n_streams=2, frames_per_stream=9)
    b = N.synth_batch(p)
    with N.Context(N.make_cfg(), 2) as ctx:
        ctx.decode(b)
        blob = ctx.state_export(0)
        before = ctx.state_export(1)
        magic, version, kind, payload = np.frombuffer(blob[-16:].tobytes(), "<u4")
        assert magic == 0x4441414A and payload == len(blob) - 16
        for k in range(4):  # each trailer word in turn
            bad = blob.copy()
            bad[-16 + 4 * k] ^= 1
            with pytest.raises(N.JaadError) as e:
                ctx.state_import(1, bad)
            assert e.value.status == N.ERR_INVALID_ARG
            assert (ctx.state_export(1) == before).all()
        ctx.state_import(1, blob)
        assert (ctx.state_export(1) == blob).all()
    up = N.make_cfg(sf_index=6, sbr=True)
    down = N.make_cfg(sf_index=6, sbr=True, down=True)
    with N.Context(up, 1) as a, N.Context(down, 1) as d:
        blob = a.state_export(0)
        assert len(blob) == len(d.state_export(0))
        with pytest.raises(N.JaadError) as e:
            d.state_import(0, blob)
        assert e.value.status == N.ERR_INVALID_ARG
