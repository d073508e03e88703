"""Failure atomicity and call ordering of the C-ABI (jaad_capi.cpp), on the GPU.

* a rejected batch must not disturb the cached chunk plan or any stream state;
* a rejected SBR call must leave every slot's host SBR state as it found it (a retry of the good
  batch is then bit-exact against the restatement);
* device-path calls queued on different HIP streams are ordered after each other, and the
  state_* entry points wait for them;
* the device path clamps malformed side info instead of reading or writing out of bounds.
"""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _halves(b, cut):
    """Both halves have the same run layout when every run has 2*cut frames."""
    first, second = b.split_frames(cut)
    assert np.array_equal(first.frame_begin, second.frame_begin)
    return first, second


def _dup_slot(b):
    bad = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot.copy(), b.frame_begin, b.nch, b.sbr)
    bad.stream_slot[-1] = bad.stream_slot[0]
    return bad


def test_rejected_batch_keeps_plan_and_state():
    p = N.synth_params(2, n_streams=4, frames_per_stream=26)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    want = O.decode_batch(cfg, b, O.Streams(4), N.PCM_FLOAT32)
    first, second = _halves(b, 13)
    with N.Context(cfg, 4) as ctx:
        g1 = ctx.decode(first, N.PCM_FLOAT32)
        # a duplicate slot is rejected while planning; so is a differently laid out batch
        with pytest.raises(N.JaadError) as e:
            ctx.decode(_dup_slot(second), N.PCM_FLOAT32)
        assert e.value.status == N.ERR_INVALID_ARG
        g2 = ctx.decode(second, N.PCM_FLOAT32)  # same layout as `first`: the cached plan
    fb = b.frame_begin
    for r in range(4):
        assert np.array_equal(g1[13 * r:13 * (r + 1)], want[fb[r]:fb[r] + 13])
        assert np.array_equal(g2[13 * r:13 * (r + 1)], want[fb[r] + 13:fb[r + 1]])


def test_rejected_sbr_call_is_atomic_and_retry_is_bitexact():
    p = N.synth_params(4, n_streams=3, frames_per_stream=16)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(3), N.PCM_BIG_ENDIAN)
    first, second = _halves(b, 8)
    s = second.sbr.copy()
    s["ch"]["L_E"][-3, 0] = 9  # run 2, frame 5 of the call: runs 0, 1 and part of 2 were built
    bad = N.Batch(second.q, second.sf, second.cb, second.ics, second.ms_used, second.tns, second.stream_slot,
                  second.frame_begin, second.nch, s)
    with N.Context(cfg, 3) as ctx:
        g1 = ctx.decode(first, N.PCM_BIG_ENDIAN)
        with pytest.raises(N.JaadError) as e:
            ctx.decode(bad, N.PCM_BIG_ENDIAN)
        assert e.value.status == N.ERR_BITSTREAM
        g2 = ctx.decode(second, N.PCM_BIG_ENDIAN)
    fb = b.frame_begin
    for r in range(3):
        assert np.array_equal(g1[8 * r:8 * (r + 1)], want[fb[r]:fb[r] + 8]), r
        assert np.array_equal(g2[8 * r:8 * (r + 1)], want[fb[r] + 8:fb[r + 1]]), r


def _to_dev(torch, b, dev):
    keep = {k: torch.from_numpy(np.ascontiguousarray(getattr(b, k)).view(np.uint8).reshape(-1)).to(dev)
            for k in ("q", "sf", "cb", "ics", "ms_used")}
    return keep, {k: v.data_ptr() for k, v in keep.items()}


def test_device_calls_on_different_streams_are_ordered():
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    p = N.synth_params(3, n_streams=6, frames_per_stream=24)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    want = O.decode_batch(cfg, b, O.Streams(6), N.PCM_FLOAT32)
    # the second call has a different run layout (new chunk table) and runs on another stream
    first, second = b.split_frames(10)
    second = second.select_runs([5, 0, 3, 1, 4, 2])
    nb = N.pcm_frame_bytes(N.PCM_FLOAT32)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    k1, d1 = _to_dev(torch, first, dev)
    k2, d2 = _to_dev(torch, second, dev)
    o1 = torch.empty(first.n_frames * nb, dtype=torch.uint8, device=dev)
    o2 = torch.empty(second.n_frames * nb, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    with N.Context(cfg, 6) as ctx:
        ctx.decode_device(d1, first, o1.data_ptr(), o1.numel(), N.PCM_FLOAT32, sa.cuda_stream)
        ctx.decode_device(d2, second, o2.data_ptr(), o2.numel(), N.PCM_FLOAT32, sb.cuda_stream)
        st = [ctx.state_export(s) for s in range(6)]  # waits for both calls
        assert N.lib().jaad_wait(ctx.h) == 0
    torch.cuda.synchronize(dev)
    g1 = o1.cpu().numpy().reshape(first.n_frames, nb)
    g2 = o2.cpu().numpy().reshape(second.n_frames, nb)
    fb = b.frame_begin
    for r in range(6):
        assert np.array_equal(g1[10 * r:10 * (r + 1)], want[fb[r]:fb[r] + 10]), r
    for i, r in enumerate([5, 0, 3, 1, 4, 2]):
        assert np.array_equal(g2[14 * i:14 * (i + 1)], want[fb[r] + 10:fb[r + 1]]), r
    # the exported overlap is the one after the last frame of each stream
    with N.Context(cfg, 6) as ref:
        ref.decode(b, N.PCM_FLOAT32)
        for s in range(6):
            assert np.array_equal(st[s], ref.state_export(s)), s


def test_device_path_clamps_malformed_side_info():
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    p = N.synth_params(3, n_streams=2, frames_per_stream=8)
    b = N.synth_batch(p, with_tns=False)
    rng = np.random.default_rng(7)
    b.ics["max_sfb"][:] = 255
    b.ics["window_sequence"][::3] = 7
    b.ics["window_shape"][:] = 9
    b.ics["flags"][:] |= N.ICS_HAS_PNS | N.ICS_HAS_IS
    b.cb[:] = rng.integers(0, 256, b.cb.shape, dtype=np.uint8)
    b.sf[:] = rng.integers(0, 256, b.sf.shape, dtype=np.uint8)
    b.q[:] = rng.integers(-32768, 32767, b.q.shape, dtype=np.int16)
    cfg = N.make_cfg()
    with N.Context(cfg, 2) as ctx:
        with pytest.raises(N.JaadError) as e:  # the host path rejects it
            ctx.decode(b)
        assert e.value.status == N.ERR_BITSTREAM
        keep, d = _to_dev(torch, b, dev)
        out = torch.empty(b.n_frames * 4096, dtype=torch.uint8, device=dev)
        ctx.decode_device(d, b, out.data_ptr(), out.numel(), N.PCM_BIG_ENDIAN, None)
        assert N.lib().jaad_wait(ctx.h) == 0  # completed, no fault
        # the context stays usable: reset the slots and decode a good batch bit-exactly
        for s in range(2):
            ctx.state_reset(s)
        good = N.synth_batch(p)
        got = ctx.decode(good, N.PCM_FLOAT32)
    want = O.decode_batch(cfg, good, O.Streams(2), N.PCM_FLOAT32)
    assert np.array_equal(got, want)
