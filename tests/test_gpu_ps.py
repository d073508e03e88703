"""GPU parity for parametric stereo (HE-AAC v2, C5): SCE core + SBR + PS through the C-ABI against
the C restatement (oracle/jaad_oracle_ps.c, pinned by tests/test_ps_oracle.py).  Bar: bit-exact
PCM and bit-exact float32 output."""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

from test_gpu_sbr import _assert_same, _decode_both, _edit

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_LITTLE_ENDIAN, N.PCM_FLOAT32])
def test_c5_ps(flags):
    p = N.synth_params(5, n_streams=3, frames_per_stream=18)
    b = N.synth_batch(p)
    got, want = _decode_both(p, b, flags)
    _assert_same(got, want, flags)


def _modes(iid_mode, icc_mode, rng):
    def fn(s):
        ps = s["ps"]
        ps["iid_mode"], ps["icc_mode"] = iid_mode, icc_mode
        steps = 15 if iid_mode >= 3 else 7
        ps["iid"][:] = np.clip(ps["iid"].astype(np.int32) * (2 if steps == 15 else 1)
                               + rng.integers(-1, 2, ps["iid"].shape), -steps, steps)
    return fn


@pytest.mark.parametrize("iid_mode,icc_mode", [(4, 1), (1, 4), (5, 3), (0, 5)])
def test_c5_fine_iid_and_type_b_mixing(iid_mode, icc_mode):
    p = N.synth_params(5, n_streams=2, frames_per_stream=14)
    b = _edit(N.synth_batch(p), _modes(iid_mode, icc_mode, np.random.default_rng(iid_mode * 7 + icc_mode)))
    got, want = _decode_both(p, b, N.PCM_FLOAT32)
    _assert_same(got, want, N.PCM_FLOAT32)


def _var_envelopes(s, rng):
    """1..5 envelopes with variable borders per frame (PSImpl.java:103-134 fix-ups keep them
    strictly increasing from 0 to 32)."""
    for f in range(len(s)):
        ps = s[f]["ps"]
        ne = int(rng.integers(1, 6))
        inner = np.sort(rng.choice(np.arange(1, 32), ne - 1, replace=False))
        ps["num_env"] = ne
        ps["border"][:] = 0
        ps["border"][:ne + 1] = [0, *inner.tolist(), 32]
        ps["iid"][:ne] = rng.integers(-7, 8, (ne, 34))
        ps["icc"][:ne] = rng.integers(0, 8, (ne, 34))


def test_c5_variable_envelopes_and_transients():
    p = N.synth_params(5, n_streams=2, frames_per_stream=16)
    rng = np.random.default_rng(3)
    b = _edit(N.synth_batch(p), lambda s: _var_envelopes(s, rng))
    got, want = _decode_both(p, b, N.PCM_FLOAT32)
    _assert_same(got, want, N.PCM_FLOAT32)


@pytest.mark.parametrize("nr", [11, 17])
def test_c5_ipd_opd_phase_rotation(nr):
    """PS extension: IPD/OPD phase history and complex H interpolation (A/ps/PSImpl.java:484-679),
    toggled on and off between frames so h_prev's imaginary parts persist through frames without it."""
    p = N.synth_params(5, n_streams=3, frames_per_stream=14)
    rng = np.random.default_rng(nr)

    def fn(s):
        ps = s["ps"]
        ps["nr_ipdopd_par"] = np.where(rng.random(len(s)) < 0.8, nr, 0)
        ps["ipd"][:] = rng.integers(0, 8, ps["ipd"].shape)
        ps["opd"][:] = rng.integers(0, 8, ps["opd"].shape)
        _var_envelopes(s, rng)

    b = _edit(N.synth_batch(p), fn)
    got, want = _decode_both(p, b, N.PCM_FLOAT32)
    _assert_same(got, want, N.PCM_FLOAT32)
    cfg = N.cfg_for(p)
    first, second = b.split_frames(6)
    with N.Context(cfg, 3) as ctx:
        g = np.concatenate([ctx.decode(first, N.PCM_FLOAT32), ctx.decode(second, N.PCM_FLOAT32)])
    fb = b.frame_begin
    order = np.concatenate([np.arange(fb[r], fb[r] + 6) for r in range(3)] +
                           [np.arange(fb[r] + 6, fb[r + 1]) for r in range(3)])
    _assert_same(g, want[order], N.PCM_FLOAT32)


def test_c5_continuation_and_state_roundtrip():
    p = N.synth_params(5, n_streams=3, frames_per_stream=16)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(3), N.PCM_FLOAT32)
    first, second = b.split_frames(7)
    with N.Context(cfg, 3) as ctx:
        g1 = ctx.decode(first, N.PCM_FLOAT32)
        blob = ctx.state_export(2)
        with N.Context(cfg, 3) as ctx2:
            ctx2.state_import(2, blob)
            g2b = ctx2.decode(second.select_runs([2]), N.PCM_FLOAT32)
        g2 = ctx.decode(second, N.PCM_FLOAT32)
    fb = b.frame_begin
    for r in range(3):
        _assert_same(g1[7 * r:7 * (r + 1)], want[fb[r]:fb[r] + 7], N.PCM_FLOAT32)
        _assert_same(g2[9 * r:9 * (r + 1)], want[fb[r] + 7:fb[r + 1]], N.PCM_FLOAT32)
    _assert_same(g2b, want[fb[2] + 7:fb[3]], N.PCM_FLOAT32)


def test_c5_single_frame_calls():
    p = N.synth_params(5, n_streams=2, frames_per_stream=6)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(2), N.PCM_BIG_ENDIAN)
    out, rest = [], b
    with N.Context(cfg, 2) as ctx:
        for _ in range(6):
            one, rest = rest.split_frames(1)
            out.append(ctx.decode(one, N.PCM_BIG_ENDIAN))
    fb = b.frame_begin
    for k in range(6):
        for r in range(2):
            assert np.array_equal(out[k][r], want[fb[r] + k])


def _ps_gaps(s, pattern):
    """ps_present per frame of each stream from `pattern` (1 = PS data)."""
    for f in range(len(s)):
        s[f]["ps_present"] = pattern[f % len(pattern)]


@pytest.mark.parametrize("pattern", [
    (0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1),  # stream starts without PS: mono copies, then PS opens fresh
    (1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 1),  # PS data missing in some frames: mono copies, PS state waits
    (0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0),  # never any PS data
])
@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_FLOAT32])
def test_c5_frames_without_ps_data(pattern, flags):
    """SBR1.process without PS data (A/sbr/SBR1.java:75-81, isPSUsed :136): the mono SBR output is
    copied to the right channel, PSImpl and qmfs1 keep their state for the next PS frame."""
    p = N.synth_params(5, n_streams=3, frames_per_stream=12)
    b = _edit(N.synth_batch(p), lambda s: _ps_gaps(s, pattern))
    got, want = _decode_both(p, b, flags)
    _assert_same(got, want, flags)


def test_c5_ps_gaps_across_calls():
    """A PS gap spanning a call boundary: the next call's first PS frame takes the filterbank
    history and the right synthesis ring from the slot state."""
    p = N.synth_params(5, n_streams=2, frames_per_stream=10)
    pattern = (1, 1, 1, 0, 0, 0, 0, 1, 1, 0)
    b = _edit(N.synth_batch(p), lambda s: _ps_gaps(s, pattern))
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(2), N.PCM_BIG_ENDIAN)
    out, rest = [], b
    with N.Context(cfg, 2) as ctx:
        for n in (4, 2, 4):
            part, rest = rest.split_frames(n)
            out.append(ctx.decode(part, N.PCM_BIG_ENDIAN))
    fb = b.frame_begin
    k0 = 0
    for part, n in zip(out, (4, 2, 4)):
        for r in range(2):
            for k in range(n):
                assert np.array_equal(part[r * n + k], want[fb[r] + k0 + k]), (r, k0 + k)
        k0 += n


@pytest.mark.parametrize("name,fn,status", [
    ("bad_nr_ipdopd_par", lambda s: s["ps"].__setitem__("nr_ipdopd_par", 12), N.ERR_BITSTREAM),
    ("border_not_32", lambda s: s["ps"]["border"].__setitem__((slice(None), 1), 30), N.ERR_BITSTREAM),
    ("iid_out_of_range", lambda s: s["ps"]["iid"].__setitem__((slice(None), 0, 3), 9), N.ERR_BITSTREAM),
])
def test_c5_rejects_what_the_gpu_path_does_not_decode(name, fn, status):
    p = N.synth_params(5, n_streams=1, frames_per_stream=3)
    b = N.synth_batch(p)
    s = b.sbr.copy()
    s["ps"]["num_env"] = 1
    s["ps"]["border"][:, :2] = [0, 32]
    fn(s)
    b = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, s)
    with N.Context(N.cfg_for(p), 1) as ctx:
        with pytest.raises(N.JaadError) as e:
            ctx.decode(b, N.PCM_BIG_ENDIAN)
    assert e.value.status == status


@pytest.mark.slow
def test_c5_full_shard_bitexact():
    """One GPU's share of the 262 144-frame C5 job (32 768 frames = 256 streams x 128, the bench's
    per-GPU workload) against the restatement."""
    p = N.synth_params(5, n_streams=256, frames_per_stream=128)
    got, want = _decode_both(p, N.synth_batch(p), N.PCM_BIG_ENDIAN)
    _assert_same(got, want, N.PCM_BIG_ENDIAN)
