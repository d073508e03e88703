"""GPU parity for the SBR (HE-AAC v1) path: the HIP kernels through the C-ABI against the C
restatement of the reference's SBR (oracle/jaad_oracle_sbr.c).  Bar: bit-exact PCM and bit-exact
float32 output (SURVEY.md 8d allows |delta| <= 1 LSB / rel-RMS 1e-4; the kernels keep the Java
binary32 evaluation order, so no tolerance is needed)."""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _assert_same(got, want, flags):
    if flags & N.PCM_FLOAT32:
        g, w = got.view(np.uint32), want.view(np.uint32)
        bad = np.flatnonzero(g != w)
        gf, wf = got.view(np.float32).reshape(-1), want.view(np.float32).reshape(-1)
        assert bad.size == 0, f"{bad.size} float samples differ; first {bad[:4]}: {gf[bad[:4]]} vs {wf[bad[:4]]}"
    else:
        bad = np.flatnonzero(got.reshape(-1) != want.reshape(-1))
        assert bad.size == 0, f"{bad.size} PCM bytes differ, first at byte {bad[:4]}"


def _decode_both(p, b, flags, cfg=None):
    cfg = cfg or N.cfg_for(p)
    n = int(b.stream_slot.max()) + 1
    with N.Context(cfg, n) as ctx:
        got = ctx.decode(b, flags)
    want = O.decode_batch(cfg, b, O.Streams(n), flags, threads=8)
    return got, want


@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_LITTLE_ENDIAN, N.PCM_FLOAT32])
def test_c4_stereo(flags):
    # 40 frames per stream: chunks at 0 (state), 16 and 32 (recomputed prefix frames)
    p = N.synth_params(4, n_streams=4, frames_per_stream=40)
    b = N.synth_batch(p)
    got, want = _decode_both(p, b, flags)
    assert got.shape == (b.n_frames, (8192 if not flags & N.PCM_FLOAT32 else 16384))
    _assert_same(got, want, flags)


def test_c4_mono_sbr_duplicated():
    p = N.synth_params(4, n_streams=3, frames_per_stream=20, channel_config=1)
    b = N.synth_batch(p)
    got, want = _decode_both(p, b, N.PCM_FLOAT32)
    _assert_same(got, want, N.PCM_FLOAT32)


def _edit(b, fn):
    s = b.sbr.copy()
    fn(s)
    return N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, s)


@pytest.mark.parametrize("name,fn", [
    ("smoothing", lambda s: s["hdr"].__setitem__("smoothing_mode", 0)),
    ("no_interpol", lambda s: s["hdr"].__setitem__("interpol_freq", 0)),
    ("limiter0", lambda s: s["hdr"].__setitem__("limiter_bands", 0)),
    ("limiter3_gain0", lambda s: (s["hdr"].__setitem__("limiter_bands", 3), s["hdr"].__setitem__("limiter_gains", 0))),
    ("freq_scale0", lambda s: s["hdr"].__setitem__("freq_scale", 0)),
    ("freq_scale3_xover1", lambda s: (s["hdr"].__setitem__("freq_scale", 3), s["hdr"].__setitem__("xover_band", 1))),
    ("amp_res0", lambda s: s["hdr"].__setitem__("amp_res", 0)),
])
def test_c4_header_variants(name, fn):
    p = N.synth_params(4, n_streams=2, frames_per_stream=34)
    b = _edit(N.synth_batch(p), fn)
    got, want = _decode_both(p, b, N.PCM_FLOAT32)
    _assert_same(got, want, N.PCM_FLOAT32)


def _var_grids(s, rng):
    """Rewrite every second frame as a VARVAR / FIXVAR / VARFIX grid with 2..4 envelopes."""
    for f in range(1, len(s), 2):
        for c in range(2):
            ch = s[f]["ch"][c]
            if ch["L_E"] == 1:  # FIXFIX with one envelope coded 1.5 dB steps: back to 3 dB units
                ch["E"] //= 2
            cls = int(rng.integers(1, 4))
            L_E = int(rng.integers(2, 5))
            lead = 0 if cls == 1 else int(rng.integers(0, 3))
            trail = 16 if cls == 2 else 16 + int(rng.integers(0, 3))
            inner = np.sort(rng.choice(np.arange(lead + 1, trail), L_E - 1, replace=False))
            tE = [2 * lead] + [2 * int(x) for x in inner] + [2 * trail]
            ch["frame_class"], ch["L_E"], ch["L_Q"] = cls, L_E, 2
            ch["bs_pointer"] = int(rng.integers(0, L_E + 1))
            ch["t_E"][:] = 0
            ch["t_E"][:L_E + 1] = tE
            mid = max(1, min(L_E - 1, L_E // 2))
            ch["t_Q"][:] = [tE[0], tE[mid], tE[L_E]]
            ch["f"][:L_E] = rng.integers(0, 2, L_E)


def test_c4_variable_grids_and_sinusoids():
    p = N.synth_params(4, n_streams=2, frames_per_stream=36)
    b = N.synth_batch(p)
    rng = np.random.default_rng(7)
    b = _edit(b, lambda s: _var_grids(s, rng))
    assert (b.sbr["ch"]["frame_class"] > 0).any() and (b.sbr["ch"]["add_harmonic"] != 0).any()
    got, want = _decode_both(p, b, N.PCM_FLOAT32)
    _assert_same(got, want, N.PCM_FLOAT32)


def test_c4_continuation_and_state_roundtrip():
    p = N.synth_params(4, n_streams=3, frames_per_stream=30)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(3), N.PCM_BIG_ENDIAN)
    first, second = b.split_frames(13)
    with N.Context(cfg, 3) as ctx:
        g1 = ctx.decode(first, N.PCM_BIG_ENDIAN)
        blob = ctx.state_export(1)
        with N.Context(cfg, 3) as ctx2:  # resume stream 1 in another context
            ctx2.state_import(1, blob)
            g2b = ctx2.decode(second.select_runs([1]), N.PCM_BIG_ENDIAN)
        g2 = ctx.decode(second, N.PCM_BIG_ENDIAN)
    fb = b.frame_begin
    for r in range(3):
        assert np.array_equal(g1[13 * r:13 * (r + 1)], want[fb[r]:fb[r] + 13])
        assert np.array_equal(g2[17 * r:17 * (r + 1)], want[fb[r] + 13:fb[r + 1]])
    assert np.array_equal(g2b, want[fb[1] + 13:fb[2]])


def _header_changes(s, fps):
    """Mid-stream SBR header changes that move kx and M: xover_band 2 from frame 12 of each
    stream, start_freq 7 (k0 up) from frame 24.  Both shrink the band count, so the envelope data
    drawn for the first header stays valid."""
    f = np.arange(len(s)) % fps
    s["hdr"]["xover_band"][f >= 12] = 2
    s["hdr"]["start_freq"][f >= 24] = 7


@pytest.mark.parametrize("cfgid", [4, 5])
def test_header_change_moves_kx_across_calls(cfgid):
    """kx / M change inside a run and at a call boundary.  Where kx rises after a frame whose last
    envelope ended past slot 32, rows 2..7 of bands [kx_prev, kx) are frame f-1's adjusted high
    band (sbr_save_matrix): those frames (kSbrDep) run again in an HF fix pass on frame f-1's
    final carry rows; the call boundary hands them over through the slot state."""
    fps = 36
    p = N.synth_params(cfgid, n_streams=3, frames_per_stream=fps)
    rng = np.random.default_rng(11)
    b = _edit(N.synth_batch(p), lambda s: (_header_changes(s, fps), _var_grids(s, rng)))
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(3), N.PCM_FLOAT32, threads=8)
    first, second = b.split_frames(23)
    with N.Context(cfg, 3) as ctx:
        g1 = ctx.decode(first, N.PCM_FLOAT32)
        g2 = ctx.decode(second, N.PCM_FLOAT32)
    fb = b.frame_begin
    for r in range(3):
        _assert_same(g1[23 * r:23 * (r + 1)], want[fb[r]:fb[r] + 23], N.PCM_FLOAT32)
        _assert_same(g2[13 * r:13 * (r + 1)], want[fb[r] + 23:fb[r + 1]], N.PCM_FLOAT32)


@pytest.mark.parametrize("cfgid", [4, 5])
@pytest.mark.parametrize("direction", ["fall", "rise"])
def test_band_limit_moves_across_calls(cfgid, direction):
    """The stages skip the QMF bands from the run's band limit up (SbrRec::blim: the stream's
    highest kx + M so far).  stop_freq 9 -> 5 moves kx + M from 45 to 32: falling (frame 12 on), the
    PS all-pass / delay state of bands 32..44 keeps ringing and must still run; rising (frame 23 =
    the call boundary), the history rows the slot state carries must read as zero from 32 up.
    Float32 output, bit-exact against the restatement (A/sbr/Channel.java:618-645)."""
    fps = 36
    p = N.synth_params(cfgid, n_streams=3, frames_per_stream=fps)

    def edit(s):
        f = np.arange(len(s)) % fps
        s["hdr"]["stop_freq"][(f >= 12) if direction == "fall" else (f < 23)] = 5

    b = _edit(N.synth_batch(p), edit)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(3), N.PCM_FLOAT32, threads=8)
    first, second = b.split_frames(23)
    with N.Context(cfg, 3) as ctx:
        g1 = ctx.decode(first, N.PCM_FLOAT32)
        g2 = ctx.decode(second, N.PCM_FLOAT32)
    fb = b.frame_begin
    for r in range(3):
        _assert_same(g1[23 * r:23 * (r + 1)], want[fb[r]:fb[r] + 23], N.PCM_FLOAT32)
        _assert_same(g2[13 * r:13 * (r + 1)], want[fb[r] + 23:fb[r + 1]], N.PCM_FLOAT32)


@pytest.mark.parametrize("cfgid,smoothing", [(4, 1), (5, 1), (4, 0)])
def test_dropped_patch_with_trailing_borders(cfgid, smoothing):
    """A header whose patch_construction drops bands (start_freq 0, stop_freq 7, freq_scale 0 at
    48 kHz: kx 7, M 31, the patches generate 21 bands) with envelopes ending past slot 32: the
    bands without patch carry frame f-1's adjusted rows into the envelope estimate, chains of
    kSbrDep frames run through the HF fix passes.  With G/Q smoothing (bs_smoothing_mode 0) the
    frame after a recomputed one is recomputed too (its smoothing ring came from that frame)."""
    fps = 36
    p = N.synth_params(cfgid, n_streams=3, frames_per_stream=fps)
    rng = np.random.default_rng(5)

    def edit(s):
        s["hdr"]["start_freq"], s["hdr"]["stop_freq"], s["hdr"]["freq_scale"] = 0, 7, 0
        s["hdr"]["smoothing_mode"] = smoothing
        _var_grids(s, rng)

    b = _edit(N.synth_batch(p), edit)
    info = O.sbr_table_info(b.sbr["hdr"][0], 3)[0]
    assert info["gen_cnt"] < info["M"], info
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(3), N.PCM_FLOAT32, threads=8)
    first, second = b.split_frames(17)
    with N.Context(cfg, 3) as ctx:
        g1 = ctx.decode(first, N.PCM_FLOAT32)
        g2 = ctx.decode(second, N.PCM_FLOAT32)
    fb = b.frame_begin
    for r in range(3):
        _assert_same(g1[17 * r:17 * (r + 1)], want[fb[r]:fb[r] + 17], N.PCM_FLOAT32)
        _assert_same(g2[19 * r:19 * (r + 1)], want[fb[r] + 17:fb[r + 1]], N.PCM_FLOAT32)


def test_long_dependent_chain_uses_the_chain_walker():
    """With G/Q smoothing a kSbrDep frame makes every later frame of the run depend on the one
    before it: chains far longer than kSbrFixPasses (8) links.  The links past 8 run in the
    sequential chain walker (one wave per run and channel) instead of one launch per link."""
    fps = 120
    p = N.synth_params(4, n_streams=2, frames_per_stream=fps)
    rng = np.random.default_rng(9)

    def edit(s):
        s["hdr"]["start_freq"], s["hdr"]["stop_freq"], s["hdr"]["freq_scale"] = 0, 7, 0
        s["hdr"]["smoothing_mode"] = 0
        _var_grids(s, rng)

    b = _edit(N.synth_batch(p), edit)
    got, want = _decode_both(p, b, N.PCM_FLOAT32)
    _assert_same(got, want, N.PCM_FLOAT32)


def test_c4_single_frame_runs_and_empty_runs():
    p = N.synth_params(4, n_streams=4, frames_per_stream=9)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(4), N.PCM_FLOAT32)
    with N.Context(cfg, 4) as ctx:
        out = []
        for cut in range(9):  # one frame per call, every stream
            one, b2 = b.split_frames(1) if cut == 0 else rest.split_frames(1)
            rest = b2
            out.append(ctx.decode(one, N.PCM_FLOAT32))
    fb = b.frame_begin
    for k in range(9):
        for r in range(4):
            assert np.array_equal(out[k][r], want[fb[r] + k])


@pytest.mark.parametrize("cfgid,flags", [(4, N.PCM_BIG_ENDIAN), (4, N.PCM_FLOAT32), (5, N.PCM_LITTLE_ENDIAN),
                                         (5, N.PCM_FLOAT32)])
def test_downsampled_sbr(cfgid, flags):
    """Downsampled SBR (a15': extension rate = core rate, SynthesisFilterbank32): 1024 samples per
    frame at the core rate; GPU == the oracle's restatement bit for bit (both run the reference's own
    DCT4_32 / DST4_32 straight-line programs, carried as op lists in tables/jaad_sbr_dct32.inc, so the
    binary32 operations and their order are the reference's: DESIGN.md section 0)."""
    p = N.synth_params(cfgid, n_streams=3, frames_per_stream=36)
    b = N.synth_batch(p)
    cfg = N.make_cfg(p.sf_index, p.channel_config, sbr=True, ps=p.sbr == 2, down=True)
    got, want = _decode_both(p, b, flags, cfg)
    assert got.shape == (b.n_frames, 4096 * (2 if flags & N.PCM_FLOAT32 else 1))
    _assert_same(got, want, flags)


@pytest.mark.slow
def test_c4_full_batch_bitexact():
    """The whole 32 768-frame C4 batch (the bench workload, 128 streams x 256) against the restatement."""
    p = N.synth_params(4)
    assert p.n_streams * p.frames_per_stream == 32768
    got, want = _decode_both(p, N.synth_batch(p), N.PCM_BIG_ENDIAN)
    _assert_same(got, want, N.PCM_BIG_ENDIAN)


def _recouple(s):
    """Coupled frames: channel 1 carries channel 0's grid (Channel.couple, A/sbr/Channel.java:103-122)."""
    for f in np.flatnonzero(s["coupling"]):
        c0, c1 = s[f]["ch"][0], s[f]["ch"][1]
        for k in ("frame_class", "L_E", "L_Q", "bs_pointer", "t_E", "t_Q", "f", "invf_mode"):
            c1[k] = c0[k]
        r = s[f]
        r["ch"][1] = c1
        s[f] = r


@pytest.mark.parametrize("name,fn", [
    ("plain", None),
    ("amp_res0_var_grids", lambda s, rng: (s["hdr"].__setitem__("amp_res", 0), _var_grids(s, rng), _recouple(s))),
    ("smoothing_limiter3", lambda s, rng: (s["hdr"].__setitem__("smoothing_mode", 0),
                                           s["hdr"].__setitem__("limiter_bands", 3))),
])
def test_c4_coupled_stereo(name, fn):
    """Coupled stereo SBR (bs_coupling, the usual coding of low-rate HE-AAC v1): both channels'
    envelopes and noise floors come from channel 0's level and channel 1's balance
    (NoiseEnvelope.unmap incl. its double-precision sqrt(2) step and the Q_div left / right tables,
    A/sbr/NoiseEnvelope.java:192-240, 299-344), split over two calls."""
    p = N.synth_params(4, n_streams=3, frames_per_stream=36, coupling_percent=60)
    b = N.synth_batch(p)
    if fn is not None:
        rng = np.random.default_rng(3)
        b = _edit(b, lambda s: fn(s, rng))
    assert b.sbr["coupling"].sum() > 20
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(3), N.PCM_FLOAT32, threads=8)
    first, second = b.split_frames(15)
    with N.Context(cfg, 3) as ctx:
        g1 = ctx.decode(first, N.PCM_FLOAT32)
        g2 = ctx.decode(second, N.PCM_FLOAT32)
    fb = b.frame_begin
    for r in range(3):
        _assert_same(g1[15 * r:15 * (r + 1)], want[fb[r]:fb[r] + 15], N.PCM_FLOAT32)
        _assert_same(g2[21 * r:21 * (r + 1)], want[fb[r] + 15:fb[r + 1]], N.PCM_FLOAT32)


@pytest.mark.parametrize("cfgid,flags,down", [(4, N.PCM_BIG_ENDIAN, False), (4, N.PCM_FLOAT32, False),
                                              (5, N.PCM_LITTLE_ENDIAN, False), (5, N.PCM_FLOAT32, False),
                                              (4, N.PCM_FLOAT32, True)])
def test_sbr_fallback_frames(cfgid, flags, down):
    """Frames before the stream's first SBR header (QMF banks on the low band only,
    Channel.process_channel with hdr == null, A/sbr/Channel.java:589-617) and frames without
    usable SBR data (JAAD_SBR_UPSAMPLE: SBR.upsample of the core, A/sbr/SBR.java:302-309, the SBR
    state untouched -- the next SBR frame continues from the last processed one), with calls that
    cut through them: byte-exact against the restatement."""
    p = N.synth_params(cfgid, n_streams=3, frames_per_stream=40, upsample_percent=20, nohdr_frames=5,
                       coupling_percent=30 if cfgid == 4 else 0)
    b = N.synth_batch(p)
    st = b.sbr["status"].reshape(3, 40)
    assert (st == N.SBR_UPSAMPLE).any(axis=1).all()
    cfg = N.make_cfg(p.sf_index, p.channel_config, sbr=True, ps=p.sbr == 2, down=down)
    want = O.decode_batch(cfg, b, O.Streams(3), flags, threads=8)
    cuts = [0, 3, 7, 19, 20, 40]
    rest = b
    out = []
    with N.Context(cfg, 3) as ctx:
        for k in range(1, len(cuts)):
            part, rest = rest.split_frames(cuts[k] - cuts[k - 1])
            out.append(ctx.decode(part, flags))
    fb = b.frame_begin
    for k in range(1, len(cuts)):
        n = cuts[k] - cuts[k - 1]
        for r in range(3):
            _assert_same(out[k - 1][n * r:n * (r + 1)], want[fb[r] + cuts[k - 1]:fb[r] + cuts[k]], flags)


def test_upsample_only_call_and_state():
    """A call whose every frame upsamples: no SBR stage runs and the slot's SBR state stays for the
    next call's SBR frames."""
    p = N.synth_params(4, n_streams=2, frames_per_stream=12)
    b = N.synth_batch(p)
    s = b.sbr.copy()
    for r in range(2):
        s[12 * r + 4:12 * r + 7]["status"] = N.SBR_UPSAMPLE
        s[12 * r + 4:12 * r + 7]["header_present"] = 0
    b = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, s)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(2), N.PCM_BIG_ENDIAN)
    a, rest = b.split_frames(4)
    mid, c = rest.split_frames(3)
    with N.Context(cfg, 2) as ctx:
        g = [ctx.decode(x, N.PCM_BIG_ENDIAN) for x in (a, mid, c)]
    fb = b.frame_begin
    for r in range(2):
        assert np.array_equal(g[0][4 * r:4 * (r + 1)], want[fb[r]:fb[r] + 4])
        assert np.array_equal(g[1][3 * r:3 * (r + 1)], want[fb[r] + 4:fb[r] + 7])
        assert np.array_equal(g[2][5 * r:5 * (r + 1)], want[fb[r] + 7:fb[r + 1]])
    # the upsampled frames repeat the core sample pairs (index 1 keeps core sample 1)
    L = g[1].view(">i2").reshape(-1, 2048, 2)[..., 0].astype(np.int32)
    assert np.array_equal(L[:, 2::2], L[:, 3::2])


@pytest.mark.parametrize("cfgid", [4, 5])
def test_fused_analysis_equals_the_separate_kernels(cfgid, monkeypatch):
    """Round 6: a launch without smoothing or HF fix passes runs the QMF analysis inside the HF kernel
    (sbr_hf_kernel<5>); JAAD_SBR_FUSED=0 keeps sbr_analysis_kernel + sbr_hf_kernel<0>.  Both give the
    same PCM, and it is the restatement's, across a continuation call (rows 0..7 of a run's first
    record from the slot state, of the others recomputed from the previous frame's samples)."""
    p = N.synth_params(cfgid, n_streams=4, frames_per_stream=24)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    n = int(b.stream_slot.max()) + 1
    halves = b.split_frames(12)
    outs = {}
    for fz in ("1", "0"):
        monkeypatch.setenv("JAAD_SBR_FUSED", fz)
        with N.Context(cfg, n) as ctx:
            outs[fz] = [ctx.decode(h, N.PCM_BIG_ENDIAN) for h in halves]
    want = O.decode_batch(cfg, b, O.Streams(n), N.PCM_BIG_ENDIAN, threads=8)
    fb = b.frame_begin
    for k in range(2):
        _assert_same(outs["1"][k], outs["0"][k], N.PCM_BIG_ENDIAN)
    for r in range(len(fb) - 1):
        assert np.array_equal(outs["1"][0][12 * r:12 * (r + 1)], want[fb[r]:fb[r] + 12])
        assert np.array_equal(outs["1"][1][12 * r:12 * (r + 1)], want[fb[r] + 12:fb[r + 1]])
