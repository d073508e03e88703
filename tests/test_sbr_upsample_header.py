"""An SBR header on a frame whose SBR data is unusable (JAAD_SBR_UPSAMPLE).

SBR.decode reads the header and, when it differs, recomputes the frequency tables before sbr_data
fails (A/sbr/SBR.java:168-177, readHeader :212-221); the frame itself upsamples the core.  Patches
and limiter bands are rebuilt only by a frame that runs SBR with a reset (HFGeneration :27-28,
HFAdjustment limiter table on reset), so the frames after it run with the new frequency tables and
the old patches until a processed frame changes the header again.  The library keeps that mixed
table set (SbrHost::take_header) and refuses the mixes where the reference indexes outside its
arrays (M changes, patches past band 63, patch sources at or above the new kx).

CPU: the restatement's accept/refuse decisions.  GPU: HIP parity against the restatement, with
calls that cut between the header frame and the frames that use the mixed tables."""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

FPS = 30


def _batch(cfgid, changes, n_streams=2):
    """changes: list of (frame, status, header-field dict) applied to every stream (fields persist
    from that frame on, as a stream's header does)."""
    p = N.synth_params(cfgid, n_streams=n_streams, frames_per_stream=FPS)
    b = N.synth_batch(p)
    s = b.sbr.copy()
    f = np.arange(len(s)) % FPS
    for frame, status, fields in changes:
        for k, v in fields.items():
            s["hdr"][k][f >= frame] = v
        if status == N.SBR_UPSAMPLE:
            s["status"][f == frame] = N.SBR_UPSAMPLE
            s["header_present"][f == frame] = 1
    return p, N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, s)


U, K = N.SBR_UPSAMPLE, N.SBR_OK
# accepted: frequency tables move, M stays; old patches still inside the new bands
ACCEPTED = {
    "freq_scale": [(8, U, dict(freq_scale=3))],
    "noise_bands": [(8, U, dict(noise_bands=1))],
    "kx_up": [(8, U, dict(start_freq=8, stop_freq=15))],
    "kx_up_then_reset": [(8, U, dict(start_freq=9, stop_freq=10, freq_scale=3)), (20, K, dict(xover_band=1))],
    "back_and_forth": [(6, U, dict(freq_scale=3)), (11, U, dict(freq_scale=2)), (17, U, dict(start_freq=8, stop_freq=15))],
}
# refused: M changes (start_freq 7 alone), old patch sources above the new kx (kx 9)
REFUSED = {
    "M_changes": [(8, U, dict(start_freq=7))],
    "src_above_kx": [(8, U, dict(start_freq=1, stop_freq=8, freq_scale=0))],
}


def _refused(rc_text):
    return f"oracle decode failed: {N.ERR_UNSUPPORTED}" in rc_text


@pytest.mark.parametrize("name", sorted(ACCEPTED))
def test_oracle_accepts(name):
    p, b = _batch(4, ACCEPTED[name])
    out = O.decode_batch(N.cfg_for(p), b, O.Streams(2), N.PCM_FLOAT32, threads=4)
    assert np.isfinite(out.view(np.float32)).all()


@pytest.mark.parametrize("name", sorted(REFUSED))
def test_oracle_refuses(name):
    p, b = _batch(4, REFUSED[name])
    with pytest.raises(RuntimeError) as e:
        O.decode_batch(N.cfg_for(p), b, O.Streams(2), N.PCM_FLOAT32)
    assert _refused(str(e.value))


def test_oracle_header_before_any_sbr_frame_refused():
    """No SBR frame has run yet: there are no patches to keep."""
    p, b = _batch(4, [(0, U, dict(freq_scale=3))])
    with pytest.raises(RuntimeError) as e:
        O.decode_batch(N.cfg_for(p), b, O.Streams(2), N.PCM_FLOAT32)
    assert _refused(str(e.value))


def test_mixed_tables_differ_from_a_reset():
    """The mixed tables are not the pure ones: the same stream with frame 8 upsampled without a
    header and the change arriving on frame 9 (a processed frame: reset, new patches) decodes the
    same up to frame 8 and differently after it."""
    p, mixed = _batch(4, ACCEPTED["kx_up"])
    _, pure = _batch(4, [(9, K, dict(start_freq=8, stop_freq=15))])
    s = pure.sbr.copy()
    s["status"][np.arange(len(s)) % FPS == 8] = N.SBR_UPSAMPLE
    s["header_present"][np.arange(len(s)) % FPS == 8] = 0
    pure = N.Batch(pure.q, pure.sf, pure.cb, pure.ics, pure.ms_used, pure.tns, pure.stream_slot,
                   pure.frame_begin, pure.nch, s)
    cfg = N.cfg_for(p)
    a = O.decode_batch(cfg, mixed, O.Streams(2), N.PCM_FLOAT32)
    bb = O.decode_batch(cfg, pure, O.Streams(2), N.PCM_FLOAT32)
    assert np.array_equal(a[:9], bb[:9])
    assert not np.array_equal(a[9:FPS], bb[9:FPS])


# ------------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------------

def _same(got, want):
    bad = np.flatnonzero(got.view(np.uint32).reshape(-1) != want.view(np.uint32).reshape(-1))
    assert bad.size == 0, f"{bad.size} float samples differ, first at {bad[:4]}"


@pytest.mark.gpu
@pytest.mark.parametrize("cfgid", [4, 5])
@pytest.mark.parametrize("name", sorted(ACCEPTED))
def test_gpu_upsample_header_matches_oracle(name, cfgid):
    p, b = _batch(cfgid, ACCEPTED[name])
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(2), N.PCM_FLOAT32, threads=8)
    cuts = [0, 9, 13, FPS]  # a call ends right after the header frame
    rest, out = b, []
    with N.Context(cfg, 2) as ctx:
        for k in range(1, len(cuts)):
            part, rest = rest.split_frames(cuts[k] - cuts[k - 1])
            out.append(ctx.decode(part, N.PCM_FLOAT32))
    fb = b.frame_begin
    for k in range(1, len(cuts)):
        n = cuts[k] - cuts[k - 1]
        for r in range(2):
            _same(out[k - 1][n * r:n * (r + 1)], want[fb[r] + cuts[k - 1]:fb[r] + cuts[k]])


@pytest.mark.gpu
def test_gpu_upsample_header_state_export_import():
    """The mixed table set travels in the slot state: a stream resumed in another context after
    the header frame decodes as the restatement does."""
    p, b = _batch(4, ACCEPTED["kx_up"])
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, b, O.Streams(2), N.PCM_FLOAT32, threads=8)
    first, second = b.split_frames(10)
    with N.Context(cfg, 2) as ctx:
        ctx.decode(first, N.PCM_FLOAT32)
        blob = ctx.state_export(1)
    with N.Context(cfg, 2) as ctx2:
        ctx2.state_import(1, blob)
        got = ctx2.decode(second.select_runs([1]), N.PCM_FLOAT32)
    fb = b.frame_begin
    _same(got, want[fb[1] + 10:fb[2]])


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(REFUSED))
def test_gpu_upsample_header_refused(name):
    p, b = _batch(4, REFUSED[name])
    with N.Context(N.cfg_for(p), 2) as ctx:
        with pytest.raises(N.JaadError) as e:
            ctx.decode(b, N.PCM_FLOAT32)
    assert e.value.status == N.ERR_UNSUPPORTED


# ------------------------------------------------------------------------------------------------
# A dropped frame (jaad_batch.frame_status) whose SBR payload was read whole before the bitstream
# ended: Decoder.decodeFrame catches the EOSException after SBR.decode swapped in the header
# (A/Decoder.java:89-101, A/sbr/SBR.java:162-184) and skips process() -- the same SBR state change
# as an upsampled frame's header, without any PCM.
# ------------------------------------------------------------------------------------------------

def _dropped(b, frame):
    """b with frame `frame` of every stream marked dropped (its records, header included, kept)."""
    st = np.zeros(b.n_frames, np.uint8)
    st[np.arange(b.n_frames) % FPS == frame] = N.FRAME_EOS
    d = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, b.sbr.copy())
    d.frame_status = st
    return d


@pytest.mark.parametrize("name", ["kx_up", "back_and_forth", "kx_up_then_reset"])
def test_oracle_dropped_frame_takes_its_header(name):
    """The header of the dropped frame is in the SBR state afterwards: the next frame, which carries
    the same header, runs without a reset on the mixed tables (SbrHost::take_header), so the stream
    decodes differently from the same batch with the dropped frame's header removed (the next frame
    then resets), and equally up to the dropped frame."""
    p, up = _batch(4, ACCEPTED[name])
    frame = ACCEPTED[name][0][0]
    cfg = N.cfg_for(p)
    with_hdr = _dropped(up, frame)
    no_hdr = _dropped(up, frame)
    no_hdr.sbr["header_present"][np.arange(up.n_frames) % FPS == frame] = 0
    a = O.decode_batch(cfg, with_hdr, O.Streams(2), N.PCM_FLOAT32, threads=4)
    b = O.decode_batch(cfg, no_hdr, O.Streams(2), N.PCM_FLOAT32, threads=4)
    rows = np.arange(up.n_frames) % FPS
    assert not a[rows == frame].any() and not b[rows == frame].any()
    assert np.array_equal(a[rows < frame], b[rows < frame])
    assert not np.array_equal(a[rows > frame], b[rows > frame])


def test_oracle_dropped_first_header_refused():
    """A stream's first SBR header on a dropped frame: no processed frame has built patches."""
    p, b = _batch(4, [])
    s = b.sbr.copy()
    s["header_present"][np.arange(b.n_frames) % FPS == 1] = 0  # frame 1 would bring the header too
    d = _dropped(N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, s), 0)
    with pytest.raises(RuntimeError) as e:
        O.decode_batch(N.cfg_for(p), d, O.Streams(2), N.PCM_FLOAT32)
    assert _refused(str(e.value))


def _cut_after_payload():
    """A stream whose frame k = FPS // 2 changes the SBR header, written with a fill element after
    the SBR payload (the writer's `extras`), and the shortest cut of frame k that leaves the SBR
    payload whole.  Returns (p, cfg, frames, k, cut, cut_batch, whole_batch)."""
    from tests.test_parse_sbr import _stream
    k = FPS // 2
    # a header change the SBR state can take on a frame it does not process (ACCEPTED["kx_up"])
    p, b = _stream(4, FPS, 5, header_gaps=False, header_change=True, new_header=dict(start_freq=8, stop_freq=15))
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, extras=1, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 5))
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    whole = P.parse(frames)
    P.close()
    for cut in range(1, 8):
        P = N.Parser(cfg)
        P.pns_state = int(b.ics["pns_state"][0])
        try:
            got = P.parse(frames[:k] + [frames[k][:-cut]] + frames[k + 1:], drop_eos=True)
        except N.JaadError as e:
            assert e.status == N.ERR_UNSUPPORTED  # a cut inside the SBR payload is refused
            continue
        finally:
            P.close()
        assert np.flatnonzero(got.frame_status).tolist() == [k]
        if got.sbr[k]["header_present"]:
            return p, cfg, frames, k, cut, got, whole
    raise AssertionError("no cut of frame k left its SBR payload whole")


def test_parser_frame_cut_after_its_sbr_payload_keeps_the_header():
    """a HE-AAC frame whose bitstream ends after its SBR payload is dropped with the
    payload's record, the new header included, and the frames after it parse as in the whole stream
    (the parser state moved with the payload, as the reference's SBR.decode had run); a cut inside
    the SBR payload is refused instead (the reference would have applied part of it)."""
    p, cfg, frames, k, cut, got, whole = _cut_after_payload()
    assert whole.sbr[k]["hdr"].tobytes() != whole.sbr[k - 1]["hdr"].tobytes()
    assert got.sbr[k]["hdr"].tobytes() == whole.sbr[k]["hdr"].tobytes()
    assert got.sbr[k + 1:].tobytes() == whole.sbr[k + 1:].tobytes()
    assert (got.q[(k + 1) * got.nch:] == whole.q[(k + 1) * got.nch:]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("cfgid", [4, 5])
def test_gpu_dropped_frame_header_matches_oracle(cfgid):
    p, up = _batch(cfgid, ACCEPTED["kx_up"])
    d = _dropped(up, 8)
    cfg = N.cfg_for(p)
    want = O.decode_batch(cfg, d, O.Streams(2), N.PCM_FLOAT32, threads=8)
    nb = want.shape[1]
    out = np.full((d.n_frames, nb), 0x6B, np.uint8)
    with N.Context(cfg, 2) as ctx:
        ctx.decode(d, N.PCM_FLOAT32, out=out)
    rows = np.arange(d.n_frames) % FPS
    assert (out[rows == 8] == 0x6B).all()
    _same(out[rows != 8], want[rows != 8])


@pytest.mark.gpu
def test_gpu_bitstream_frame_cut_after_its_sbr_payload():
    """The parsed stream of test_parser_frame_cut_after_its_sbr_payload_keeps_the_header through the
    HIP path == the restatement (both take the dropped frame's header); its PCM slot untouched."""
    p, cfg, frames, k, cut, got, whole = _cut_after_payload()
    want = O.decode_batch(cfg, got, O.Streams(1), N.PCM_BIG_ENDIAN)
    with N.Context(cfg, 1) as ctx:
        out = np.full(want.shape, 0x22, np.uint8)
        ctx.decode(got, N.PCM_BIG_ENDIAN, out=out)
    assert (out[k] == 0x22).all()
    assert (np.delete(out, k, 0) == np.delete(want, k, 0)).all()
