"""SBR / PS part of the host bitstream front end (jaadec_amd/csrc/jaad_parse_sbr.cpp).

Pinning, as for the core syntax (tests/test_parse.py): the reference ships no HE-AAC bitstreams,
so parsed-frame records are written as sbr_extension_data by the test writer
(oracle/jaad_writer_sbr.c, the reference's SBR / PS Huffman trees) and must parse back to the
same records.  The writer draws the coding choices (frequency / time deltas, CRC, explicit
header defaults, repeated PS headers) from a seed, so every stream exercises the delta
decoding against the previous frame (sbr_save_prev_data) and the resolution mapping of
extract_envelope_data.  Grids other than FIXFIX carry borders and t_Q computed here by a
restatement of envelope_time_border_vector / noise_floor_time_border_vector
(A/sbr/Channel.java:455-583).
"""
import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O


def _canonical(rec, nch, out_sf):
    """The record as the parser emits it: meaningful entries only (see to_record)."""
    r = rec.copy()
    (n0, n1, NQ, Nhigh, _), _ = O.sbr_res_tables(r["hdr"], out_sf)
    n = (n0, n1)
    for c in range(2):
        ch = r["ch"][c]
        if c >= nch:
            r["ch"][c] = np.zeros((), N.SBR_CHANNEL_DTYPE)
            continue
        L_E, L_Q = int(ch["L_E"]), int(ch["L_Q"])
        E = np.zeros_like(ch["E"])
        for l in range(L_E):
            nb = n[int(ch["f"][l]) & 1]
            E[l, :nb] = ch["E"][l, :nb]
        ch["E"] = E
        Q = np.zeros_like(ch["Q"])
        Q[:L_Q, :NQ] = ch["Q"][:L_Q, :NQ]
        ch["Q"] = Q
        ch["t_E"][L_E + 1:] = 0
        ch["f"][L_E:] = 0
        ch["invf_mode"][NQ:] = 0
        ch["add_harmonic"] = int(ch["add_harmonic"]) & ((1 << Nhigh) - 1) if ch["add_harmonic_flag"] else 0
        r["ch"][c] = ch
    if r["ps_present"]:
        ps = r["ps"]
        ne = int(ps["num_env"])
        for name, mode in (("iid", int(ps["iid_mode"])), ("icc", int(ps["icc_mode"]))):
            a = ps[name].copy()
            a[ne:] = 0
            a[:, 34 if mode % 3 == 2 else 20:] = 0
            ps[name] = a
        ps["border"][ne + 1:] = 0
        r["ps"] = ps
    return r


def _assert_sbr_equal(got, want, nch, out_sf):
    seen_hdr = False
    for f in range(len(want)):
        g = got[f]
        assert g["status"] == want[f]["status"], (f, "status")
        if want[f]["status"] == N.SBR_UPSAMPLE or not (seen_hdr or want[f]["header_present"]):
            # no usable SBR data / no header yet: the record carries nothing else
            assert g["header_present"] == want[f]["header_present"], (f, "header_present")
            continue
        seen_hdr = True
        w = _canonical(want[f], nch, out_sf)
        for key in ("header_present", "coupling", "ps_present"):
            assert g[key] == w[key], (f, key)
        assert g["hdr"].tobytes() == w["hdr"].tobytes(), f
        for c in range(nch):
            for name in N.SBR_CHANNEL_DTYPE.names:
                if name == "reserved":
                    continue
                assert np.array_equal(g["ch"][c][name], w["ch"][c][name]), (f, c, name, g["ch"][c][name], w["ch"][c][name])
        if w["ps_present"]:
            for name in N.PS_FRAME_DTYPE.names:
                if name in ("reserved", "pad"):
                    continue
                assert np.array_equal(g["ps"][name], w["ps"][name]), (f, name, g["ps"][name], w["ps"][name])


def _middle_border(cls, L_E, ptr):
    if cls == 0:
        m = L_E // 2
    elif cls == 2:
        m = 1 if ptr == 0 else (L_E - 1 if ptr == 1 else ptr - 1)
    else:
        m = L_E + 1 - ptr if ptr > 1 else L_E - 1
    return max(m, 0)


_LOG2 = [0, 0, 1, 2, 2, 3, 3, 3, 3, 4]


def _random_grid(ch, rng):
    """Give a channel record a FIXVAR / VARFIX / VARVAR grid (borders in QMF slots, rate 2)."""
    cls = int(rng.integers(1, 4))
    L_E = int(rng.integers(1, 5))
    t = np.zeros(6, np.int64)
    if cls == 1:  # FIXVAR: relative borders from the trailing one
        trail = 16 + int(rng.integers(0, 4))
        t[L_E] = 2 * trail
        b = trail
        for i in range(L_E - 1, 0, -1):
            b -= 2 * int(rng.integers(1, 3))
            t[i] = 2 * b
        t[0] = 0
    else:  # VARFIX / VARVAR: from the leading one (VARVAR trail 16..19)
        lead = int(rng.integers(0, 4))
        t[0] = 2 * lead
        b = lead
        for i in range(1, L_E):
            b += 2 * int(rng.integers(1, 3))
            t[i] = 2 * b
        t[L_E] = 32 if cls == 2 else 2 * (16 + int(rng.integers(0, 4)))
    while True:  # a pointer whose middle border lies inside the grid
        ptr = int(rng.integers(0, 1 << _LOG2[L_E + 1])) if _LOG2[L_E + 1] else 0
        if _middle_border(cls, L_E, ptr) <= L_E:
            break
    ch["frame_class"] = cls
    ch["L_E"] = L_E
    ch["L_Q"] = 2 if L_E > 1 else 1
    ch["bs_pointer"] = ptr
    ch["t_E"] = t
    if L_E == 1:
        ch["t_Q"] = [t[0], t[1], 0]
    else:
        ch["t_Q"] = [t[0], t[_middle_border(cls, L_E, ptr)], t[L_E]]
    ch["f"] = [int(rng.integers(0, 2)) for _ in range(6)]
    E = ch["E"]
    for l in range(1, 5):
        if not E[l].any():
            E[l] = E[l - 1]
    ch["E"] = E
    Q = ch["Q"]
    if not Q[1].any():
        Q[1] = Q[0]
    ch["Q"] = Q


def _random_ps(ps, rng, prev_modes):
    iid_mode, icc_mode = (int(rng.integers(0, 6)), int(rng.integers(0, 6))) if rng.integers(0, 3) == 0 or \
        prev_modes is None else prev_modes
    ne = int(rng.choice([1, 2, 4]))
    ps["iid_mode"], ps["icc_mode"], ps["num_env"] = iid_mode, icc_mode, ne
    ps["border"] = [e * 32 // ne for e in range(ne + 1)] + [0] * (5 - ne)
    steps = 15 if iid_mode >= 3 else 7
    iid = np.zeros((5, 34), np.int8)
    icc = np.zeros((5, 34), np.int8)
    for e in range(ne):
        for arr, mode, lo, hi in ((iid, iid_mode, -steps, steps), (icc, icc_mode, 0, 7)):
            nb = 34 if mode % 3 == 2 else 20
            v = np.clip(int(rng.integers(lo, hi + 1)) + np.cumsum(rng.choice([-1, 0, 0, 1], nb)), lo, hi)
            if mode % 3 == 0:  # 10 parameters, each covering two bands
                v = np.repeat(v[:10], 2)
            arr[e, :nb] = v
    ps["iid"], ps["icc"] = iid, icc
    return iid_mode, icc_mode


def _stream(cfgid, frames, seed, grids=False, ps_modes=False, header_gaps=True, header_change=False, new_header=None):
    p = N.synth_params(cfgid, n_streams=1, frames_per_stream=frames)
    b = N.synth_batch(p)
    rng = np.random.default_rng(seed)
    prev_modes = None
    for f in range(frames):
        r = b.sbr[f]
        if header_gaps and f > 0 and rng.integers(0, 3):
            r["header_present"] = 0
        if header_change and f >= frames // 2:
            h = r["hdr"]
            for key, v in (new_header or dict(start_freq=4, stop_freq=6, alter_scale=0)).items():
                h[key] = v
            r["hdr"] = h
            if f == frames // 2:
                r["header_present"] = 1
        for c in range(b.nch):
            if grids and rng.integers(0, 2):
                ch = r["ch"][c]
                _random_grid(ch, rng)
                r["ch"][c] = ch
        if ps_modes and r["ps_present"]:
            ps = r["ps"]
            prev_modes = _random_ps(ps, rng, prev_modes)
            r["ps"] = ps
        b.sbr[f] = r
    # FIXFIX reads no pointer: Channel.bs_pointer keeps the one of the last grid that had one
    last = [0, 0]
    for f in range(frames):
        for c in range(b.nch):
            ch = b.sbr[f]["ch"][c]
            if ch["frame_class"] == 0:
                ch["bs_pointer"] = last[c]
            last[c] = int(ch["bs_pointer"])
    return p, b


def _round_trip(p, b, seed, extras=0):
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, extras=extras, sbr_writer=O.SbrWriter(cfg.ext_sf_index, seed))
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    got = P.parse(frames)
    _assert_sbr_equal(got.sbr, b.sbr, b.nch, cfg.ext_sf_index)
    assert np.array_equal(got.q, b.q) and np.array_equal(got.ics, b.ics)
    return frames, got


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("cfgid,opts", [
    (4, {}),
    (4, dict(grids=True)),
    (4, dict(grids=True, header_change=True)),
    (5, {}),
    (5, dict(grids=True, ps_modes=True)),
    (5, dict(ps_modes=True, header_change=True)),
], ids=["c4", "c4_grids", "c4_hdr_change", "c5", "c5_grids_psmodes", "c5_psmodes_hdr_change"])
def test_sbr_write_parse_round_trip(cfgid, opts, seed):
    p, b = _stream(cfgid, 24, seed, **opts)
    _round_trip(p, b, seed, extras=seed & 1)


def test_sbr_frames_before_the_first_header_and_missing_payloads():
    p, b = _stream(4, 4, 7, header_gaps=False)
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 7))
    # an LC frame (no SBR FIL) in an SBR configuration: the element's SBR stays invalid, the
    # reference upsamples the core (A/syntax/CPE.java:201-204)
    lc = O.write_frames(b, p.sf_index, frames=[0])[0]
    got = N.Parser(cfg).parse([lc])
    assert got.sbr[0]["status"] == N.SBR_UPSAMPLE
    # the same SBR FIL in an LC configuration (implicit SBR) is refused, not skipped
    lc_cfg = N.make_cfg(p.sf_index, p.channel_config)
    with pytest.raises(N.JaadError) as e:
        N.Parser(lc_cfg).parse([frames[0]])
    assert e.value.status == N.ERR_UNSUPPORTED
    # a header-less SBR payload before any header: valid, nothing read (A/sbr/SBR.java:179-184)
    b2 = b.select_runs([0])
    b2.sbr = b.sbr.copy()
    b2.sbr[1]["header_present"] = 0
    w = O.SbrWriter(cfg.ext_sf_index, 7)
    f01 = O.write_frames(b2, p.sf_index, frames=[0, 1], sbr_writer=w)
    got = N.Parser(cfg).parse([f01[1]])
    assert got.sbr[0]["status"] == N.SBR_OK and got.sbr[0]["header_present"] == 0
    got = N.Parser(cfg).parse(f01)
    _assert_sbr_equal(got.sbr, b2.sbr[:2], 2, cfg.ext_sf_index)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
@pytest.mark.parametrize("cfgid", [4, 5])
def test_sbr_coupling_fallbacks_round_trip(cfgid, seed):
    """Coupled CPE frames (SBR2.sbr_data's coupled branch, channel 1 balance coded), frames
    before the first header, and frames whose SBR data is missing or fails its grid
    (JAAD_SBR_UPSAMPLE) parse back to the generator's records."""
    p = N.synth_params(cfgid, n_streams=1, frames_per_stream=40, coupling_percent=50, upsample_percent=20,
                       nohdr_frames=3, seed=0x5EED00 + seed)
    b = N.synth_batch(p)
    assert (b.sbr["status"] == N.SBR_UPSAMPLE).any()
    if cfgid == 4:
        assert b.sbr["coupling"].any()
    frames, got = _round_trip(p, b, seed)
    assert got.sbr["status"].tolist() == b.sbr["status"].tolist()


def test_sbr_truncated_payload_is_eos_and_atomic():
    p, b = _stream(5, 6, 11, ps_modes=True)
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 11))
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    out = []
    for i, fr in enumerate(frames):
        if i == 3:
            for cut in (len(fr) - 1, len(fr) - 3):
                with pytest.raises(N.JaadError):
                    P.parse([fr[:cut]])
        out.append(P.parse([fr]).sbr[0])
    _assert_sbr_equal(np.array(out), b.sbr, 1, cfg.ext_sf_index)


def test_ps_payload_in_a_config_without_ps_is_refused():
    p, b = _stream(5, 2, 5, header_gaps=False)
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 5))
    mono_sbr = N.make_cfg(p.sf_index, 1, sbr=True)
    with pytest.raises(N.JaadError) as e:
        N.Parser(mono_sbr).parse(frames[:1])
    assert e.value.status == N.ERR_UNSUPPORTED


@pytest.mark.gpu
@pytest.mark.parametrize("cfgid", [4, 5])
def test_he_aac_bitstream_decodes_on_the_gpu(cfgid):
    """HE-AAC v1 / v2 bitstream -> host parser -> HIP DSP path == the restatement's PCM of the
    records the bitstream was written from, byte for byte."""
    p, b = _stream(cfgid, 24, 21, grids=False, ps_modes=cfgid == 5)
    cfg = N.cfg_for(p)
    frames, got = _round_trip(p, b, 21)
    want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    with N.Context(cfg, 1) as ctx:
        pcm = ctx.decode(got, N.PCM_BIG_ENDIAN)
    assert pcm.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("cfgid", [4, 5])
def test_coupled_and_fallback_bitstream_decodes_on_the_gpu(cfgid):
    """Coupled frames, frames before the first header, and missing / failing SBR payloads, from
    the bitstream through the host parser and the HIP path == the restatement, byte for byte."""
    p = N.synth_params(cfgid, n_streams=1, frames_per_stream=40, coupling_percent=50, upsample_percent=20,
                       nohdr_frames=3, seed=0x5EED07)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    frames, got = _round_trip(p, b, 8)
    want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    with N.Context(cfg, 1) as ctx:
        pcm = ctx.decode(got, N.PCM_BIG_ENDIAN)
    assert pcm.tobytes() == want.tobytes()


def test_implicit_sbr_probe_and_upgraded_config():
    """ADTS / LC-only signalling: SBR is found in the payload (implicit SBR)."""
    for cfgid in (4, 5):
        p, b = _stream(cfgid, 2, 3, header_gaps=False)
        cfg = N.cfg_for(p)
        sbr_frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 3))
        lc_frames = O.write_frames(b, p.sf_index)
        core = N.make_cfg(p.sf_index, p.channel_config)
        assert N.probe_sbr(core, sbr_frames[0]) and not N.probe_sbr(core, lc_frames[0])
        up = N.implicit_sbr_cfg(core)
        assert (up.sbr, up.ps, up.ext_sf_index) == (1, int(p.channel_config == 1), p.sf_index - 3)
        # the upgraded configuration parses the stream to the records it was written from
        P = N.Parser(up)
        P.pns_state = int(b.ics["pns_state"][0])
        got = P.parse(sbr_frames)
        _assert_sbr_equal(got.sbr, b.sbr, b.nch, up.ext_sf_index)
    # 64 kHz core: no doubled rate, the SBR runs downsampled at the core rate
    down = N.implicit_sbr_cfg(N.make_cfg(2, 2))
    assert (down.sbr, down.ext_sf_index) == (1, 2) and N.sbr_downsampled(down)
    # explicit AOT 5 mono: PS stays enabled, as psEnabled is by default
    cfg = N.asc_parse(bytes([0x2B, 0x09, 0x88, 0x00]))
    assert (cfg.sbr, cfg.ps, cfg.channel_config) == (1, 1, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("cfgid", [4, 5])
def test_adts_he_aac_with_implicit_sbr_through_the_decoder_facade(cfgid):
    """An ADTS HE-AAC stream (the header says LC at the core rate) through ADTSDemultiplexer +
    Decoder: the façade finds the SBR payload, re-opens at the doubled rate, and the PCM equals
    the restatement's decode of the records, byte for byte."""
    from jaadec_amd.decoder import ADTSDemultiplexer, Decoder, SampleBuffer
    p, b = _stream(cfgid, 12, 9, ps_modes=cfgid == 5)
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 9))
    stream = O.adts_wrap(frames, p.sf_index, p.channel_config)
    demux = ADTSDemultiplexer(stream)
    dec = Decoder.create(demux.getDecoderInfo())
    payloads = []
    while True:
        try:
            payloads.append(demux.readNextFrame())
        except EOFError:
            break
    bufs = [SampleBuffer() for _ in payloads]
    assert not dec.getConfig().sbr
    dec.decodeFrames(payloads, bufs)  # no PNS bands in C4/C5: the parser's LCG start is moot
    assert dec.getConfig().getSampleLength() == 2048 and dec.getConfig().getOutputFrequency() == 48000
    want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    assert b"".join(x.data for x in bufs) == want.tobytes()
    dec.close()
