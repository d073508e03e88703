"""Coupling channel elements (A/syntax/CCE.java) and dependent coupling
(ChannelElement.processDependentCoupling A/syntax/ChannelElement.java:105-130, CCE.applyDependentCoupling
A/syntax/CCE.java:188-215).

CPU: CCE elements written by the test writer parse into records and terms equal to a Python
restatement of CCE.decode's gain lists and of processDependentCoupling's target walk (including
the SCE/LFE tag quirk and the never-applied independent-switching CCE).  GPU: batches with
coupling terms decode byte-exactly as the C restatement (oracle/jaad_oracle.c orc_couple) --
stereo, mono, 5.1, spec TNS between the two coupling points, noise bands in the CCE, short windows, several terms per frame -- through the
host entry, the device entry and the Decoder facade."""
import math

import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

CCE_SCALE = [1.09050773266525765921, 1.18920711500272106672, 1.4142135623730950488016887, 2.0]


def nbands(ic) -> int:
    groups = 8 - bin(int(ic["grouping"]) & 0x7F).count("1") if ic["window_sequence"] == 2 else 1
    return groups * int(ic["max_sfb"])


def ref_gains(d, cb, ic) -> tuple[int, np.ndarray]:
    """CCE.decode's gain lists (A/syntax/CCE.java:141-174) for a writer description."""
    point = 2 * int(d["ind_sw"]) + int(d["domain"])
    point |= point >> 1
    count = int(d["count"])
    gain_count = sum(1 + (1 if d["pair"][c] and d["chs"][c] == 3 else 0) for c in range(count + 1))
    scale = float(np.float32(CCE_SCALE[int(d["scale"])]))
    g = np.zeros((16, 120), np.float32)
    for i in range(gain_count):
        cge, xg, gc = 1, 0, np.float32(1.0)
        if i > 0:
            cge = 1 if point == 2 else int(d["cge"][i])
            xg = int(d["code"][i][0]) if cge else 0
            gc = np.float32(math.pow(scale, -xg))
        if point == 2:
            g[i][0] = gc
            continue
        for idx in range(nbands(ic)):
            if cb[idx] == 0:
                continue
            if cge == 0:
                t = int(d["code"][i][idx])
                if t != 0:
                    s = 1
                    xg += t
                    t = xg
                    if not d["sign"]:
                        s -= 2 * (t & 1)
                        t >>= 1
                    gc = np.float32(math.pow(scale, -t) * s)
            g[i][idx] = gc
    return point, g


def ref_terms(descs, recs, elements):
    """processDependentCoupling for every channel element (is_cpe, tag, first channel): the terms
    (channel, point, cce, gain row) in the reference's order per target."""
    out = []
    for k, d in enumerate(descs):
        point, g = ref_gains(d, recs[k][2], recs[k][3])
        if point not in (0, 1):
            continue
        for cpe, tag, ch0 in elements:
            index = 0
            for c in range(int(d["count"]) + 1):
                chs = int(d["chs"][c]) if d["pair"][c] else 2
                if bool(d["pair"][c]) == cpe and int(d["id"][c]) == tag:
                    if chs != 1:
                        out.append((ch0, point, k, g[index].copy()))
                        if chs != 0:
                            index += 1
                    if chs != 2:
                        out.append((ch0 + 1, point, k, g[index].copy()))
                        index += 1
                else:
                    index += 1 + (1 if chs == 3 else 0)
    return out


def cce_records(n, seed, pns=0, short=1, sf_index=3):
    """n CCE ICStream records (a mono synthetic stream's channel records)."""
    p = N.synth_params(3, n_streams=1, frames_per_stream=max(n, 1), channel_config=1, pns_percent=pns, tns_percent=0,
                       window_switching=short, sf_index=sf_index)
    p.seed = p.seed ^ (0xCCE0 + seed)
    b = N.synth_batch(p)
    ics = b.ics.copy()
    ics["window_shape_prev"] = 0  # a CCE's ICStream is never windowed
    ics["flags"] &= ~np.uint8(N.ICS_TNS)
    return b.q[:n].copy(), b.sf[:n].copy(), b.cb[:n].copy(), ics[:n].copy()


def rand_desc(rng, targets, cb, ic, pos, ind_sw=0):
    """A writer description coupling to `targets` [(pair, id, chs)] with random gains."""
    d = np.zeros((), O.CCE_DESC_DTYPE)
    d["ind_sw"], d["domain"], d["sign"], d["scale"], d["pos"] = ind_sw, rng.integers(2), rng.integers(2), rng.integers(4), pos
    d["count"] = len(targets) - 1
    for c, (pair, tid, chs) in enumerate(targets):
        d["pair"][c], d["id"][c], d["chs"][c] = pair, tid, chs if pair else 0
    gain_count = sum(1 + (1 if pr and ch == 3 else 0) for pr, _, ch in targets)
    for i in range(1, gain_count):
        d["cge"][i] = rng.integers(2)
        if d["cge"][i]:
            d["code"][i][0] = rng.integers(-6, 7)
        else:
            d["code"][i][:nbands(ic)] = rng.integers(-3, 4, nbands(ic))
    return d


def coupled_frames(cc, nf, seed, pns=0):
    """A (multi)channel batch of channel configuration cc, its raw_data_blocks with 1-2 CCEs per
    frame (random targets among the configuration's elements, some missing, one ind_sw), and the
    per-frame (descs, records)."""
    rng = np.random.default_rng(seed)
    if cc in N.MC_ELEMENTS:
        ids = N.MC_ELEMENTS[cc]
        from tests.test_multichannel import mc_synth  # noqa: F401  (same generator as the mc tests)
        b = mc_synth(cc, n_streams=1, fps=nf, seed=seed)
    else:
        ids = (0,) if cc == 1 else (1,)
        p = N.synth_params(3, n_streams=1, frames_per_stream=nf, channel_config=cc, pns_percent=pns)
        p.seed ^= seed
        b = N.synth_batch(p)
    tags, elements, ch0 = {}, [], 0
    for i in ids:
        t = tags.get(i, 0)
        tags[i] = t + 1
        elements.append((i == 1, t, ch0))
        ch0 += 2 if i == 1 else 1
    per_frame = []
    for f in range(nf):
        n = int(rng.integers(1, 3))
        q, sf, cb, ics = cce_records(n, seed * 100 + f)
        lst = []
        for k in range(n):
            targets = []
            for _ in range(int(rng.integers(1, 4))):
                cpe, tag, _ = elements[int(rng.integers(len(elements)))]
                if rng.integers(5) == 0:
                    tag = 9  # no such element
                targets.append((int(cpe), tag, int(rng.integers(4)) if cpe else 0))
            d = rand_desc(rng, targets, cb[k], ics[k], pos=int(rng.integers(len(ids) + 1)),
                          ind_sw=1 if (f == 1 and k == 0) else 0)
            lst.append((d, q[k], sf[k], cb[k], ics[k]))
        # bitstream order: the writer puts each CCE before its `pos`-th channel element
        per_frame.append(sorted(lst, key=lambda e: int(e[0]["pos"])))
    return b, ids, elements, per_frame


@pytest.mark.parametrize("cc", [1, 2, 6])
def test_cce_parse_matches_the_restatement(cc):
    b, ids, elements, per_frame = coupled_frames(cc, 6, seed=cc)
    frames = O.write_frames_cce(b, 3, ids, per_frame)
    cfg = N.make_cfg(sf_index=3, channel_config=cc)
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    got = P.parse(frames)
    for k in ("q", "sf", "cb"):
        assert getattr(got, k).tobytes() == getattr(b, k).tobytes(), k
    assert got.cce_terms is not None
    r = 0
    for f, lst in enumerate(per_frame):
        recs = [(q, sf, cb, ics) for _, q, sf, cb, ics in lst]
        for k, (q, sf, cb, ics) in enumerate(recs):
            assert (got.cce_q[r + k] == q).all() and (got.cce_sf[r + k] == sf).all() and (got.cce_cb[r + k] == cb).all()
            g = got.cce_ics[r + k]
            for fld in ("window_sequence", "window_shape", "max_sfb", "grouping"):
                assert g[fld] == ics[fld], fld
        want = ref_terms([d for d, *_ in lst], recs, elements)
        mine = got.cce_terms[got.cce_terms["frame"] == f]
        assert len(mine) == len(want), (f, len(mine), len(want))
        for t, (ch, point, k, g) in zip(mine, want):
            assert (int(t["channel"]), int(t["point"]), int(t["cce"])) == (ch, point, r + k)
            assert t["gain"].tobytes() == g.tobytes()
        r += len(recs)
    assert len(got.cce_ics) == r


def test_lfe_and_sce_share_a_target_tag():
    """The reference matches a non-pair CCE target by tag only: SCE 0 and LFE 0 of a 5.1 frame
    are both coupled (ChannelElement.processDependentCoupling; LFE extends SCE)."""
    b, ids, elements, _ = coupled_frames(6, 1, seed=7)
    q, sf, cb, ics = cce_records(1, 3)
    d = rand_desc(np.random.default_rng(1), [(0, 0, 0)], cb[0], ics[0], pos=0)
    frames = O.write_frames_cce(b, 3, ids, [[(d, q[0], sf[0], cb[0], ics[0])]])
    P = N.Parser(N.make_cfg(sf_index=3, channel_config=6))
    got = P.parse(frames)
    assert sorted(got.cce_terms["channel"].tolist()) == [0, 5]  # SCE (channel 0) and LFE (channel 5)


def test_independent_switching_cce_applies_nowhere():
    b, ids, elements, _ = coupled_frames(2, 1, seed=3)
    q, sf, cb, ics = cce_records(1, 5)
    d = rand_desc(np.random.default_rng(2), [(1, 0, 3)], cb[0], ics[0], pos=1, ind_sw=1)
    got = N.Parser(N.make_cfg(sf_index=3, channel_config=2)).parse(
        O.write_frames_cce(b, 3, ids, [[(d, q[0], sf[0], cb[0], ics[0])]]))
    assert got.n_cce == 1 and len(got.cce_terms) == 0


def test_zero_gain_term_leaves_the_int16_pcm_unchanged():
    """Oracle structure check: a term with all gains 0 adds +-0 (int16 PCM unchanged)."""
    p = N.synth_params(2, n_streams=1, frames_per_stream=8)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    q, sf, cb, ics = cce_records(1, 1)
    b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics = q, sf, cb, ics
    t = np.zeros(2, N.CCE_TERM_DTYPE)
    t["frame"] = [3, 5]
    t["channel"] = [0, 1]
    b.cce_terms = t
    got = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    assert (got == want).all()
    t["gain"][0][:] = 1.0
    got2 = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    assert (got2[3] != want[3]).any() and (got2[:3] == want[:3]).all()


# ------------------------------------------------------------------------------------------------
# GPU: coupling batches against the restatement
# ------------------------------------------------------------------------------------------------

def coupled_batch(cc, n_streams, fps, seed, pns=10):
    """A synthetic batch with random coupling: ~half the frames carry 1-3 terms on random target
    channels with random band gains (negative, zero, large), CCE records with noise bands."""
    rng = np.random.default_rng(seed)
    if cc in N.MC_ELEMENTS:
        from tests.test_multichannel import mc_synth
        b = mc_synth(cc, n_streams=n_streams, fps=fps, seed=seed)
    else:
        p = N.synth_params(3, n_streams=n_streams, frames_per_stream=fps, channel_config=cc)
        p.seed ^= seed
        b = N.synth_batch(p)
    n_rec = max(4, b.n_frames // 4)
    b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics = cce_records(n_rec, seed, pns=pns)
    terms = []
    for f in range(b.n_frames):
        if rng.integers(2):
            continue
        for _ in range(int(rng.integers(1, 4))):
            t = np.zeros((), N.CCE_TERM_DTYPE)
            t["frame"], t["channel"], t["point"] = f, rng.integers(b.nch), rng.integers(2)
            t["cce"] = rng.integers(n_rec)
            t["gain"] = rng.choice([0.0, 1.0, -0.5, 2.0, -3.25, 1.0905077], 120).astype(np.float32)
            terms.append(t)
    b.cce_terms = np.array(terms, N.CCE_TERM_DTYPE)
    return b


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [1, 2])
@pytest.mark.parametrize("flags", [N.PCM_BIG_ENDIAN, N.PCM_FLOAT32])
def test_gpu_coupling_matches_oracle(cc, flags):
    b = coupled_batch(cc, n_streams=6, fps=40, seed=11 + cc)
    cfg = N.make_cfg(channel_config=cc)
    with N.Context(cfg, 6) as ctx:
        got = ctx.decode(b, flags)
    want = O.decode_batch(cfg, b, O.Streams(6), flags, threads=8)
    assert (got == want).all(), np.flatnonzero(got.reshape(-1) != want.reshape(-1))[:8]


@pytest.mark.gpu
def test_gpu_coupling_multichannel_and_device_entry():
    import torch
    b = coupled_batch(6, n_streams=3, fps=30, seed=5)
    cfg = N.make_cfg(channel_config=6)
    with N.Context(cfg, 3) as ctx:
        got = ctx.decode(b, N.PCM_BIG_ENDIAN)
    want = O.decode_batch_mc(3, b, N.MC_ELEMENTS[6], N.PCM_BIG_ENDIAN, threads=8)
    assert (got == want).all()
    # the device-resident entry: records on the device, terms on the host
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).reshape(-1).view(np.uint8)).to(dev)
    d = {k: t(getattr(b, k)) for k in ("q", "sf", "cb", "ics", "ms_used", "cce_q", "cce_sf", "cce_cb", "cce_ics")}
    ptr = {k: v.data_ptr() for k, v in d.items()}
    nb = N.pcm_frame_bytes(0) * 3
    pcm = torch.empty(b.n_frames * nb, dtype=torch.uint8, device=dev)
    with N.Context(cfg, 3) as ctx:
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), N.PCM_BIG_ENDIAN)
        ctx.wait()
    assert (pcm.cpu().numpy().reshape(b.n_frames, -1) == want).all()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [1, 2])
def test_gpu_coupling_with_spec_tns_matches_oracle(cc):
    """JAAD_TNS_SPEC with coupling: BEFORE_TNS terms, the TNS filters, AFTER_TNS terms
    (A/syntax/CPE.java:172-179; oracle/jaad_oracle.c orc_couple / orc_tns_spec), long and short
    windows, frames with terms at both points on one channel."""
    b = coupled_batch(cc, n_streams=6, fps=40, seed=50 + cc)
    assert (b.ics["flags"] & N.ICS_TNS).any() and (b.cce_terms["point"] == 1).any()
    cfg = N.make_cfg(channel_config=cc, tns_mode=N.TNS_SPEC)
    want = O.decode_batch(cfg, b, O.Streams(6), N.PCM_BIG_ENDIAN, threads=8)
    with N.Context(cfg, 6) as ctx:
        got = ctx.decode(b, N.PCM_BIG_ENDIAN)
    assert (got == want).all(), np.flatnonzero((got != want).any(1))[:8]
    # the AFTER_TNS point is not the BEFORE_TNS one once the filters are live
    b.cce_terms["point"] ^= 1
    assert (O.decode_batch(cfg, b, O.Streams(6), N.PCM_BIG_ENDIAN, threads=8) != want).any()
    with N.Context(cfg, 6) as ctx:
        assert (ctx.decode(b, N.PCM_BIG_ENDIAN) == O.decode_batch(cfg, b, O.Streams(6), N.PCM_BIG_ENDIAN, threads=8)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [3, 4, 5, 6, 7])
def test_gpu_multichannel_coupling_with_spec_tns_matches_oracle(cc):
    """JAAD_TNS_SPEC with coupling in configurations 3-7.  The reference couples around
    TNS per channel element (SCE.process / CPE.process: BEFORE_TNS terms, the element's TNS filters,
    AFTER_TNS terms, A/syntax/SCE.java:100-108, CPE.java:172-179, CCE.java:188-215); the GPU runs
    kernel mode 3 per element with the terms' channels relative to the element.  Bit-exact against
    the restatement (oracle.decode_batch_mc, element by element), through the host entry and with
    the AFTER_TNS / BEFORE_TNS points swapped (they differ once the filters are live)."""
    from tests.test_multichannel import IDS
    b = coupled_batch(cc, n_streams=4, fps=30, seed=80 + cc)
    assert (b.ics["flags"] & N.ICS_TNS).any() and (b.cce_terms["point"] == 1).any()
    cfg = N.make_cfg(channel_config=cc, tns_mode=N.TNS_SPEC)
    for swap in (False, True):
        if swap:
            b.cce_terms["point"] ^= 1
        want = O.decode_batch_mc(3, b, IDS[cc], N.PCM_BIG_ENDIAN, threads=8, tns_mode=N.TNS_SPEC)
        with N.Context(cfg, 4) as ctx:
            got = ctx.decode(b, N.PCM_BIG_ENDIAN)
        assert (got == want).all(), (swap, np.flatnonzero((got != want).any(1))[:8])
        if not swap:
            first = want
    assert (first != want).any()  # the coupling point matters once the TNS filters run


@pytest.mark.gpu
def test_gpu_coupling_rejections():
    b = coupled_batch(2, n_streams=2, fps=8, seed=2)
    with N.Context(N.make_cfg(channel_config=2), 2) as ctx:
        bad = b.cce_terms.copy()
        bad = bad[::-1].copy()  # not sorted by frame
        b2 = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, None,
                     b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics, bad)
        with pytest.raises(N.JaadError) as e:
            ctx.decode(b2)
        assert e.value.status == N.ERR_INVALID_ARG


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [2, 6])
def test_gpu_bitstream_with_cce_through_the_decoder_facade(cc):
    """ADTS frames with CCEs -> ADTSDemultiplexer + Decoder.decodeFrame: the PCM equals the
    restatement on the parsed records and terms."""
    from jaadec_amd.decoder import ADTSDemultiplexer, Decoder, SampleBuffer
    b, ids, elements, per_frame = coupled_frames(cc, 8, seed=20 + cc)
    frames = O.write_frames_cce(b, 3, ids, per_frame)
    parsed = N.Parser(N.make_cfg(sf_index=3, channel_config=cc))
    parsed.pns_state = int(b.ics["pns_state"][0])
    pb = parsed.parse(frames)
    assert pb.cce_terms is not None and len(pb.cce_terms)
    cfg = N.make_cfg(sf_index=3, channel_config=cc)
    if cc in N.MC_ELEMENTS:
        want = O.decode_batch_mc(3, pb, N.MC_ELEMENTS[cc], N.PCM_BIG_ENDIAN)
    else:
        want = O.decode_batch(cfg, pb, O.Streams(1), N.PCM_BIG_ENDIAN)
    demux = ADTSDemultiplexer(O.adts_wrap(frames, 3, cc))
    dec = Decoder.create(demux.getDecoderInfo())
    dec._parse([])
    dec._parser.pns_state = int(b.ics["pns_state"][0])
    for i in range(len(frames)):
        buf = SampleBuffer()
        dec.decodeFrame(demux.readNextFrame(), buf)
        assert buf.getData() == want[i].tobytes(), i
    dec.close()


# ------------------------------------------------------------------------------------------------
# limits (jaad_gpu.h JAAD_CCE_GAIN_MAX, JAAD_CCE_MAX_RECORDS)
# ------------------------------------------------------------------------------------------------

def big_gain_frames(total_code):
    """One stereo frame with a CCE whose per-band gain walk (scale 2, sign coding off) reaches
    xg = total_code: its last band's gain is 2^-total_code, as CCE.decode computes it."""
    b, ids, elements, _ = coupled_frames(2, 1, seed=9)
    q, sf, cb, ics = cce_records(1, 4, short=0)
    d = rand_desc(np.random.default_rng(5), [(1, 0, 3)], cb[0], ics[0], pos=1)
    d["sign"], d["scale"] = 1, 3
    d["cge"][1] = 0
    nb = nbands(ics[0])
    coded = [i for i in range(nb) if cb[0][i] != 0]
    assert len(coded) >= 3
    codes = np.zeros(120, np.int32)
    step = int(np.sign(total_code)) * 60
    left = total_code
    for i in coded:
        c = max(-60, min(60, left)) if step > 0 else min(60, max(-60, left))
        codes[i] = c
        left -= c
    assert left == 0
    d["code"][1][:] = codes
    return O.write_frames_cce(b, 3, ids, [[(d, q[0], sf[0], cb[0], ics[0])]])


def test_cce_gain_beyond_the_bound_is_refused():
    """a gain walk past 2^60 would carry inf/NaN into the spectrum, the IMDCT and the
    overlap state: the parser refuses it (JAAD_ERR_UNSUPPORTED); one inside the bound parses."""
    P = N.Parser(N.make_cfg(sf_index=3, channel_config=2))
    got = P.parse(big_gain_frames(-60))  # gain 2^60: the bound itself
    assert np.abs(got.cce_terms["gain"]).max() == np.float32(2.0 ** 60)
    with pytest.raises(N.JaadError) as e:
        N.Parser(N.make_cfg(sf_index=3, channel_config=2)).parse(big_gain_frames(-61))
    assert e.value.status == N.ERR_UNSUPPORTED
    with pytest.raises(N.JaadError) as e:
        N.Parser(N.make_cfg(sf_index=3, channel_config=2)).parse(big_gain_frames(-180))  # 2^180: inf as a float
    assert e.value.status == N.ERR_UNSUPPORTED


def test_cce_record_count_limit_in_parse(monkeypatch):
    """jaad_cce_term.cce is 16-bit; Parser.parse raises instead of wrapping the record
    index (the limit lowered to 2 records so the test stays small)."""
    b, ids, elements, per_frame = coupled_frames(2, 4, seed=2)
    frames = O.write_frames_cce(b, 3, ids, per_frame)
    monkeypatch.setattr(N, "CCE_MAX_RECORDS", 2)
    P = N.Parser(N.make_cfg(sf_index=3, channel_config=2))
    P.pns_state = int(b.ics["pns_state"][0])
    with pytest.raises(N.JaadError) as e:
        P.parse(frames)
    assert e.value.status == N.ERR_UNSUPPORTED


@pytest.mark.gpu
def test_gpu_coupling_rejects_bad_gains_and_too_many_records():
    b = coupled_batch(2, n_streams=2, fps=8, seed=3)
    with N.Context(N.make_cfg(channel_config=2), 2) as ctx:
        for bad in (np.inf, np.nan, 2.0 ** 61):
            t = b.cce_terms.copy()
            t["gain"][0][5] = bad
            b2 = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, None,
                         b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics, t)
            with pytest.raises(N.JaadError) as e:
                ctx.decode(b2)
            assert e.value.status == N.ERR_UNSUPPORTED, bad
        # more records than the 16-bit index can address
        n = N.CCE_MAX_RECORDS + 1
        cq = np.zeros((n, 1024), np.int16)
        csf = np.zeros((n, 128), np.uint8)
        ccb = np.zeros((n, 128), np.uint8)
        cics = np.zeros(n, N.ICS_DTYPE)
        b3 = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, None,
                     cq, csf, ccb, cics, b.cce_terms)
        with pytest.raises(N.JaadError) as e:
            ctx.decode(b3)
        assert e.value.status == N.ERR_UNSUPPORTED
        # the context still decodes a good batch afterwards
        want = O.decode_batch(N.make_cfg(channel_config=2), b, O.Streams(2), N.PCM_BIG_ENDIAN)
        assert (ctx.decode(b) == want).all()


# ------------------------------------------------------------------------------------------------
# coupling with SBR: the reference couples the core spectrum before its SBR runs (A/syntax/CPE.java:
# 172-179 then :195-204; SCE.java:100-108 then :122-132)
# ------------------------------------------------------------------------------------------------

def coupled_sbr_batch(cc, n_streams, fps, seed):
    """An HE-AAC batch (mono / stereo SBR, or multichannel SBR) with random coupling terms."""
    rng = np.random.default_rng(seed)
    if cc in N.MC_ELEMENTS:
        from tests.test_mc_sbr import mc_sbr_synth
        b = mc_sbr_synth(cc, n_streams=n_streams, fps=fps, seed=seed)
    else:
        p = N.synth_params(4, n_streams=n_streams, frames_per_stream=fps, channel_config=cc)
        p.seed ^= seed
        b = N.synth_batch(p)
    n_rec = max(4, b.n_frames // 4)
    b.cce_q, b.cce_sf, b.cce_cb, b.cce_ics = cce_records(n_rec, seed, pns=10, sf_index=6)
    terms = []
    for f in range(b.n_frames):
        if rng.integers(2):
            continue
        for _ in range(int(rng.integers(1, 4))):
            t = np.zeros((), N.CCE_TERM_DTYPE)
            t["frame"], t["channel"], t["point"] = f, rng.integers(b.nch), rng.integers(2)
            t["cce"] = rng.integers(n_rec)
            t["gain"] = rng.choice([0.0, 1.0, -0.5, 2.0, -3.25, 1.0905077], 120).astype(np.float32)
            terms.append(t)
    b.cce_terms = np.array(terms, N.CCE_TERM_DTYPE)
    return b


def test_cce_with_sbr_parses():
    """A stereo HE-AAC frame with a CCE: the CCE and the SBR payload (which attaches to the last
    channel element, not to the CCE) both parse."""
    from tests.test_parse_sbr import _assert_sbr_equal
    p = N.synth_params(4, n_streams=1, frames_per_stream=4, channel_config=2)
    b = N.synth_batch(p)
    rng = np.random.default_rng(3)
    per_frame = []
    for f in range(4):
        q, sf, cb, ics = cce_records(1, 40 + f, sf_index=6)
        d = rand_desc(rng, [(1, 0, 3)], cb[0], ics[0], pos=int(rng.integers(2)))
        per_frame.append([(d, q[0], sf[0], cb[0], ics[0])])
    cfg = N.cfg_for(p)
    frames = O.write_frames_cce(b, p.sf_index, (1,), per_frame, sbr_writers=[O.SbrWriter(cfg.ext_sf_index, 5)])
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    got = P.parse(frames)
    assert got.q.tobytes() == b.q.tobytes() and got.n_cce == 4 and len(got.cce_terms) >= 4
    _assert_sbr_equal(got.sbr, b.sbr, 2, cfg.ext_sf_index)


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [1, 2, 6])
def test_gpu_coupling_with_sbr_matches_oracle(cc):
    b = coupled_sbr_batch(cc, n_streams=4, fps=16, seed=30 + cc)
    if cc in N.MC_ELEMENTS:
        cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
        want = O.decode_batch_mc(6, b, N.MC_ELEMENTS[cc], N.PCM_BIG_ENDIAN, threads=8, sbr=True)
    else:
        cfg = N.make_cfg(sf_index=6, channel_config=cc, sbr=True)
        want = O.decode_batch(cfg, b, O.Streams(4), N.PCM_BIG_ENDIAN, threads=8)
    with N.Context(cfg, 4) as ctx:
        got = ctx.decode(b, N.PCM_BIG_ENDIAN)
    assert (got == want).all(), np.flatnonzero((got != want).any(1))[:8]
