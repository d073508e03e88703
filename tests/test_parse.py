"""Host bitstream front end (include/jaad_parse.h, jaadec_amd/csrc/jaad_parse.cpp).

Pinning: the reference ships no bitstreams, so the parser is checked by round
trips -- synthetic parsed-frame records written as raw_data_blocks by the test writer
(oracle/jaad_writer.c, the reference's own codebooks) must parse back to exactly the same
records -- plus the committed bitstream fixtures (tests/golden/c1_raw_frame.npz,
c3_adts_stream.npz) whose expected PCM is the restatement's decode of those records.
"""
from pathlib import Path

import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

GOLD = Path(__file__).resolve().parent / "golden"


def _nbands(ic):
    ng = 8 - bin(int(ic["grouping"]) & 0x7F).count("1") if ic["window_sequence"] == N.EIGHT_SHORT_SEQUENCE else 1
    return ng * int(ic["max_sfb"])


def _assert_records_equal(got, want):
    for name in ("q", "sf", "cb", "ics"):
        a, b = getattr(got, name), getattr(want, name)
        bad = np.argwhere(a != b)
        assert bad.size == 0, f"{name} differs at {bad[:4].tolist()}"
    if want.ms_used is not None:  # bits beyond the frame's bands carry no meaning
        for f in range(want.n_frames):
            n = _nbands(want.ics[2 * f])
            for i in range(2):
                m = (1 << min(max(n - 64 * i, 0), 64)) - 1
                assert int(got.ms_used[f, i]) & m == int(want.ms_used[f, i]) & m, f"ms_used frame {f}"
    if want.tns is not None and want.tns["n_filters"].any():
        assert got.tns is not None and np.array_equal(got.tns, want.tns)


CASES = {
    "c2_long": (2, dict(n_streams=2, frames_per_stream=6)),
    "c3_switching_tns": (3, dict(n_streams=2, frames_per_stream=30)),
    "mono_switching_pns": (1, dict(n_streams=2, frames_per_stream=20, window_switching=1, pns_percent=8)),
    "pns_is_escapes": (3, dict(n_streams=2, frames_per_stream=24, pns_percent=8, is_percent=15, escape_permille=20)),
    "ms_all_ones": (3, dict(n_streams=1, frames_per_stream=16, ms_mode=2)),
    "independent_windows": (3, dict(n_streams=1, frames_per_stream=16, common_window=0, ms_mode=0, is_percent=10)),
    "other_rate_8k": (3, dict(n_streams=1, frames_per_stream=12, sf_index=11)),
    "other_rate_96k": (3, dict(n_streams=1, frames_per_stream=12, sf_index=0)),
}


@pytest.mark.parametrize("extras", [0, 3], ids=["plain", "dse_fil_pulse"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_write_parse_round_trip(case, extras):
    cfgid, over = CASES[case]
    p = N.synth_params(cfgid, **over)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    for r in range(len(b.stream_slot)):
        want = b.select_runs([r])
        frames = O.write_frames(want, p.sf_index, extras=extras)
        P = N.Parser(cfg)
        P.pns_state = int(want.ics["pns_state"][0])
        got = P.parse(frames, slot=int(want.stream_slot[0]))
        _assert_records_equal(got, want)


def test_adts_split_and_parse():
    p = N.synth_params(3, n_streams=1, frames_per_stream=20)
    b = N.synth_batch(p)
    stream = O.adts_wrap(O.write_frames(b, p.sf_index), p.sf_index, p.channel_config)
    # leading garbage: the sync search skips it (ADTSDemultiplexer.findNextFrame)
    stream = bytes([0x00, 0xFF, 0x12, 0x34]) + stream
    hdrs, payloads = zip(*N.adts_frames(stream))
    assert len(payloads) == 20
    assert {(h.profile, h.sf_index, h.channel_config, h.header_bytes) for h in hdrs} == {(2, 3, 2, 7)}
    cfg = N.adts_cfg(hdrs[0])
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    _assert_records_equal(P.parse(list(payloads)), b)
    # a truncated last frame is not yielded (EOF inside the payload)
    assert len(list(N.adts_frames(stream[:-5]))) == 19


def test_errors_leave_the_parser_state_untouched():
    """A frame that fails with an AACException in the reference (a bitstream error) changes
    nothing: the next good frame parses exactly as if the bad one had never been offered.  A frame
    whose bitstream ends early (EOSException, swallowed by Decoder.decodeFrame, A/Decoder.java:96-100)
    moves the state as far as the reference's reads got (tests/test_frame_status.py); restoring a
    snapshot taken before it undoes that."""
    p = N.synth_params(1, n_streams=1, frames_per_stream=12, window_switching=1, pns_percent=10)
    b = N.synth_batch(p)
    frames = O.write_frames(b, p.sf_index)
    cfg = N.cfg_for(p)
    P = N.Parser(cfg)
    P.pns_state = int(b.ics["pns_state"][0])
    out = []
    for i, fr in enumerate(frames):
        if i == 5:
            st = P.pns_state
            snap = P.snapshot()
            with pytest.raises(N.JaadError) as e:
                P.parse([fr[: len(fr) // 2]])
            assert e.value.status == N.ERR_EOS
            P.restore(snap)
            assert P.pns_state == st
            bad = bytearray(fr)
            bad[0] = (bad[0] & 0x1F) | 0x40  # element id SCE -> CCE: its bits do not parse as one
            with pytest.raises(N.JaadError) as e:
                P.parse([bytes(bad)])
            assert e.value.status in (N.ERR_BITSTREAM, N.ERR_EOS, N.ERR_UNSUPPORTED)
            if e.value.status == N.ERR_EOS:
                P.restore(snap)
            assert P.pns_state == st
            bad = bytearray(fr)
            bad[0] = (bad[0] & 0x1F) | 0x20  # element id SCE -> CPE: refused by a mono configuration
            with pytest.raises(N.JaadError) as e:
                P.parse([bytes(bad)])
            assert e.value.status == N.ERR_UNSUPPORTED
            assert P.pns_state == st
            snap.close()
        out.append(P.parse([fr]))
    for i, g in enumerate(out):
        w = b.select_runs([0])
        assert np.array_equal(g.q[0], w.q[i]) and np.array_equal(g.ics, w.ics[i:i + 1])


def test_reserved_codebook_and_unsupported_elements():
    cfg = N.make_cfg(sf_index=4, channel_config=1)
    P = N.Parser(cfg)
    # SCE whose first section uses codebook 12 ("invalid huffman codebook: 12")
    bits = "000" + "0000" + "10000010" + "0" + "00" + "0" + "110001" + "0" + "1100" + "00001"
    raw = int(bits.ljust(64, "0"), 2).to_bytes(8, "big")
    with pytest.raises(N.JaadError) as e:
        P.parse([raw])
    assert e.value.status == N.ERR_BITSTREAM
    # a CPE in a mono configuration, an LFE
    for elem in ("001", "011"):
        raw = int((elem + "0000").ljust(64, "0"), 2).to_bytes(8, "big")
        with pytest.raises(N.JaadError) as e:
            P.parse([raw])
        assert e.value.status == N.ERR_UNSUPPORTED
    # a CCE (one SCE target, an empty ICS) and END: coupling but no audio element
    cce = "010" + "0000" + "0" + "000" + "0" + "0000" + "0" + "0" + "00"
    ics = "00000000" + "0" + "00" + "0" + "000000" + "0" + "0" + "0" + "0"
    raw = int((cce + ics + "111").ljust(64, "0"), 2).to_bytes(8, "big")
    with pytest.raises(N.JaadError) as e:
        P.parse([raw])
    assert e.value.status == N.ERR_BITSTREAM
    # an empty raw_data_block (END only) carries no audio
    with pytest.raises(N.JaadError) as e:
        P.parse([bytes([0xE0])])
    assert e.value.status == N.ERR_BITSTREAM


@pytest.mark.parametrize("asc,want", [
    (bytes([0x11, 0x90]), dict(profile=2, sf_index=3, channel_config=2, sbr=0, ps=0)),      # LC 48k stereo
    (bytes([0x12, 0x08]), dict(profile=2, sf_index=4, channel_config=1, sbr=0, ps=0)),      # LC 44.1k mono (C1)
    (bytes([0x2B, 0x11, 0x88, 0x00]), dict(profile=2, sf_index=6, channel_config=2, sbr=1, ps=0, ext_sf_index=3)),  # AOT 5
    (bytes([0xEB, 0x09, 0x88, 0x00]), dict(profile=2, sf_index=6, channel_config=1, sbr=1, ps=1, ext_sf_index=3)),  # AOT 29
])
def test_audio_specific_config(asc, want):
    cfg = N.asc_parse(asc)
    for k, v in want.items():
        assert getattr(cfg, k) == v, (k, getattr(cfg, k), v)


def test_audio_specific_config_rejections():
    with pytest.raises(N.JaadError) as e:
        N.asc_parse(bytes([0x11, 0x94]))  # frameLengthFlag = 1: 960-sample frames
    assert e.value.status == N.ERR_UNSUPPORTED
    with pytest.raises(N.JaadError) as e:
        N.asc_parse(bytes([0x0A, 0x10]))  # AOT 1 (AAC Main)
    assert e.value.status == N.ERR_UNSUPPORTED


def test_parser_exports():
    L = N.lib()
    for name in N.PARSE_EXPORTS:
        assert hasattr(L, name), name


def test_c1_raw_frame_fixture_parses_to_the_golden_pcm():
    """C1: one raw AAC-LC 44.1 kHz mono frame -> records -> restatement PCM == the fixture."""
    z = np.load(GOLD / "c1_raw_frame.npz", allow_pickle=False)
    sf_index, chc, pns0, nframes = (int(v) for v in z["meta"])
    cfg = N.make_cfg(sf_index=sf_index, channel_config=chc)
    P = N.Parser(cfg)
    P.pns_state = pns0
    b = P.parse([z["data"].tobytes()])
    got = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    assert got.tobytes() == z["pcm"].tobytes()


def test_c3_adts_fixture_parses_to_the_golden_pcm():
    z = np.load(GOLD / "c3_adts_stream.npz", allow_pickle=False)
    sf_index, chc, pns0, nframes = (int(v) for v in z["meta"])
    hdrs, payloads = zip(*N.adts_frames(z["data"].tobytes()))
    assert len(payloads) == nframes
    cfg = N.adts_cfg(hdrs[0])
    P = N.Parser(cfg)
    P.pns_state = pns0
    b = P.parse(list(payloads))
    got = O.decode_batch(cfg, b, O.Streams(1), N.PCM_BIG_ENDIAN)
    assert got.tobytes() == z["pcm"].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_raw_frame", "c3_adts_stream"])
def test_bitstream_fixtures_on_the_gpu(name):
    """Bitstream -> host parser -> HIP DSP path == the golden PCM, byte for byte."""
    z = np.load(GOLD / f"{name}.npz", allow_pickle=False)
    sf_index, chc, pns0, nframes = (int(v) for v in z["meta"])
    data = z["data"].tobytes()
    if name.endswith("adts_stream"):
        hdrs, payloads = zip(*N.adts_frames(data))
        cfg = N.adts_cfg(hdrs[0])
    else:
        payloads, cfg = [data], N.make_cfg(sf_index=sf_index, channel_config=chc)
    P = N.Parser(cfg)
    P.pns_state = pns0
    b = P.parse(list(payloads))
    with N.Context(cfg, 1) as ctx:
        got = ctx.decode(b, N.PCM_BIG_ENDIAN)
    assert got.tobytes() == z["pcm"].tobytes()


def test_pulse_data_is_applied_only_in_spec_mode():
    """The reference parses pulse_data and never applies it (A/syntax/ICStream.java:148-170);
    with cfg.tns_mode = JAAD_TNS_SPEC (spec tools) the parser adds the pulses to the quantised
    values as ISO/IEC 14496-3 4.6.3.3 does: q[k] += amp if q[k] > 0 else q[k] -= amp.
    The test writer puts 2 pulses at swb 0: offset 3 (amp 5) and 3 + 7 = 10 (amp 2)."""
    p = N.synth_params(2, n_streams=1, frames_per_stream=4)
    b = N.synth_batch(p)
    frames = O.write_frames(b, p.sf_index, extras=2)
    compat = N.Parser(N.cfg_for(p)).parse(frames)
    assert np.array_equal(compat.q, b.q)
    spec = N.Parser(N.cfg_for(p, tns_mode=N.TNS_SPEC)).parse(frames)
    want = b.q.astype(np.int32).copy()
    for row in want:
        for k, amp in ((3, 5), (10, 2)):
            row[k] = row[k] + amp if row[k] > 0 else row[k] - amp
    assert np.array_equal(spec.q.astype(np.int32), want)


def test_parser_snapshot_and_restore():
    """jaad_parser_clone / jaad_parser_copy: a batch parsed after a restore is byte-identical to
    the first parse (window shapes, PNS LCG and SBR history all rolled back)."""
    p = N.synth_params(4, n_streams=1, frames_per_stream=8)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    frames = O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 3))
    P = N.Parser(cfg)
    P.parse(frames[:3])
    snap = P.snapshot()
    first = P.parse(frames[3:])
    P.restore(snap)
    again = P.parse(frames[3:])
    for k in ("q", "sf", "cb", "ics", "ms_used", "sbr"):
        assert getattr(first, k).tobytes() == getattr(again, k).tobytes(), k
    other = N.Parser(N.make_cfg(3, 2))
    with pytest.raises(N.JaadError):
        other.restore(snap)  # a snapshot of another configuration
    snap.close()


@pytest.mark.parametrize("cfgid", [2, 3, 4, 5])
def test_parse_corpus_round_trips_and_times(cfgid):
    """The host front-end corpus (tests/golden/parse_c*.bin, bench.py host_front_end) parses back to
    the synthetic records it was written from, and tools/bench_parse times it without an error."""
    import json
    import struct
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    data = (root / "tests" / "golden" / f"parse_c{cfgid}.bin").read_bytes()
    n = struct.unpack_from("<I", data, 4)[0]
    cfg = N.StreamCfg.from_buffer_copy(data[8:8 + n])
    at = 8 + n
    streams, fps = struct.unpack_from("<II", data, at)
    at += 8
    p = N.synth_params(cfgid, n_streams=streams, frames_per_stream=fps)
    b = N.synth_batch(p)
    for s in range(streams):
        pns = struct.unpack_from("<I", data, at)[0]
        at += 4
        frames = []
        for _ in range(fps):
            ln = struct.unpack_from("<I", data, at)[0]
            frames.append(data[at + 4:at + 4 + ln])
            at += 4 + ln
        P = N.Parser(cfg)
        P.pns_state = pns
        got = P.parse(frames)
        P.close()
        c0, c1 = int(b.frame_begin[s]) * b.nch, int(b.frame_begin[s + 1]) * b.nch
        assert (got.q == b.q[c0:c1]).all() and (got.sf == b.sf[c0:c1]).all() and (got.cb == b.cb[c0:c1]).all()
    tool = root / "tools" / "bench_parse"
    if not tool.exists():
        pytest.skip("tools/bench_parse not built")
    r = subprocess.run([str(tool), str(root / "tests" / "golden" / f"parse_c{cfgid}.bin"), "2", "0.1"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout)
    assert line["frames"] > 0 and line["frames_per_s"] > 0
