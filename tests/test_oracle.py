"""The C restatement (oracle/) against independent float64 closed forms and Java semantics.

The reference ships no golden vectors and cannot run here, so these checks
pin the restatement instead: FFT vs numpy, IMDCT vs its closed form, the four window sequences
vs the ISO 14496-3 block-switching definition, IQ/PNS/M-S/I-S arithmetic, Math.round + short
clamp + byte order of SampleBuffer.accept.
"""
import ctypes as C

import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

from test_tables import kbd, table

RNG = np.random.default_rng(20261015)


@pytest.mark.parametrize("n", [64, 512])
def test_fft_inverse_matches_numpy(n):
    """FFT.process(..., false) = non-scaled sum x[j] e^{+2 pi i jk/n} (A/filterbank/FFT.java:48-135)."""
    x = RNG.standard_normal(n) + 1j * RNG.standard_normal(n)
    got = O.fft(x, forward=False)
    want = np.fft.ifft(x) * n
    assert np.abs(got - want).max() / np.abs(want).max() < 3e-5


def test_fft_forward_matches_numpy():
    x = RNG.standard_normal(512) + 1j * RNG.standard_normal(512)
    got = O.fft(x, forward=True)
    want = np.fft.fft(x)
    assert np.abs(got - want).max() / np.abs(want).max() < 3e-5


def imdct_closed(X):
    """(2/N) sum_k X[k] cos(2 pi / N (n + n0)(k + 1/2)), n0 = (N/2 + 1)/2."""
    N = 2 * len(X)
    n = np.arange(N)[:, None]
    k = np.arange(N // 2)[None, :]
    n0 = (N / 2 + 1) / 2
    return (2.0 / N) * (np.cos(2 * np.pi / N * (n + n0) * (k + 0.5)) @ X)


@pytest.mark.parametrize("n", [1024, 128])
def test_imdct_closed_form(n):
    X = RNG.standard_normal(n) * 1000
    got = O.imdct(X.astype(np.float32)).astype(np.float64)
    want = imdct_closed(X.astype(np.float32).astype(np.float64))
    rel = np.abs(got - want).max() / np.abs(want).max()
    assert rel < (2e-5 if n == 1024 else 2e-6), rel


def windows():
    s_long = np.sin(np.pi * (np.arange(1024) + 0.5) / 2048)
    s_short = np.sin(np.pi * (np.arange(128) + 0.5) / 256)
    return [s_long, kbd(1024, 4.0)], [s_short, kbd(128, 6.0)]


def iso_frame(seq, shape, prev, X):
    """Windowed 2048-sample IMDCT output of one frame by the ISO 14496-3 block-switching rules."""
    LW, SW = windows()
    out = np.zeros(2048)
    if seq == N.EIGHT_SHORT_SEQUENCE:
        for w in range(8):
            y = imdct_closed(X[128 * w:128 * (w + 1)])
            rise = SW[prev if w == 0 else shape]
            win = np.concatenate([rise, SW[shape][::-1]])
            out[448 + 128 * w:448 + 128 * w + 256] += y * win
        return out
    y = imdct_closed(X)
    if seq in (N.ONLY_LONG_SEQUENCE, N.LONG_START_SEQUENCE):
        first = LW[prev]
    else:  # LONG_STOP
        first = np.concatenate([np.zeros(448), SW[prev], np.ones(448)])
    if seq in (N.ONLY_LONG_SEQUENCE, N.LONG_STOP_SEQUENCE):
        second = LW[shape][::-1]
    else:  # LONG_START
        second = np.concatenate([np.ones(448), SW[shape][::-1], np.zeros(448)])
    return y * np.concatenate([first, second])


def test_filterbank_window_sequences_match_iso_definition():
    """FilterBank.process over an OL/LS/ES/ES/LT/... chain with shape changes."""
    seqs = [0, 1, 2, 2, 3, 0, 0, 1, 2, 3, 1, 2, 3, 0]
    shapes = RNG.integers(0, 2, len(seqs))
    ov = np.zeros(1024, np.float32)
    ov64 = np.zeros(1024)
    prev = 0
    worst = 0.0
    for seq, shape in zip(seqs, shapes):
        X = (RNG.standard_normal(1024) * 2000).astype(np.float32)
        got = O.filterbank(seq, int(shape), prev, X, ov)
        full = iso_frame(seq, int(shape), prev, X.astype(np.float64))
        want = ov64 + full[:1024]
        ov64 = full[1024:]
        worst = max(worst, np.abs(got - want).max() / np.abs(want).max())
        prev = int(shape)
    assert worst < 3e-5, worst


def _one_ics(seq, max_sfb, grouping=0, pns_state=0x1F2E3D4C, flags=0):
    ic = np.zeros(1, N.ICS_DTYPE)
    ic["window_sequence"], ic["max_sfb"], ic["grouping"] = seq, max_sfb, grouping
    ic["pns_state"], ic["flags"] = pns_state, flags
    return ic


def _dequant(ic, q, sf, cb, sf_index=3):
    iq = np.zeros(1024, np.float32)
    rs = np.array([ic["pns_state"][0]], np.uint32)
    rc = O.lib().orc_dequant(ic.ctypes.data, sf_index, q.ctypes.data, sf.ctypes.data, cb.ctypes.data,
                             rs.ctypes.data, iq.ctypes.data)
    assert rc == 0
    return iq, int(rs[0])


def test_dequant_iq_formula_and_zero_tail():
    swb = table("JAAD_SWB_OFFSET_1024_48").astype(int)
    q = RNG.integers(-200, 200, 1024).astype(np.int16)
    sf = RNG.integers(90, 160, 128).astype(np.uint8)
    cb = np.full(128, 11, np.uint8)
    cb[5] = 0  # ZERO_HCB band
    ic = _one_ics(0, 40)
    iq, _ = _dequant(ic, q, sf, cb)
    want = np.zeros(1024)
    for b in range(40):
        if cb[b] == 0:
            continue
        sl = slice(swb[b], swb[b + 1])
        want[sl] = np.sign(q[sl]) * np.abs(q[sl].astype(np.float64)) ** (4 / 3) * 2.0 ** ((int(sf[b]) - 100) / 4)
    assert np.abs(iq - want).max() <= 2e-7 * np.abs(want).max()
    assert (iq[swb[40]:] == 0).all()
    assert (iq[swb[5]:swb[6]] == 0).all()
    # q == 0 in a spectral band is -IQ_TABLE[0] * sf = -0.0 (A/syntax/ICStream.java:266)
    z = np.flatnonzero((q == 0) & (np.arange(1024) < swb[5]))
    if z.size:
        assert np.signbit(iq[z]).all()


def test_pns_lcg_energy_and_state_advance():
    """PNS (ICStream.java:241-257): static LCG, per-window energy normalised to the band gain."""
    swb = table("JAAD_SWB_OFFSET_1024_48").astype(int)
    q = np.zeros(1024, np.int16)
    sf = np.full(128, 120, np.uint8)
    cb = np.full(128, 11, np.uint8)
    noise = [3, 17, 30]
    for b in noise:
        cb[b] = 13
    ic = _one_ics(0, 49)
    iq, rs = _dequant(ic, q, sf, cb)
    state = 0x1F2E3D4C
    for b in noise:
        n = swb[b + 1] - swb[b]
        vals = []
        for _ in range(n):
            state = (1664525 * state + 1013904223) & 0xFFFFFFFF
            vals.append(np.float32(np.int32(np.uint32(state).view(np.int32))))
        v = np.array(vals, np.float64)
        g = -(2.0 ** ((120 - 100) / 4))
        want = v * (g / np.sqrt((np.float32(v) ** 2).astype(np.float64).sum()))
        got = iq[swb[b]:swb[b + 1]]
        assert np.abs(got - want).max() < 1e-5 * np.abs(want).max()
        assert abs(np.sum(got.astype(np.float64) ** 2) - g * g) < 1e-4 * g * g
    assert rs == state


def test_ms_and_is_identities():
    L0 = (RNG.standard_normal(1024) * 100).astype(np.float32)
    R0 = (RNG.standard_normal(1024) * 100).astype(np.float32)
    swb = table("JAAD_SWB_OFFSET_1024_48").astype(int)
    cbL = np.full(128, 11, np.uint8)
    cbR = np.full(128, 11, np.uint8)
    cbR[7] = 13  # noise band: M/S skipped
    cbR[20], cbR[21] = 15, 14  # intensity bands
    ms = np.zeros(2, np.uint64)
    for b in (2, 7, 20, 33):
        ms[b >> 6] |= np.uint64(1 << (b & 63))
    sfR = np.full(128, 95, np.uint8)
    icL = _one_ics(0, 49, flags=N.ICS_MS_PRESENT | N.ICS_COMMON_WINDOW)
    icR = _one_ics(0, 49)
    L, R = L0.copy(), R0.copy()
    lib = O.lib()
    lib.orc_ms.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_is.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_ms(icL.ctypes.data, 3, cbL.ctypes.data, cbR.ctypes.data, ms.ctypes.data, L.ctypes.data, R.ctypes.data)
    lib.orc_is(icL.ctypes.data, icR.ctypes.data, 3, cbR.ctypes.data, sfR.ctypes.data, ms.ctypes.data,
               L.ctypes.data, R.ctypes.data)
    for b in range(49):
        sl = slice(swb[b], swb[b + 1])
        if b in (2, 33):  # M/S: L' = L + R, R' = L - R (no scaling, A/tools/MS.java:31-34)
            assert (L[sl] == L0[sl] + R0[sl]).all() and (R[sl] == L0[sl] - R0[sl]).all()
        elif b in (20, 21):  # I/S: R = L * c * 2^((100-sf)/4 ...); cb15 -> +, cb14 -> -, flipped by ms
            c = (1 if b == 20 else -1) * (-1 if b == 20 else 1)
            g = np.float32(2.0 ** ((int(sfR[b]) - 100) / 4))
            assert (R[sl] == L0[sl] * np.float32(c) * g).all()
        else:
            assert (L[sl] == L0[sl]).all() and (R[sl] == R0[sl]).all()


def test_pcm_pack_java_round_clamp_and_byte_order():
    """Math.round(float) ties toward +inf, NaN -> 0, then the short clamp (S/SampleBuffer.java:193-206)."""
    vals = np.array([0.5, -0.5, 1.5, -1.5, 2.5, -2.5, 0.49999997, -0.49999997, 32767.4, 32767.5, 40000.0,
                     -32768.4, -32768.5, -1e9, np.nan, -0.0, 123.25, -123.75], np.float32)
    want = [1, 0, 2, -1, 3, -2, 0, 0, 32767, 32767, 32767, -32768, -32768, -32768, 0, 0, 123, -124]
    be = O.pcm_pack([vals], flags=N.PCM_BIG_ENDIAN)
    le = O.pcm_pack([vals], flags=N.PCM_LITTLE_ENDIAN)
    assert list(np.frombuffer(be, ">i2")) == want
    assert list(np.frombuffer(le, "<i2")) == want
    f32 = np.frombuffer(O.pcm_pack([vals], flags=N.PCM_FLOAT32), np.float32)
    assert np.array_equal(f32, vals, equal_nan=True)


def test_batch_matches_frame_by_frame_streaming():
    """One batch call == the same frames decoded in two calls with the state carried over."""
    p = N.synth_params(3, n_streams=3, frames_per_stream=14, pns_percent=5, is_percent=10)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    whole = O.decode_batch(cfg, b, O.Streams(3), N.PCM_FLOAT32)
    st = O.Streams(3)
    a, rest = b.split_frames(5)
    pa = O.decode_batch(cfg, a, st, N.PCM_FLOAT32)
    pb = O.decode_batch(cfg, rest, st, N.PCM_FLOAT32)
    fb = b.frame_begin
    i = j = 0
    for r in range(3):
        n = int(fb[r + 1] - fb[r])
        assert (whole[fb[r]:fb[r] + 5] == pa[i:i + 5]).all()
        assert (whole[fb[r] + 5:fb[r + 1]] == pb[j:j + n - 5]).all()
        i += 5
        j += n - 5


def test_multithreaded_oracle_is_identical():
    p = N.synth_params(2, n_streams=8, frames_per_stream=6)
    b = N.synth_batch(p)
    cfg = N.make_cfg()
    one = O.decode_batch(cfg, b, O.Streams(8), 0, threads=1)
    many = O.decode_batch(cfg, b, O.Streams(8), 0, threads=4)
    assert (one == many).all()


def test_synthetic_c2_amplitudes_are_meaningful():
    """PCM RMS in the hundreds..low thousands, no clipping on the C2 recipe."""
    p = N.synth_params(2, n_streams=4, frames_per_stream=8)
    b = N.synth_batch(p)
    pcm = O.decode_batch(N.make_cfg(), b, O.Streams(4), 0).view(">i2").astype(np.float64)
    rms = np.sqrt((pcm ** 2).mean())
    assert 200 < rms < 5000 and np.abs(pcm).max() < 32767
