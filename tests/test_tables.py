"""The reference's constant tables, carried as data (jaadec_amd/csrc/tables/jaad_tables.inc),
re-derived from their closed forms."""
import re
from pathlib import Path

import numpy as np
import pytest

INC = Path(__file__).resolve().parents[1] / "jaadec_amd" / "csrc" / "tables" / "jaad_tables.inc"


def table(name):
    src = INC.read_text()
    m = re.search(r"static const (?:float|short|unsigned char) " + name + r"\[[^=]*=\s*\{(.*?)\};", src, re.S)
    assert m, name
    toks = re.findall(r"-?0x[0-9a-fA-Fp+\-.]+f|-?\d+\.\d+f|-?\d+", m.group(1))
    out = []
    for t in toks:
        if "x" in t:
            out.append(float.fromhex(t[:-1]))
        elif t.endswith("f"):
            out.append(float(t[:-1]))
        else:
            out.append(float(t))
    return np.array(out)


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def test_iq_table_is_f32_of_i_pow_4_3():
    # A/syntax/IQTable.java: 8191 entries, IQ[i] = i^(4/3)
    iq = table("JAAD_IQ_TABLE").astype(np.float32)
    assert iq.size == 8191
    i = np.arange(8191, dtype=np.float64)
    assert (iq == np.float32(i ** (4.0 / 3.0))).all()


def test_scalefactor_table_is_pow2_quarter():
    # A/syntax/ScaleFactorTable.java: 2^((i-200)/4)
    sf = table("JAAD_SCALEFACTOR_TABLE").astype(np.float32)
    assert sf.size == 428
    j = np.arange(428)
    assert (sf == np.float32(2.0 ** ((j - 200) / 4.0))).all()


@pytest.mark.parametrize("name,N", [("JAAD_MDCT_TABLE_2048", 2048), ("JAAD_MDCT_TABLE_128", 256)])
def test_mdct_twiddles_closed_form(name, N):
    # MDCTTables: sqrt(2/N) * (cos, sin)(2 pi (k + 1/8) / N)
    t = table(name).astype(np.float32).reshape(-1, 2)
    k = np.arange(N // 4)
    a = 2 * np.pi * (k + 0.125) / N
    assert (t[:, 0] == np.float32(np.sqrt(2.0 / N) * np.cos(a))).all()
    assert (t[:, 1] == np.float32(np.sqrt(2.0 / N) * np.sin(a))).all()


@pytest.mark.parametrize("name,N", [("JAAD_SINE_1024", 1024), ("JAAD_SINE_128", 128)])
def test_sine_windows(name, N):
    w = table(name).astype(np.float32)
    n = np.arange(N)
    assert (w == np.float32(np.sin(np.pi * (n + 0.5) / (2 * N)))).all()


def kbd(N, alpha):
    """Kaiser-Bessel-derived window of length 2N, first half (float64)."""
    n = np.arange(N + 1)
    w = np.i0(np.pi * alpha * np.sqrt(1.0 - ((2.0 * n - N) / N) ** 2))
    c = np.cumsum(w)
    return np.sqrt(c[:N] / c[N])


@pytest.mark.parametrize("name,N,alpha", [("JAAD_KBD_1024", 1024, 4.0), ("JAAD_KBD_128", 128, 6.0)])
def test_kbd_windows_within_one_ulp(name, N, alpha):
    w = table(name).astype(np.float32)
    assert ulp_diff(w, np.float32(kbd(N, alpha))).max() <= 1


def test_fft512_table_is_float32_recurrence():
    """FFT_TABLE_512 is w[k+1] = f32(w[k] * w1), not the closed form."""
    f = table("JAAD_FFT_TABLE_512").astype(np.float32).reshape(-1, 3)
    wr, wi = f[1, 0], f[1, 1]
    cr, ci = np.float32(1), np.float32(0)
    re, im = [cr], [ci]
    for _ in range(1, 512):
        cr, ci = np.float32(np.float32(cr * wr) - np.float32(ci * wi)), np.float32(np.float32(cr * wi) + np.float32(ci * wr))
        re.append(cr)
        im.append(ci)
    assert (f[:, 0] == np.array(re)).all() and (f[:, 1] == np.array(im)).all()
    assert (f[:, 2] == -f[:, 1]).all()
    k = np.arange(512)
    err = np.abs(f[:, 0] - np.cos(2 * np.pi * k / 512)).max()
    assert 1e-6 < err < 2e-5  # the recurrence drifts away from the exact cosine


def test_fft64_table_close_to_exact():
    f = table("JAAD_FFT_TABLE_64").astype(np.float32).reshape(-1, 2)
    k = np.arange(64)
    assert np.abs(f[:, 0] - np.cos(2 * np.pi * k / 64)).max() < 1e-6
    assert np.abs(f[:, 1] - np.sin(2 * np.pi * k / 64)).max() < 1e-6


@pytest.mark.parametrize("name,bits", [("JAAD_TNS_COEF_0_3", 3), ("JAAD_TNS_COEF_0_4", 4)])
def test_tns_tables_are_negated_iso_quantiser(name, bits):
    """TNSTables hold -sin(...) of ISO 14496-3 4.6.9.3's inverse quantiser (spec TNS negates)."""
    t = table(name).astype(np.float32)
    iqfac = ((1 << (bits - 1)) - 0.5) / (np.pi / 2.0)
    iqfac_m = ((1 << (bits - 1)) + 0.5) / (np.pi / 2.0)
    idx = np.arange(1 << bits)
    signed = np.where(idx >= (1 << (bits - 1)), idx - (1 << bits), idx)
    iso = np.sin(signed / np.where(signed >= 0, iqfac, iqfac_m))
    assert np.abs(t + iso).max() < 1e-6


def test_swb_tables_end_at_frame_length():
    for tag, total in (("1024", 1024), ("128", 128)):
        for rate in ("96", "64", "48", "32", "24", "16", "8") if tag == "1024" else ("96", "64", "48", "24", "16", "8"):
            o = table(f"JAAD_SWB_OFFSET_{tag}_{rate}")
            assert o[0] == 0 and o[-1] == total and (np.diff(o) > 0).all() and (o % 4 == 0).all()
