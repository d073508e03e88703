#!/usr/bin/env python3
"""One-off extractor: reference constant tables -> C data (hex-float literals).

Runs ONLY in the build container (it reads the read-only reference checkout at
/root/reference); its OUTPUT, `jaadec_amd/csrc/tables/jaad_tables.inc`, is the
committed artefact.  SURVEY.md section 0 item 10 / section 7 step 0: the FFT
twiddles come from a float32 recurrence and the KBD windows differ from a float64
derivation in the last ulp, so the reference's float constants are carried over
verbatim as *data* (each decimal literal rounded to the nearest binary32 exactly
as java.lang.Float.parseFloat does) instead of being regenerated.

Every emitted array is re-derived from its closed form in tests/test_tables.py.
"""
from __future__ import annotations

import re
import sys
from fractions import Fraction
from pathlib import Path

import numpy as np

REF = Path("/root/reference/aac/src/main/java/net/sourceforge/jaad/aac")
OUT = Path(__file__).resolve().parents[1] / "jaadec_amd" / "csrc" / "tables" / "jaad_tables.inc"

# (java file, java array name, C name, kind)  kind: f32 | f32x2 (first 2 columns) | f32x3 | i32
TABLES = [
    ("syntax/IQTable.java", "IQ_TABLE", "JAAD_IQ_TABLE", "f32"),
    ("syntax/ScaleFactorTable.java", "SCALEFACTOR_TABLE", "JAAD_SCALEFACTOR_TABLE", "f32"),
    ("filterbank/SineWindows.java", "SINE_1024", "JAAD_SINE_1024", "f32"),
    ("filterbank/SineWindows.java", "SINE_128", "JAAD_SINE_128", "f32"),
    ("filterbank/KBDWindows.java", "KBD_1024", "JAAD_KBD_1024", "f32"),
    ("filterbank/KBDWindows.java", "KBD_128", "JAAD_KBD_128", "f32"),
    ("filterbank/MDCTTables.java", "MDCT_TABLE_2048", "JAAD_MDCT_TABLE_2048", "f32x2"),
    ("filterbank/MDCTTables.java", "MDCT_TABLE_128", "JAAD_MDCT_TABLE_128", "f32x2"),
    ("filterbank/FFTTables.java", "FFT_TABLE_512", "JAAD_FFT_TABLE_512", "f32x3"),
    ("filterbank/FFTTables.java", "FFT_TABLE_64", "JAAD_FFT_TABLE_64", "f32x2"),
    ("tools/TNSTables.java", "TNS_COEF_0_3", "JAAD_TNS_COEF_0_3", "f32"),
    ("tools/TNSTables.java", "TNS_COEF_0_4", "JAAD_TNS_COEF_0_4", "f32"),
    ("tools/TNSTables.java", "TNS_COEF_1_3", "JAAD_TNS_COEF_1_3", "f32"),
    ("tools/TNSTables.java", "TNS_COEF_1_4", "JAAD_TNS_COEF_1_4", "f32"),
]

# SBR (HE-AAC v1) tables -> jaad_sbr_tables.inc.  kind: f32 | f32xN | f32_2d (ragged rows) | i32 | i32_2d
SBR_OUT = OUT.with_name("jaad_sbr_tables.inc")
SBR_TABLES = [
    ("sbr/Filterbank.java", "qmf_c", "JAAD_QMF_C", "f32"),
    ("sbr/DCT.java", "w_array_real", "JAAD_DCT_W_RE", "f32"),
    ("sbr/DCT.java", "w_array_imag", "JAAD_DCT_W_IM", "f32"),
    ("sbr/DCT.java", "dct4_64_tab", "JAAD_DCT4_64_TAB", "f32"),
    ("sbr/DCT.java", "bit_rev_tab", "JAAD_DCT_BIT_REV", "i32"),
    ("sbr/NoiseTable.java", "NOISE_TABLE", "JAAD_SBR_NOISE_TABLE", "f32x2"),
    ("sbr/NoiseEnvelope.java", "E_deq_tab", "JAAD_SBR_E_DEQ", "f32"),
    ("sbr/NoiseEnvelope.java", "Q_div_tab", "JAAD_SBR_Q_DIV", "f32"),
    ("sbr/NoiseEnvelope.java", "Q_div2_tab", "JAAD_SBR_Q_DIV2", "f32"),
    ("sbr/NoiseEnvelope.java", "Q_div_tab_left", "JAAD_SBR_Q_DIV_LEFT", "f32_2d"),
    ("sbr/NoiseEnvelope.java", "Q_div_tab_right", "JAAD_SBR_Q_DIV_RIGHT", "f32_2d"),
    ("sbr/NoiseEnvelope.java", "Q_div2_tab_left", "JAAD_SBR_Q_DIV2_LEFT", "f32_2d"),
    ("sbr/NoiseEnvelope.java", "Q_div2_tab_right", "JAAD_SBR_Q_DIV2_RIGHT", "f32_2d"),
    ("sbr/NoiseEnvelope.java", "E_pan_tab", "JAAD_SBR_E_PAN", "f32"),
    ("sbr/HFAdjustment.java", "h_smooth", "JAAD_SBR_H_SMOOTH", "f32"),
    ("sbr/HFAdjustment.java", "limGain", "JAAD_SBR_LIM_GAIN", "f32"),
    ("sbr/HFGeneration.java", "goalSbTab", "JAAD_SBR_GOAL_SB", "i32"),
    ("sbr/FBT.java", "startMinTable", "JAAD_SBR_START_MIN", "i32"),
    ("sbr/FBT.java", "offsetIndexTable", "JAAD_SBR_OFFSET_INDEX", "i32"),
    ("sbr/FBT.java", "OFFSET", "JAAD_SBR_OFFSET", "i32_2d"),
    ("sbr/FBT.java", "stopMinTable", "JAAD_SBR_STOP_MIN", "i32"),
    ("sbr/FBT.java", "STOP_OFFSET_TABLE", "JAAD_SBR_STOP_OFFSET", "i32_2d"),
    ("sbr/FBT.java", "limiterBandsCompare", "JAAD_SBR_LIMITER_COMPARE", "f32"),
    ("sbr/SynthesisFilterbank32.java", "qmf32_pre_twiddle", "JAAD_QMF32_PRE_TWIDDLE", "f32x2"),
]

# The downsampled synthesis's 32-point DCT-IV / DST-IV (A/sbr/SynthesisFilterbank32.java
# DCT4_32 / DST4_32) are generated straight-line binary32 code.  They are carried as DATA too: an
# op list per transform over one register file -- slots 0..31 = the in/out array (the reference
# calls both in place: DCT4_32(x1, x1)), slot 32 + k = temporary f<k> -- each op
# {kind, dst, a, b}: kind 0 = r[a] - r[b], 1 = r[a] + r[b], 2 = K * r[a] with K the op's constant.
# The oracle interprets the list; the GPU kernel unrolls it at compile time.
DCT32_OUT = OUT.with_name("jaad_sbr_dct32.inc")
DCT32_PROGS = [("DCT4_32", "JAAD_SBR_DCT4_32"), ("DST4_32", "JAAD_SBR_DST4_32")]

# PS (HE-AAC v2) tables -> jaad_ps_tables.inc (f32_flat: all numbers of a nested array, in order)
PS_OUT = OUT.with_name("jaad_ps_tables.inc")
PS_TABLES = [
    ("ps/PSTables.java", "filter_a", "JAAD_PS_FILTER_A", "f32"),
    ("ps/PSTables.java", "group_border20", "JAAD_PS_GROUP_BORDER20", "i32"),
    ("ps/PSTables.java", "delay_length_d", "JAAD_PS_DELAY_LENGTH_D", "i32"),
    ("ps/PSTables.java", "Phi_Fract_Qmf", "JAAD_PS_PHI_FRACT_QMF", "f32_2d"),
    ("ps/PSTables.java", "Phi_Fract_SubQmf20", "JAAD_PS_PHI_FRACT_SUBQMF20", "f32_2d"),
    ("ps/PSTables.java", "Q_Fract_allpass_Qmf", "JAAD_PS_Q_FRACT_ALLPASS_QMF", "f32_flat"),
    ("ps/PSTables.java", "Q_Fract_allpass_SubQmf20", "JAAD_PS_Q_FRACT_ALLPASS_SUBQMF20", "f32_flat"),
    ("ps/PSTables.java", "cos_alphas", "JAAD_PS_COS_ALPHAS", "f32"),
    ("ps/PSTables.java", "sin_alphas", "JAAD_PS_SIN_ALPHAS", "f32"),
    ("ps/PSTables.java", "cos_betas_normal", "JAAD_PS_COS_BETAS_NORMAL", "f32_flat"),
    ("ps/PSTables.java", "sin_betas_normal", "JAAD_PS_SIN_BETAS_NORMAL", "f32_flat"),
    ("ps/PSTables.java", "cos_betas_fine", "JAAD_PS_COS_BETAS_FINE", "f32_flat"),
    ("ps/PSTables.java", "sin_betas_fine", "JAAD_PS_SIN_BETAS_FINE", "f32_flat"),
    ("ps/PSTables.java", "sincos_alphas_B_normal", "JAAD_PS_SINCOS_ALPHAS_B_NORMAL", "f32_flat"),
    ("ps/PSTables.java", "sincos_alphas_B_fine", "JAAD_PS_SINCOS_ALPHAS_B_FINE", "f32_flat"),
    ("ps/PSTables.java", "cos_gammas_normal", "JAAD_PS_COS_GAMMAS_NORMAL", "f32_flat"),
    ("ps/PSTables.java", "cos_gammas_fine", "JAAD_PS_COS_GAMMAS_FINE", "f32_flat"),
    ("ps/PSTables.java", "sin_gammas_normal", "JAAD_PS_SIN_GAMMAS_NORMAL", "f32_flat"),
    ("ps/PSTables.java", "sin_gammas_fine", "JAAD_PS_SIN_GAMMAS_FINE", "f32_flat"),
    ("ps/PSTables.java", "sf_iid_normal", "JAAD_PS_SF_IID_NORMAL", "f32"),
    ("ps/PSTables.java", "sf_iid_fine", "JAAD_PS_SF_IID_FINE", "f32"),
    ("ps/PSTables.java", "ipdopd_cos_tab", "JAAD_PS_IPDOPD_COS", "f32"),
    ("ps/PSTables.java", "ipdopd_sin_tab", "JAAD_PS_IPDOPD_SIN", "f32"),
    ("ps/Filter8.java", "p8_13_20", "JAAD_PS_P8_13_20", "f32"),
    ("ps/Filter2.java", "p2_13_20", "JAAD_PS_P2_13_20", "f32"),
]

# Huffman codebooks -> jaad_huffman_tables.inc (host parser): AAC spectral/scalefactor codebooks
# as {length, codeword, values...} rows (A/huffman/Codebooks.java), SBR and PS binary trees as
# {child0, child1} rows, negative = leaf (A/sbr/HuffmanTables.java, A/ps/Huffman.java)
HUFF_OUT = OUT.with_name("jaad_huffman_tables.inc")
HUFF_TABLES = [("huffman/Codebooks.java", n, "JAAD_" + n, "i32_2d") for n in
               ["HCB1", "HCB2", "HCB3", "HCB4", "HCB5", "HCB6", "HCB7", "HCB8", "HCB9", "HCB10", "HCB11", "HCB_SF"]]
HUFF_TABLES += [("sbr/HuffmanTables.java", n, "JAAD_SBR_" + n, "i32_2d") for n in
                ["T_HUFFMAN_ENV_1_5DB", "F_HUFFMAN_ENV_1_5DB", "T_HUFFMAN_ENV_BAL_1_5DB", "F_HUFFMAN_ENV_BAL_1_5DB",
                 "T_HUFFMAN_ENV_3_0DB", "F_HUFFMAN_ENV_3_0DB", "T_HUFFMAN_ENV_BAL_3_0DB", "F_HUFFMAN_ENV_BAL_3_0DB",
                 "T_HUFFMAN_NOISE_3_0DB", "T_HUFFMAN_NOISE_BAL_3_0DB"]]
HUFF_TABLES += [("ps/Huffman.java", n, "JAAD_PS_" + n.upper(), "i32_2d") for n in
                ["f_huff_iid_def", "t_huff_iid_def", "f_huff_iid_fine", "t_huff_iid_fine", "f_huff_icc", "t_huff_icc",
                 "f_huff_ipd", "t_huff_ipd", "f_huff_opd", "t_huff_opd"]]

SWB = [  # ScaleFactorBands: per sampling-frequency-index offset tables
    ("SWB_OFFSET_1024_96", "SWB_OFFSET_1024_64", "SWB_OFFSET_1024_48", "SWB_OFFSET_1024_32",
     "SWB_OFFSET_1024_24", "SWB_OFFSET_1024_16", "SWB_OFFSET_1024_8"),
    ("SWB_OFFSET_128_96", "SWB_OFFSET_128_64", "SWB_OFFSET_128_48", "SWB_OFFSET_128_24",
     "SWB_OFFSET_128_16", "SWB_OFFSET_128_8"),
]


def f32_from_decimal(tok: str) -> np.float32:
    """Nearest-even binary32 to the exact decimal value (Float.parseFloat semantics)."""
    tok = tok.strip().rstrip("fFdD")
    exact = Fraction(tok)
    if exact == 0:  # Java keeps the sign of a zero literal: -0.0f is negative zero
        return np.float32(-0.0) if tok.lstrip().startswith("-") else np.float32(0.0)
    cand = np.float32(float(exact))  # may suffer double rounding: fix below
    best = None
    for c in (np.nextafter(cand, np.float32(-np.inf)), cand, np.nextafter(cand, np.float32(np.inf))):
        if not np.isfinite(c):
            continue
        err = abs(Fraction(float(c)) - exact)
        key = (err, int(np.frombuffer(np.float32(c).tobytes(), np.uint32)[0]) & 1)
        if best is None or key < best[0]:
            best = (key, np.float32(c))
    return best[1]


def strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def find_array(src: str, name: str) -> str:
    m = re.search(r"\b" + re.escape(name) + r"\s*=\s*\{", src)
    if not m:
        raise KeyError(name)
    i = m.end() - 1
    depth = 0
    for j in range(i, len(src)):
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                return src[i:j + 1]
    raise ValueError("unterminated " + name)


def parse_rows(body: str):
    inner = body.strip()[1:-1]
    if "{" in inner:
        rows = re.findall(r"\{([^{}]*)\}", inner)
        return [[t for t in r.split(",") if t.strip()] for r in rows]
    return [t for t in inner.split(",") if t.strip()]


def hexf(x: np.float32) -> str:
    v = float(x)
    if v == 0.0:
        return "-0.0f" if np.signbit(x) else "0.0f"
    mant, exp = float.hex(v).split("p")
    if "." in mant:
        mant = mant.rstrip("0").rstrip(".")
    return f"{mant}p{exp}f"


def main() -> int:
    out = ["/* GENERATED by tools/extract_tables.py -- binary32 constant tables of the",
           " * reference decoder, carried as data (SURVEY.md s0 item 10). Do not edit. */",
           "#pragma once", ""]
    for fname, jname, cname, kind in TABLES:
        src = strip_comments((REF / fname).read_text())
        rows = parse_rows(find_array(src, jname))
        if kind == "f32":
            vals = [f32_from_decimal(t) for t in rows]
            out.append(f"static const float {cname}[{len(vals)}] = {{")
            for i in range(0, len(vals), 6):
                out.append("  " + ", ".join(hexf(v) for v in vals[i:i + 6]) + ",")
        else:
            ncol = int(kind[-1])
            vals = [[f32_from_decimal(t) for t in r[:ncol]] for r in rows]
            assert all(len(r) == ncol for r in vals), cname
            out.append(f"static const float {cname}[{len(vals)}][{ncol}] = {{")
            for r in vals:
                out.append("  {" + ", ".join(hexf(v) for v in r) + "},")
        out.append("};")
        out.append(f"/* from {fname}:{jname} */")
        out.append("")
    src = strip_comments((REF / "syntax/ScaleFactorBands.java").read_text())
    for group, tag in zip(SWB, ("LONG", "SHORT")):
        for jname in group:
            vals = [int(t) for t in parse_rows(find_array(src, jname))]
            vals = [v for v in vals if v >= 0]  # the reference terminates each table with -1
            out.append(f"static const short JAAD_{jname}[{len(vals)}] = {{" + ", ".join(map(str, vals)) + "};")
        for cnt in (f"SWB_{tag}_WINDOW_COUNT",):
            vals = [int(t) for t in parse_rows(find_array(src, cnt))]
            out.append(f"static const unsigned char JAAD_{cnt}[{len(vals)}] = {{" + ", ".join(map(str, vals)) + "};")
        names = [t.strip() for t in parse_rows(find_array(src, f"SWB_OFFSET_{tag}_WINDOW"))]
        out.append(f"static const short* const JAAD_SWB_OFFSET_{tag}_WINDOW[{len(names)}] = {{"
                   + ", ".join("JAAD_" + n for n in names) + "};")
        out.append("")
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text("\n".join(out) + "\n")
    print("wrote", OUT, sum(1 for _ in out), "lines")
    emit(SBR_TABLES, SBR_OUT)
    emit(PS_TABLES, PS_OUT)
    emit(HUFF_TABLES, HUFF_OUT)
    emit_dct32()
    return 0


def _method_body(src: str, name: str) -> str:
    m = re.search(r"\b" + name + r"\s*\(\s*float\[\]\s*y\s*,\s*float\[\]\s*x\s*\)\s*\{", src)
    if not m:
        raise KeyError(name)
    depth, i = 0, m.end() - 1
    for j in range(i, len(src)):
        depth += src[j] == "{"
        depth -= src[j] == "}"
        if depth == 0:
            return src[i + 1:j]
    raise ValueError("unterminated " + name)


def dct32_program(body: str):
    """(ops, constants) of one straight-line transform: statements `dst = a-b | a+b | (c*a)`."""
    def slot(tok: str) -> int:
        tok = tok.strip()
        m = re.fullmatch(r"([xy])\[(\d+)\]", tok)
        if m:
            return int(m.group(2))
        m = re.fullmatch(r"f(\d+)", tok)
        if m:
            return 32 + int(m.group(1))
        raise ValueError(tok)

    ops, ks = [], []
    for stmt in body.split(";"):
        stmt = stmt.strip()
        if not stmt or stmt.startswith("float"):
            continue
        dst, expr = (t.strip() for t in stmt.split("=", 1))
        m = re.fullmatch(r"\(\s*(-?[0-9.]+f?)\s*\*\s*(\w+(?:\[\d+\])?)\s*\)", expr)
        if m:
            ops.append((2, slot(dst), slot(m.group(2)), 0))
            ks.append(f32_from_decimal(m.group(1)))
            continue
        m = re.fullmatch(r"(\w+(?:\[\d+\])?)\s*([-+])\s*(\w+(?:\[\d+\])?)", expr)
        if not m:
            raise ValueError(stmt)
        ops.append((0 if m.group(2) == "-" else 1, slot(dst), slot(m.group(1)), slot(m.group(3))))
        ks.append(np.float32(0.0))
    return ops, ks


def emit_dct32() -> None:
    src = strip_comments((REF / "sbr/SynthesisFilterbank32.java").read_text())
    out = ["/* GENERATED by tools/extract_tables.py -- the downsampled SBR synthesis's 32-point",
           " * DCT-IV / DST-IV (A/sbr/SynthesisFilterbank32.java DCT4_32, DST4_32) as op lists:",
           " * {kind, dst, a, b} over registers 0..31 (in/out array) and 32+k (temporary f<k>);",
           " * kind 0: r[a] - r[b], 1: r[a] + r[b], 2: K[i] * r[a].  Do not edit.",
           " * A C++ includer may define JAAD_DCT32_TABLE as `static constexpr` (compile-time use). */",
           "#pragma once", "#ifndef JAAD_DCT32_TABLE", "#define JAAD_DCT32_TABLE static const", "#endif", ""]
    for jname, cname in DCT32_PROGS:
        ops, ks = dct32_program(_method_body(src, jname))
        nreg = 1 + max(max(o[1], o[2], o[3]) for o in ops)
        out.append(f"#define {cname}_NOPS {len(ops)}")
        out.append(f"#define {cname}_NREG {nreg}")
        out.append(f"JAAD_DCT32_TABLE unsigned short {cname}_OPS[{len(ops)}][4] = {{")
        for i in range(0, len(ops), 6):
            out.append("  " + ", ".join("{%d, %d, %d, %d}" % o for o in ops[i:i + 6]) + ",")
        out.append("};")
        out.append(f"JAAD_DCT32_TABLE float {cname}_K[{len(ops)}] = {{")
        for i in range(0, len(ks), 6):
            out.append("  " + ", ".join(hexf(v) for v in ks[i:i + 6]) + ",")
        out.append("};")
        out.append(f"/* from sbr/SynthesisFilterbank32.java:{jname} */")
        out.append("")
    DCT32_OUT.write_text("\n".join(out) + "\n")
    print("wrote", DCT32_OUT, len(out), "lines")


def emit(tables, path: Path) -> None:
    out = ["/* GENERATED by tools/extract_tables.py -- binary32/int constant tables of the",
           " * reference decoder, carried as data (SURVEY.md s0 item 10). Do not edit. */",
           "#pragma once", ""]
    for fname, jname, cname, kind in tables:
        src = strip_comments((REF / fname).read_text())
        rows = parse_rows(find_array(src, jname))
        if kind == "f32":
            vals = [f32_from_decimal(t) for t in rows]
            out.append(f"static const float {cname}[{len(vals)}] = {{")
            for i in range(0, len(vals), 6):
                out.append("  " + ", ".join(hexf(v) for v in vals[i:i + 6]) + ",")
        elif kind == "f32_flat":
            body = find_array(src, jname)
            toks = [t for t in re.split(r"[{},\s]+", body) if t]
            vals = [f32_from_decimal(t) for t in toks]
            out.append(f"static const float {cname}[{len(vals)}] = {{")
            for i in range(0, len(vals), 6):
                out.append("  " + ", ".join(hexf(v) for v in vals[i:i + 6]) + ",")
        elif kind == "i32":
            vals = [int(t) for t in rows]
            out.append(f"static const int {cname}[{len(vals)}] = {{" + ", ".join(map(str, vals)) + ",")
        elif kind == "i32_2d":
            ncol = len(rows[0])
            assert all(len(r) == ncol for r in rows), cname
            out.append(f"static const int {cname}[{len(rows)}][{ncol}] = {{")
            for r in rows:
                out.append("  {" + ", ".join(str(int(t)) for t in r) + "},")
        else:
            ncol = len(rows[0]) if kind == "f32_2d" else int(kind[-1])
            vals = [[f32_from_decimal(t) for t in r[:ncol]] for r in rows]
            assert all(len(r) == ncol for r in vals), cname
            out.append(f"static const float {cname}[{len(vals)}][{ncol}] = {{")
            for r in vals:
                out.append("  {" + ", ".join(hexf(v) for v in r) + "},")
        out.append("};")
        out.append(f"/* from {fname}:{jname} */")
        out.append("")
    path.write_text("\n".join(out) + "\n")
    print("wrote", path, len(out), "lines")


if __name__ == "__main__":
    sys.exit(main())
