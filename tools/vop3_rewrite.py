#!/usr/bin/env python3
"""Re-encode VCC-implicit VOP2/VOPC instructions of a gfx950 device assembly listing as VOP3.

gfx950 issues a VOP2 v_cndmask_b32 (whose lane mask is the implicit VCC operand) at ~13.9 SIMD
cycles per wave-instruction at 3 waves/SIMD, against ~3.6 for the VOP3 v_cndmask_b32_e64
(tools/valu_rate.hip, profiles/round4_valu_rate.txt).  The compiler's instruction shrinking picks
the short VOP2 form whenever the mask lives in VCC; this pass, run between `hipcc -S` and the
assembler (jaadec_amd/build.py), rewrites the forms listed in FORMS to their _e64 encoding with the
same operands -- the same operation on the same registers, so results are bit-identical.  A form
whose src0 is a 32-bit literal has no VOP3 encoding on gfx9 and is left as it is.

    python3 tools/vop3_rewrite.py in.s out.s [form ...]
"""
import re
import sys

# gfx9 inline constants (VOP3 takes these, not 32-bit literals)
_INLINE_F = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0", "0.15915494"}


def _inline(op: str) -> bool:
    op = op.strip()
    if re.fullmatch(r"-?\d+", op):
        return -16 <= int(op) <= 64
    if op.startswith(("0x", "-0x")):
        v = int(op, 16)
        return -16 <= v <= 64
    if re.fullmatch(r"-?\d+\.\d*(e-?\d+)?", op):
        return op in _INLINE_F
    return True  # a register (v*, s*, vcc, exec, ...) or a symbolic operand


CNDMASK = re.compile(r"^(\s*)v_cndmask_b32_e32(\s+)(\S+),\s*(\S+),\s*(\S+),\s*vcc\s*$")
VOPC = re.compile(r"^(\s*)(v_cmp\w*|v_cmpx\w*)_e32(\s+)vcc,\s*(\S+),\s*(\S+)\s*$")


def rewrite(lines, forms=("cndmask",)):
    n = {"cndmask": 0, "vopc": 0, "kept_literal": 0}
    out = []
    for line in lines:
        m = CNDMASK.match(line)
        if m and "cndmask" in forms:
            if _inline(m.group(4)):
                out.append(f"{m.group(1)}v_cndmask_b32_e64{m.group(2)}{m.group(3)}, {m.group(4)}, {m.group(5)}, vcc\n")
                n["cndmask"] += 1
                continue
            n["kept_literal"] += 1
        m = VOPC.match(line)
        if m and "vopc" in forms and not m.group(2).startswith("v_cmpx"):
            if _inline(m.group(4)):
                out.append(f"{m.group(1)}{m.group(2)}_e64{m.group(3)}vcc, {m.group(4)}, {m.group(5)}\n")
                n["vopc"] += 1
                continue
            n["kept_literal"] += 1
        out.append(line)
    return out, n


def main():
    src, dst = sys.argv[1], sys.argv[2]
    forms = tuple(sys.argv[3:]) or ("cndmask",)
    with open(src) as f:
        lines = f.readlines()
    out, n = rewrite(lines, forms)
    with open(dst, "w") as f:
        f.writelines(out)
    print(f"vop3_rewrite {src}: {n}", file=sys.stderr)


if __name__ == "__main__":
    main()
