"""Build experimental variants of libjaadgpu.so into .tmp/exp/ (ablation macros of the kernels)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import build as B  # noqa: E402

KSRC = ("jaad_lc.hip", "jaad_sbr.hip", "jaad_ps.hip")
# name: (defines, extra flags, VOP3 rewrite forms per kernel source or None for the product's)
VARIANTS = {
    "b_head": ([], [], None),
    "c_vop3": ([], [], {k: ("cndmask", "vopc") for k in KSRC}),
    "d_vop3c": ([], [], {k: ("cndmask",) for k in KSRC}),
    "s_stamps": (["JAAD_STAMPS"], [], None),
    "g_w8": (["JAAD_LC_WAVES=8"], [], None),
    "d_plain": (["JAAD_DECOR_ROLES_PLAIN"], [], None),
    "d_stamps": (["JAAD_DECOR_STAMPS"], [], None),
    "h_w4": (["JAAD_LC_WAVES=4"], [], None),
}

if __name__ == "__main__":
    out = ROOT / ".tmp" / "exp"
    out.mkdir(parents=True, exist_ok=True)
    for f in out.glob("lib_*.so"):
        if f.stem[4:] in VARIANTS and (len(sys.argv) < 2 or f.stem[4:] in sys.argv[1:]): f.unlink()
    only = set(sys.argv[1:])
    from concurrent.futures import ThreadPoolExecutor
    todo = [(n, d) for n, d in VARIANTS.items() if not only or n in only]
    with ThreadPoolExecutor(6) as ex:
        list(ex.map(lambda nd: B.build_gpu(out=out / f"lib_{nd[0]}.so", defines=nd[1][0], extra=nd[1][1],
                                           vop3=nd[1][2], force=True), todo))
