"""Build experimental variants of libjaadgpu.so into .tmp/exp/ (ablation macros of jaad_lc.hip)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import build as B  # noqa: E402

VARIANTS = {
    "a_base": [],
    "b_no_iq": ["JAAD_ABL_NO_IQ"],
    "c_no_ms": ["JAAD_ABL_NO_MS"],
    "d_no_imdct": ["JAAD_ABL_NO_IMDCT"],
    "e_no_pcmlds": ["JAAD_ABL_NO_PCMLDS"],
    "f_no_store": ["JAAD_ABL_NO_STORE"],
    "g_no_barrier": ["JAAD_ABL_NO_BARRIER"],
    "h_w2": ["JAAD_WAVES_PER_EU=2"],
}

if __name__ == "__main__":
    out = ROOT / ".tmp" / "exp"
    out.mkdir(parents=True, exist_ok=True)
    for f in out.glob("lib_*.so"):
        f.unlink()
    only = set(sys.argv[1:])
    for name, defs in VARIANTS.items():
        if only and name not in only:
            continue
        B.build_gpu(out=out / f"lib_{name}.so", defines=defs)
