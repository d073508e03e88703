"""Build experimental variants of libjaadgpu.so into exp/ (git-ignored; unlike .tmp/ it travels to
the GPU box with gpurun).  Round 6.

    python scripts/build_exp.py NAME [-DMACRO[=V] ...] [-- extra hipcc flags]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import build as B  # noqa: E402

if __name__ == "__main__":
    name, rest = sys.argv[1], sys.argv[2:]
    extra = rest[rest.index("--") + 1:] if "--" in rest else []
    defs = [a[2:] for a in (rest[:rest.index("--")] if "--" in rest else rest) if a.startswith("-D")]
    out = ROOT / "exp" / f"lib_{name}.so"
    out.parent.mkdir(exist_ok=True)
    B.build_gpu(out=out, defines=defs, extra=extra, force=True)
    print(out)
