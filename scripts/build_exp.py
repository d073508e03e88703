"""Build experimental variants of libjaadgpu.so into exp/ (git-ignored; unlike .tmp/ it travels to
the GPU box with gpurun).  Round 6.  Only the given kernel sources are recompiled with the macros;
the other objects are the product build's (build/obj/libjaadgpu, from build_gpu()).

    python scripts/build_exp.py NAME [-DMACRO[=V] ...] [--src=jaad_lc.hip,...] [--alt=jaad_sbr.hip:PATH]
                                [-- extra hipcc flags]

--alt compiles PATH in place of that source (e.g. a `git show HEAD:...` copy: an A/B against the
committed kernel).
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import build as B  # noqa: E402

if __name__ == "__main__":
    name, rest = sys.argv[1], sys.argv[2:]
    extra = rest[rest.index("--") + 1:] if "--" in rest else []
    opts = rest[:rest.index("--")] if "--" in rest else rest
    defs = [a[2:] for a in opts if a.startswith("-D")]
    srcs = ["jaad_lc.hip"]
    alt = {}
    for a in opts:
        if a.startswith("--src="):
            srcs = a[6:].split(",")
        if a.startswith("--alt="):
            name_, path_ = a[6:].split(":", 1)
            alt[name_] = Path(path_).resolve()
    srcs += [a for a in alt if a not in srcs]
    B.build_gpu()  # the product objects are current
    prod = ROOT / "build" / "obj" / "libjaadgpu"
    objdir = ROOT / "build" / "obj" / f"exp_{name}"
    objdir.mkdir(parents=True, exist_ok=True)
    common = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
              "-fno-slp-vectorize", "-fno-gpu-rdc", "-Wall", "-Wno-unused-function", "-I", str(ROOT / "include"), "-I", str(B.CSRC)]
    common += [f"-D{d}" for d in defs] + extra
    objs = []
    for o in sorted(prod.glob("*.o")):
        src = o.name[:-2]
        if src in srcs:
            new = objdir / o.name
            subprocess.run(common + ["-c", "-o", str(new), str(alt.get(src, B.CSRC / src))], check=True)
            objs.append(new)
        else:
            objs.append(o)
    out = ROOT / "exp" / f"lib_{name}.so"
    out.parent.mkdir(exist_ok=True)
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fno-gpu-rdc", "-o", str(out)] + [str(o) for o in objs],
                   check=True)
    print(out)
