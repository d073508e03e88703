"""Build the native pieces in-tree.

* ``jaadec_amd/libjaadgpu.so`` -- the product: C-ABI (include/jaad_gpu.h) + gfx950 HIP kernels.
* ``jaadec_amd/libjaadsynth.so`` -- host-side synthetic batch generator (bench/test inputs).
* ``oracle/liboracle.so`` -- TEST INFRASTRUCTURE: the C restatement of the reference DSP.

Everything is compiled with ``-ffp-contract=off``: the reference (Java >= 17) evaluates binary32
arithmetic strictly, without fused multiply-add, and both the oracle and the HIP kernels follow
its evaluation order so their results are bit-identical.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "jaadec_amd"
CSRC = PKG / "csrc"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

LIB = PKG / "libjaadgpu.so"
SYNTH_LIB = PKG / "libjaadsynth.so"
ORACLE_LIB = ROOT / "oracle" / "liboracle.so"


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _deps(*globs: str) -> list[Path]:
    out: list[Path] = []
    for g in globs:
        out += sorted(ROOT.glob(g))
    return out


# per-source extra flags (the LC kernel: see DESIGN.md §4a, scheduler strategy)
GPU_FILE_FLAGS: dict[str, list[str]] = {
    # the +-1 LSB LC kernels (modes 4, 6): LLVM's iterative-ILP machine scheduler (-2.2 % on C2, round 6)
    "jaad_lc_fast.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
}
# kernel sources whose device assembly goes through tools/vop3_rewrite.py (VCC-implicit VOP2 /
# VOPC forms re-encoded as VOP3: DESIGN.md §4a, round 4) before it is assembled
VOP3_REWRITE: dict[str, tuple[str, ...]] = {}
LLVM = Path(os.environ.get("ROCM_LLVM", "/opt/rocm/lib/llvm/bin"))


def _hip_obj_rewritten(cmd_common: list[str], src: Path, obj: Path, forms: tuple[str, ...]) -> None:
    """hipcc -c of `src` with its device code taken through vop3_rewrite: device assembly
    (branches kept within 2^14 words so the longer encodings still reach), rewrite, assemble,
    link the code object, bundle it, then the host compile embeds the bundle."""
    base = obj.with_suffix("")
    s, s2, do, co, fb = (base.with_suffix(x) for x in (".dev.s", ".dev3.s", ".dev.o", ".dev.co", ".hipfb"))
    _run(cmd_common + ["--cuda-device-only", "-S", "-mllvm", "-amdgpu-s-branch-bits=14", "-o", str(s), str(src)])
    _run([sys.executable, str(ROOT / "tools" / "vop3_rewrite.py"), str(s), str(s2)] + list(forms))
    _run([str(LLVM / "clang"), "-cc1as", "-triple", "amdgcn-amd-amdhsa", "-target-cpu", ARCH, "-filetype", "obj",
          "-o", str(do), str(s2)])
    _run([str(LLVM / "lld"), "-flavor", "gnu", "-m", "elf64_amdgpu", "--no-undefined", "-shared", "-o", str(co), str(do)])
    _run([str(LLVM / "clang-offload-bundler"), "-type=o", "-bundle-align=4096",
          f"-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--{ARCH}", "-input=/dev/null",
          f"-input={co}", f"-output={fb}"])
    _run(cmd_common + ["--cuda-host-only", "-Xclang", "-fcuda-include-gpubinary", "-Xclang", str(fb), "-c", "-o", str(obj),
                       str(src)])


def build_gpu(force: bool = False, out: Path | None = None, defines: list[str] | None = None,
              extra: list[str] | None = None, vop3: dict[str, tuple[str, ...]] | None = None) -> Path:
    """Build the product library (or, with `defines`/`vop3`, an experimental variant at `out`): every
    source compiled on its own (in parallel, with its GPU_FILE_FLAGS; VOP3_REWRITE sources through
    the re-encoding pipeline), then linked."""
    out = out or LIB
    rewrite = VOP3_REWRITE if vop3 is None else vop3
    srcs = [CSRC / "jaad_lc.hip", CSRC / "jaad_lc_fast.hip", CSRC / "jaad_sbr.hip", CSRC / "jaad_ps.hip", CSRC / "jaad_capi.cpp", CSRC / "jaad_sbr_host.cpp",
            CSRC / "jaad_parse.cpp", CSRC / "jaad_parse_sbr.cpp", CSRC / "jaad_mp4.cpp"]
    deps = srcs + _deps("jaadec_amd/csrc/*.h", "jaadec_amd/csrc/tables/*.inc", "include/*.h") + [ROOT / "tools" / "vop3_rewrite.py"]
    if force or defines or extra or vop3 is not None or _stale(out, deps):
        objdir = ROOT / "build" / "obj" / out.stem
        objdir.mkdir(parents=True, exist_ok=True)
        common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                  "-fno-slp-vectorize", "-fno-gpu-rdc", "-Wall", "-Wno-unused-function", "-I", str(ROOT / "include")]
        common += [f"-D{d}" for d in (defines or [])] + (extra or [])
        objs = [objdir / (s.name + ".o") for s in srcs]
        from concurrent.futures import ThreadPoolExecutor
        def one(so):
            src, obj = so
            cmd = common + GPU_FILE_FLAGS.get(src.name, [])
            if src.name in rewrite:
                _hip_obj_rewritten(cmd, src, obj, rewrite[src.name])
            else:
                _run(cmd + ["-c", "-o", str(obj), str(src)])

        with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
            list(ex.map(one, zip(srcs, objs)))
        tmp = out.with_suffix(".so.tmp")
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fno-gpu-rdc", "-o", str(tmp)] + [str(o) for o in objs])
        tmp.replace(out)
    return out


def build_synth(force: bool = False) -> Path:
    srcs = [CSRC / "jaad_synth.cpp"]
    deps = srcs + _deps("include/*.h", "jaadec_amd/csrc/tables/*.inc")
    if force or _stale(SYNTH_LIB, deps):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
              "-I", str(ROOT / "include"), "-o", str(SYNTH_LIB)] + [str(s) for s in srcs])
    return SYNTH_LIB


def build_oracle(force: bool = False) -> Path:
    srcs = [ROOT / "oracle" / "jaad_oracle.c", ROOT / "oracle" / "jaad_oracle_sbr.c", ROOT / "oracle" / "jaad_oracle_ps.c",
            ROOT / "oracle" / "jaad_writer.c",
            ROOT / "oracle" / "jaad_writer_sbr.c"]
    deps = srcs + _deps("oracle/*.h", "include/*.h", "jaadec_amd/csrc/tables/*.inc")
    if force or _stale(ORACLE_LIB, deps):
        _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
              "-Wall", "-o", str(ORACLE_LIB)] + [str(s) for s in srcs] + ["-lm", "-lpthread"])
    return ORACLE_LIB


def jni_include() -> Path | None:
    """$JAVA_HOME/include when a JDK is installed (none in this image)."""
    home = os.environ.get("JAVA_HOME")
    if home and (Path(home) / "include" / "jni.h").exists():
        return Path(home) / "include"
    return None


def build_jni(force: bool = False) -> Path | None:
    """libjaadjni.so: the JNI glue over libjaadgpu.so. Skipped without a JDK."""
    inc = jni_include()
    if inc is None:
        print("JNI glue skipped: no $JAVA_HOME/include/jni.h", flush=True)
        return None
    out = PKG / "libjaadjni.so"
    srcs = [CSRC / "jaad_jni.c"]
    if force or _stale(out, srcs + [LIB]):
        _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-Wall", "-I", str(ROOT / "include"), "-I", str(inc),
              "-I", str(inc / "linux"), "-o", str(out), str(srcs[0]), "-L", str(PKG), "-ljaadgpu",
              "-Wl,-rpath,$ORIGIN"])
    return out


def build_jni_mock(force: bool = False) -> Path:
    """TEST INFRASTRUCTURE: the JNI glue (jaad_jni.c) compiled against tests/jni_mock/jni.h and a
    mock JNIEnv, so tests/test_jni_glue.py runs its argument checks without a JDK."""
    mock = ROOT / "tests" / "jni_mock"
    out = mock / "libjaadjni_mock.so"
    srcs = [CSRC / "jaad_jni.c", mock / "jni_mock.c"]
    if force or _stale(out, srcs + [mock / "jni.h", LIB]):
        _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-Wall", "-I", str(mock), "-I", str(ROOT / "include"),
              "-o", str(out)] + [str(x) for x in srcs] + ["-L", str(PKG), "-ljaadgpu", f"-Wl,-rpath,{PKG}",
                                                          "-Wl,-rpath,$ORIGIN/../../jaadec_amd"])
    return out


def build_tools(force: bool = False) -> Path:
    """tools/bench_parse: the host front end's frames/s over a bitstream corpus (bench.py host_parse)."""
    out = ROOT / "tools" / "bench_parse"
    src = ROOT / "tools" / "bench_parse.cpp"
    if force or _stale(out, [src, ROOT / "include" / "jaad_parse.h", LIB]):
        _run(["g++", "-O2", "-std=c++17", "-pthread", "-Wall", "-I", str(ROOT / "include"), "-o", str(out), str(src),
              "-L", str(PKG), "-ljaadgpu", f"-Wl,-rpath,{PKG}", "-Wl,-rpath,$ORIGIN/../jaadec_amd"])
    return out


def build_all(force: bool = False) -> None:
    build_oracle(force)
    build_synth(force)
    build_gpu(force)
    build_jni(force)
    build_jni_mock(force)
    build_tools(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
