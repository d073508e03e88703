"""Host parser robustness: a sanitizer (ASan + UBSan) build of the bitstream front end
(jaadec_amd/csrc/jaad_parse*.cpp, tools/fuzz_parse.cpp) parses bit-flipped and truncated
versions of valid LC / HE-AAC v1 / v2 frames.  Any status is a valid outcome (the reference
throws or drops such frames); out-of-bounds access or undefined behaviour is not."""
import shutil
import struct
import subprocess
import sys
from pathlib import Path

import pytest

from jaadec_amd import native as N
from oracle import oracle as O

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(Path(__file__).resolve().parent))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_parser_survives_mutated_frames_under_sanitizers(tmp_path):
    from test_parse_sbr import _stream
    seeds = tmp_path / "seeds.bin"
    with open(seeds, "wb") as out:
        for cfgid, opts in ((4, dict(grids=True)), (5, dict(ps_modes=True, grids=True))):
            p, b = _stream(cfgid, 24, 5, **opts)
            cfg = N.cfg_for(p)
            for f in O.write_frames(b, p.sf_index, sbr_writer=O.SbrWriter(cfg.ext_sf_index, 5)):
                out.write(struct.pack("<BI", cfgid, len(f)) + f)
        p = N.synth_params(3, n_streams=1, frames_per_stream=24, pns_percent=8, is_percent=10)
        b = N.synth_batch(p)
        for f in O.write_frames(b, p.sf_index, extras=3):
            out.write(struct.pack("<BI", 3, len(f)) + f)
    exe = tmp_path / "fuzz_parse"
    csrc = ROOT / "jaadec_amd" / "csrc"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{ROOT / 'include'}", f"-I{csrc}",
                    str(ROOT / "tools" / "fuzz_parse.cpp"), str(csrc / "jaad_parse.cpp"), str(csrc / "jaad_parse_sbr.cpp"),
                    str(csrc / "jaad_sbr_host.cpp"), str(csrc / "jaad_mp4.cpp"), "-o", str(exe)], check=True, timeout=300)
    r = subprocess.run([str(exe), str(seeds), "30000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "status 0:" in r.stdout  # some mutants still parse: the fuzz reaches the deep syntax
    # the MP4 feeder (jaad_mp4.cpp) on mutated file images
    from oracle import mp4_writer as W
    p = N.synth_params(3, n_streams=1, frames_per_stream=12)
    b = N.synth_batch(p)
    mp4 = tmp_path / "a.mp4"
    mp4.write_bytes(W.write_mp4(O.write_frames(b, p.sf_index), bytes([0x11, 0x90]), 48000, 2, video_track=True,
                                long_desc=True, chunk_sizes=(2, 3)))
    r = subprocess.run([str(exe), "mp4", str(mp4), "20000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
