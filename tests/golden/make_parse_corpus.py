"""Bitstream corpora for the host front-end timing (tools/bench_parse.cpp, bench.py `host_parse`):
raw_data_blocks of the synthetic C2..C5 workloads, written by the TEST WRITER (oracle/jaad_writer*.c)
from the same synthetic records the GPU benchmarks decode.  Test infrastructure: run here, the .bin
files are committed data.

    python tests/golden/make_parse_corpus.py

Format (little endian): b"JPC1", u32 sizeof(jaad_stream_cfg), the cfg bytes, u32 streams,
u32 frames per stream, then per stream u32 initial PNS LCG state and per frame u32 length + bytes.
"""
import struct
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402
from oracle import oracle as O  # noqa: E402

STREAMS, FRAMES = 4, 64


def corpus(cfgid: int) -> bytes:
    p = N.synth_params(cfgid, n_streams=STREAMS, frames_per_stream=FRAMES)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    raw = bytes(cfg)
    out = [b"JPC1", struct.pack("<I", len(raw)), raw, struct.pack("<II", STREAMS, FRAMES)]
    for s in range(STREAMS):
        f0, f1 = int(b.frame_begin[s]), int(b.frame_begin[s + 1])
        # each stream from a fresh SBR/PS writer: its first frame codes no deltas against another
        kw = {"sbr_writer": O.SbrWriter(cfg.ext_sf_index, 5)} if p.sbr else {}
        frames = O.write_frames(b, p.sf_index, frames=range(f0, f1), **kw)
        out.append(struct.pack("<I", int(b.ics["pns_state"][f0 * b.nch])))
        for fr in frames:
            out.append(struct.pack("<I", len(fr)))
            out.append(fr)
    return b"".join(out)


if __name__ == "__main__":
    for cid in (2, 3, 4, 5):
        out = Path(__file__).with_name(f"parse_c{cid}.bin")
        out.write_bytes(corpus(cid))
        print(out.name, out.stat().st_size, "bytes")
