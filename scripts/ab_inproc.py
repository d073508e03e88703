"""Same-process A/B of libjaadgpu.so builds: every lib gets its own context on the same device
inputs, and blocks of launches alternate between the libs (A B C A B C ...), so clock drift and
box state hit all alike.  Prints per lib: median / min ms per batch over the blocks, PCM hash.

    python scripts/ab_inproc.py CONFIG BLOCKS LAUNCHES_PER_BLOCK lib1.so lib2.so ...

A lib argument may carry environment settings applied before its context is created, e.g.
``lib_b.so@JAAD_LC_PAIR=0`` (copies of one build then differ only in those settings), or
``lib.so@precision=1`` (the context's jaad_stream_cfg.precision), ``lib.so@hint=1`` (its calls pass
JAAD_HINT_SHORT_WINDOWS).
"""
import os
import hashlib
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402


def main():
    cfgid, blocks, per = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    paths = sys.argv[4:]
    p = N.synth_params(cfgid)
    b = N.synth_batch(p)
    cfg = N.cfg_for(p)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
    d = {"q": t(b.q), "sf": t(b.sf), "cb": t(b.cb), "ics": t(b.ics)}
    if b.ms_used is not None:
        d["ms_used"] = t(b.ms_used)
    if b.tns is not None:
        d["tns"] = t(b.tns)
    ptr = {k: v.data_ptr() for k, v in d.items()}
    ptr.setdefault("ms_used", None)
    ptr.setdefault("tns", None)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    runs = []
    for arg in paths:
        path, *envs = arg.split("@")
        ccfg = N.cfg_for(p)
        flags = 0
        for kv in envs:
            k, v = kv.split("=", 1)
            if k == "precision":  # a jaad_stream_cfg field, not an environment setting
                ccfg.precision = int(v)
            elif k == "hint":  # jaad_decode_batch_device flags: JAAD_HINT_SHORT_WINDOWS
                flags |= N.HINT_SHORT_WINDOWS if int(v) else 0
            else:
                os.environ[k] = v
        L = N.load_lib(path)
        N._lib = L
        ctx = N.Context(ccfg, int(b.stream_slot.max()) + 1)
        pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, bool(p.sbr)), dtype=torch.uint8, device=dev)
        runs.append((Path(path).stem + ("@" + "@".join(envs) if envs else ""), L, ctx, pcm, [], flags))
        for kv in envs:
            if not kv.startswith(("precision=", "hint=")):
                os.environ.pop(kv.split("=", 1)[0], None)
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.4:  # warm-up past the GPU clock's load-onset transient
        for name, L, ctx, pcm, _, fl in runs:
            N._lib = L
            for _ in range(5):
                ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), fl, s.cuda_stream)
        torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for blk in range(blocks):
        order = runs if blk % 2 == 0 else runs[::-1]
        for name, L, ctx, pcm, times, fl in order:
            N._lib = L
            ev[0].record(s)
            for _ in range(per):
                ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), fl, s.cuda_stream)
            ev[1].record(s)
            torch.cuda.synchronize()
            times.append(ev[0].elapsed_time(ev[1]) / per)
        print(f"block {blk}: " + "  ".join(f"{r[0]} {r[4][-1]:.4f}" for r in runs), flush=True)
    ref = runs[0][3].cpu().numpy().view(">i2").astype(np.int32)
    for name, L, ctx, pcm, times, _ in runs:
        h = hashlib.blake2b(pcm.cpu().numpy().tobytes(), digest_size=6).hexdigest()
        d = np.abs(pcm.cpu().numpy().view(">i2").astype(np.int32) - ref)
        print(f"{name:24s} median {np.median(times):.4f} min {np.min(times):.4f} ms  pcm {h}  "
              f"vs first: max |d| {d.max()} LSB, {int((d != 0).sum())} samples differ")
    for name, L, ctx, pcm, times, _ in runs:
        N._lib = L
        ctx.close()


if __name__ == "__main__":
    main()
