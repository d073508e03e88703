"""C2 batch time over several seconds of back-to-back launches (blocks of 50), to see where the
clock settles under sustained load.   python scripts/warm_long.py [CONFIG] [SECONDS]"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

cfgid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
p = N.synth_params(cfgid)
b = N.synth_batch(p)
cfg = N.cfg_for(p)
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
d = {"q": t(b.q), "sf": t(b.sf), "cb": t(b.cb), "ics": t(b.ics)}
if b.ms_used is not None:
    d["ms_used"] = t(b.ms_used)
ptr = {k: v.data_ptr() for k, v in d.items()}
ptr.setdefault("ms_used", None)
ptr["tns"] = None
pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, bool(p.sbr)), dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, int(b.stream_slot.max()) + 1)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
t0 = time.perf_counter()
out = []
while time.perf_counter() - t0 < secs:
    ev[0].record(s)
    for _ in range(50):
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
    ev[1].record(s)
    torch.cuda.synchronize()
    out.append(ev[0].elapsed_time(ev[1]) / 50)
    if len(out) % 10 == 0:
        print(f"{time.perf_counter() - t0:6.2f} s: " + " ".join(f"{x:.4f}" for x in out[-10:]), flush=True)
print("overall median %.4f ms, last-half median %.4f ms" % (np.median(out), np.median(out[len(out) // 2:])))
