"""How the C2 batch time evolves with back-to-back launches and after idle gaps (GPU clock ramp vs
one-time warming): blocks of 10 launches, printed per block.

    python scripts/warm_probe.py [CONFIG]
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

cfgid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
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


def block(n=10):
    ev[0].record(s)
    for _ in range(n):
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
    ev[1].record(s)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / n


ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
torch.cuda.synchronize()
for phase, (gap, nb) in enumerate([(0.0, 40), (1.0, 6), (0.05, 6), (2.0, 3), (0.0, 20)]):
    time.sleep(gap)
    ms = [block() for _ in range(nb)]
    print(f"phase {phase} (idle {gap:.2f} s before): " + " ".join(f"{x:.4f}" for x in ms), flush=True)
single = []
for _ in range(20):
    single.append(block(1))
print("single launches: " + " ".join(f"{x:.4f}" for x in single))
