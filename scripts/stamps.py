"""Run a JAAD_STAMPS build on C2 and summarize per-wave phase timings (s_memtime ticks)."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

p = N.synth_params(2); b = N.synth_batch(p); cfg = N.make_cfg()
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
d = {"q": t(b.q), "sf": t(b.sf), "cb": t(b.cb), "ics": t(b.ics), "ms_used": t(b.ms_used)}
ptr = {k: v.data_ptr() for k, v in d.items()}
pcm = torch.empty(b.n_frames * 4096, dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, 256)
nw = 4096 * 4
dbg = torch.zeros(nw * 32, dtype=torch.int32, device=dev)
N.lib().jaad__debug_attach.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
N.lib().jaad__debug_attach(ctx.h, dbg.data_ptr(), -1)
for _ in range(3):
    ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, None)
torch.cuda.synchronize()
S = dbg.cpu().numpy().view(np.uint32).reshape(nw, 32).astype(np.int64)
names = ["iter start", "side->LDS raw", "gain table", "IQ", "store_spec(+PNS) + B1 wait", "phase C", "B2 wait", "D: IMDCT+OLA+PCM->LDS", ]
for it in range(3):
    b0 = 2 + 9 * it
    row = []
    for k in range(7):
        d = (S[:, b0 + k + 1] - S[:, b0 + k]) & 0xffffffff
        row.append(np.median(d))
    nxt = (S[:, b0 + 9] if it < 2 else S[:, 31])
    print("it", 4 + it, " ".join(f"{names[k+1]}={row[k]:.0f}" for k in range(7)))
