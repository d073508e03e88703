"""Decode one config's batch N times on the device (inputs resident) after a settle: a short
program for rocprofv3 kernel traces of a library variant (JAAD_LIB=...).
    python scripts/decode_loop.py CONFIG N [STREAMS]"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

cfgid, n = int(sys.argv[1]), int(sys.argv[2])
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # streams (0: the config's default job)
p = N.synth_params(cfgid, n_streams=ns) if ns else N.synth_params(cfgid)
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
pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, bool(p.sbr), N.sbr_downsampled(cfg)), dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, int(b.stream_slot.max()) + 1)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
    torch.cuda.synchronize()
for _ in range(n):
    ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
torch.cuda.synchronize()
ctx.close()
