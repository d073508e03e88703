"""One timing child of scripts/time_variants.py (JAAD_LIB selects the library)."""

import sys, time, numpy as np, torch
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jaadec_amd import native as N
cfgid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
p = N.synth_params(cfgid); b = N.synth_batch(p); cfg = N.cfg_for(p)
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
d = {"q": t(b.q), "sf": t(b.sf), "cb": t(b.cb), "ics": t(b.ics)}
if b.ms_used is not None: d["ms_used"] = t(b.ms_used)
ptr = {k: v.data_ptr() for k, v in d.items()}
ptr.setdefault("ms_used", None); ptr["tns"] = None
pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, bool(p.sbr)), dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, int(b.stream_slot.max()) + 1)
s = torch.cuda.Stream(dev); torch.cuda.set_stream(s)
for _ in range(3): ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(s)
for _ in range(20): ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
ev[1].record(s); torch.cuda.synchronize()
print("%.4f" % (ev[0].elapsed_time(ev[1]) / 20))
