"""Run a JAAD_STAMPS build (JAAD_LIB=...) on C2 and print the per-phase share of wave time
(s_memtime ticks summed over each wave's frames; median over waves)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

cfgid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
prec = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # jaad_stream_cfg.precision (round 6: 1 = the +-1 LSB kernel)
p = N.synth_params(cfgid); b = N.synth_batch(p); cfg = N.cfg_for(p, precision=prec)
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
d = {"q": t(b.q), "sf": t(b.sf), "cb": t(b.cb), "ics": t(b.ics)}
if b.ms_used is not None: d["ms_used"] = t(b.ms_used)
ptr = {k: v.data_ptr() for k, v in d.items()}
ptr.setdefault("ms_used", None); ptr["tns"] = None
pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, bool(p.sbr)), dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, int(b.stream_slot.max()) + 1)
nw = 8192
dbg = torch.zeros(nw * 16, dtype=torch.int32, device=dev)
N.lib().jaad__debug_attach.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
N.lib().jaad__debug_attach(ctx.h, dbg.data_ptr(), -1)
import time
t_end = time.perf_counter() + 0.4  # past the clock's load-onset transient, then the measured call
while time.perf_counter() < t_end:
    for _ in range(10):
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, None)
    torch.cuda.synchronize()
dbg.zero_()
ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, None)
torch.cuda.synchronize()
S = dbg.cpu().numpy().view(np.uint32).reshape(nw, 16).astype(np.int64)
S = S[S.sum(1) > 0]
names = ["top: rest of side info (+ early IQ issue)", "band records", "prefetch issue (+PNS)", "M/S, I/S", "spectra to LDS",
         "loop back + wave priority", "prefetched side info in (vmcnt)", "-", "IMDCT + OLA (both channels)", "drain next frame's loads",
         "PCM stage + stores", "chunk tail", "IQ R", "IQ L", "band record reads"]
med = np.median(S, axis=0)
tot = med[:15].sum()
for k in range(15):
    print(f"{k:2d} {names[k]:32.32s} {med[k]:12.0f} ticks {100 * med[k] / tot:5.1f} %")
print("waves", S.shape[0], "total median ticks", tot)
