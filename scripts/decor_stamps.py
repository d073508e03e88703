"""Per-role busy share of the pipelined decorrelator (JAAD_DECOR_STAMPS build, JAAD_LIB=...): C5 at
the per-GPU size, s_memtime ticks of each wave's step bodies vs its whole step loop."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

p = N.synth_params(5, n_streams=256)
b = N.synth_batch(p)
cfg = N.cfg_for(p)
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
d = {"q": t(b.q), "sf": t(b.sf), "cb": t(b.cb), "ics": t(b.ics)}
ptr = {k: v.data_ptr() for k, v in d.items()}
ptr["ms_used"] = None
ptr["tns"] = None
pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, True), dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, int(b.stream_slot.max()) + 1)
W = 8  # waves per run (kDecorWaves; 12 in the mixing-role experiments)
dbg = torch.zeros(4096 + 256 * W * 4 + 64, dtype=torch.int32, device=dev)
N.lib().jaad__sbr_debug_attach.argtypes = [C.c_void_p, C.c_void_p]
N.lib().jaad__sbr_debug_attach(ctx.h, dbg.data_ptr())
for _ in range(5):
    ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, None)
torch.cuda.synchronize()
D = dbg.cpu().numpy().view(np.uint32)[4096:4096 + 256 * W * 4].reshape(256, W, 4).astype(np.int64)
names = {0: "Q0 QMF delay+link0", 1: "Q1 QMF link1", 2: "Q2 QMF link2", 3: "H0 hyb delay+link0",
         4: "H1 hyb link1 + ratio", 5: "H2 hyb link2", 6: "T transient", 7: "P param scan",
         8: "M0 mix QMF slots 0-10", 9: "M1 mix QMF 11-21", 10: "M2 mix QMF 22-31", 11: "MH mix hybrid"}
for w in range(W):
    role = int(D[0, w, 2])
    busy, tot = np.median(D[:, w, 0]), np.median(D[:, w, 1])
    print(f"wave {w} role {role} {names[role]:22s} busy {busy:9.0f} total {tot:9.0f} ticks ({100 * busy / tot:5.1f} %)")
print("frames per run", int(D[0, 0, 3]))
ctx.close()
