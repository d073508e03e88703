"""Phase timeline of sbr_hf_kernel<0> (JAAD_HF_STAMPS build, JAAD_LIB=exp/lib_hfstamps.so): the C4
batch, s_memtime at each phase boundary of every channel-frame (jaad_sbr.hip HF_STAMP)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

cfgid = int(sys.argv[1]) if len(sys.argv) > 1 else 4
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
pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, True), dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, int(b.stream_slot.max()) + 1)
n_cf = b.n_frames * (2 if p.channel_config == 2 else 1)
dbg = torch.zeros(n_cf * 16, dtype=torch.int64, device=dev)
N.lib().jaad__sbr_debug_attach.argtypes = [C.c_void_p, C.c_void_p]
N.lib().jaad__sbr_debug_attach(ctx.h, dbg.data_ptr())
for _ in range(5):
    ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, None)
torch.cuda.synchronize()
T = dbg.cpu().numpy().reshape(n_cf, 16)[:, [0, 1, 10, 11, 2, 3, 4, 5, 6, 7, 8, 9]].astype(np.int64)
T = T[T[:, -1] > 0]
names = ["start->barrier (noise, record)", "table copy", "record fields, rows issued", "parameter lookups",
         "autocorr (rows wait)", "generation", "envelope estimate", "calculate_gain", "G/Q ring", "assembly",
         "outputs"]
tot = T[:, -1] - T[:, 0]
print(f"channel-frames {len(T)}  wave life median {np.median(tot):.0f} mean {tot.mean():.0f} ticks")
for k, n in enumerate(names):
    dk = T[:, k + 1] - T[:, k]
    print(f"  {n:36s} median {np.median(dk):8.0f}  mean {dk.mean():8.0f}  ({100 * dk.mean() / tot.mean():5.1f} %)")
span = T[:, -1].max() - T[:, 0].min()
print(f"launch span {span} ticks; waves x life / span = {tot.sum() / span:.1f} resident on average")
ctx.close()
