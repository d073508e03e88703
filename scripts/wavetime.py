"""Per-wave lifetime of a JAAD_WAVETIME build (JAAD_LIB=...) on the C2 batch: s_memrealtime
(100 MHz) at the first and last instruction of each wave, relative to the earliest start."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from jaadec_amd import native as N  # noqa: E402

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
nw = 8192
dbg = torch.zeros(nw * 8, dtype=torch.int32, device=dev)
N.lib().jaad__debug_attach.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
N.lib().jaad__debug_attach(ctx.h, dbg.data_ptr(), -1)
import time
t_end = time.perf_counter() + 0.4  # past the clock's load-onset transient, then the measured call
while time.perf_counter() < t_end:
    for _ in range(10):
        ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, None)
    torch.cuda.synchronize()
ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, None)
torch.cuda.synchronize()
S = dbg.cpu().numpy().view(np.uint64).reshape(nw, 4).astype(np.int64)
S = S[S[:, 0] > 0]
t0 = S[:, 0].min()
st, en = (S[:, 0] - t0) / 100.0, (S[:, 1] - t0) / 100.0  # us
life = en - st
print(f"waves {len(S)}  kernel span {en.max():.1f} us")
print(f"start: p50 {np.median(st):.1f} p99 {np.percentile(st, 99):.1f} max {st.max():.1f} us")
print(f"end:   min {en.min():.1f} p10 {np.percentile(en, 10):.1f} p50 {np.median(en):.1f} p90 {np.percentile(en, 90):.1f} max {en.max():.1f} us")
print(f"life:  mean {life.mean():.1f} = {100 * life.sum() / (len(S) * en.max()):.1f} % of span x waves")
xcc, nf = S[:, 2] & 15, S[:, 3]
for x in range(8):
    m = xcc == x
    if m.any(): print(f"  xcc {x}: waves {m.sum()} end p50 {np.median(en[m]):.1f} max {en[m].max():.1f}  us/frame {np.median(life[m] / np.maximum(nf[m], 1)):.2f}")
idx = np.flatnonzero(dbg.cpu().numpy().view(np.uint64).reshape(nw, 4)[:, 0] > 0)
for sl in range(3):  # waves w, w+4, w+8 of a 12-wave workgroup share a SIMD
    m = (idx % 12) // 4 == sl
    if m.any(): print(f"  simd slot {sl}: waves {m.sum()} end p50 {np.median(en[m]):.1f} frames mean {nf[m].mean():.2f}")
for k in sorted(set(nf.tolist())):
    m = nf == k
    print(f"  frames {k}: waves {m.sum()} end p50 {np.median(en[m]):.1f}")
h, e = np.histogram(en, bins=12)
for c, lo in zip(h, e): print(f"  end {lo:7.1f} us: {c}")
