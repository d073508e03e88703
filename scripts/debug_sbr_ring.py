"""Smoothing-ring debug: kernel's ring at frame 1 start vs oracle ring after frame 0 (GPU box)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import ctypes as C
import numpy as np
import torch
from jaadec_amd import native as N
from oracle import oracle as O

p = N.synth_params(4, n_streams=1, frames_per_stream=2)
b = N.synth_batch(p)
s = b.sbr.copy(); s["hdr"]["smoothing_mode"] = 0
b = N.Batch(b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, b.stream_slot, b.frame_begin, b.nch, s)
cfg = N.cfg_for(p)
dbg = torch.zeros(4096, device="cuda")
with N.Context(cfg, 1) as ctx:
    L = N.lib()
    L.jaad__sbr_debug_attach.argtypes = [C.c_void_p, C.c_void_p]
    L.jaad__sbr_debug_attach(ctx.h, dbg.data_ptr())
    got = ctx.decode(b, N.PCM_FLOAT32)
g = dbg.cpu().numpy()[:640].reshape(2, 5, 64)
# oracle: decode frame 0 only, then read the ring
first, _ = b.split_frames(1)
st = O.Streams(1)
O.decode_batch(cfg, first, st, N.PCM_FLOAT32)
Lo = O.lib()
Lo.orc_sbr_debug_ring.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
sbr_ptr = int(np.frombuffer(st.state[0].tobytes()[8192:8200], np.uint64)[0])
ring = np.zeros(640, np.float32)
idx = Lo.orc_sbr_debug_ring(sbr_ptr, 0, ring.ctypes.data)
ring = ring.reshape(2, 5, 64)
print("oracle idx", idx)
kx = 13
for j in range(5):
    print(j, "kernel", g[0, j, kx:kx + 4], "oracle", ring[0, j, :4])
want = O.decode_batch(cfg, b, O.Streams(1), N.PCM_FLOAT32)
print("frames equal:", [bool(np.array_equal(got[i], want[i])) for i in range(2)])
