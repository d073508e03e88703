"""Are __fsqrt_rn / __fdiv_rn correctly rounded on this device? (debug helper, GPU box)"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import ctypes as C
import numpy as np
import torch
from jaadec_amd import native as N
n = 1 << 20
rng = np.random.default_rng(0)
a = np.exp(rng.uniform(-40, 40, n)).astype(np.float32)
b = np.exp(rng.uniform(-20, 20, n)).astype(np.float32)
ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
sq, dv = torch.empty_like(ta), torch.empty_like(ta)
L = N.lib()
L.jaad__math_test.argtypes = [C.c_void_p] * 4 + [C.c_int]
print("rc", L.jaad__math_test(ta.data_ptr(), tb.data_ptr(), sq.data_ptr(), dv.data_ptr(), n))
want_sq = np.sqrt(a.astype(np.float64)).astype(np.float32)
want_dv = (a.astype(np.float64) / b.astype(np.float64)).astype(np.float32)
gs, gd = sq.cpu().numpy(), dv.cpu().numpy()
print("dsqrt mismatches", (gs != want_sq).sum(), "sqrtf mismatches", (gd != want_sq).sum())
i = np.flatnonzero(gs != want_sq)[:3]
print(a[i], gs[i], want_sq[i])
