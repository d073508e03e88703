"""Distributed DCT-IV kernel vs the oracle's DCT.dct4_kernel restatement (debug helper, GPU box)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import ctypes as C
import numpy as np
import torch
from jaadec_amd import native as N
from oracle import oracle as O

def table(name):
    src = (N.PKG / "csrc" / "tables" / "jaad_sbr_tables.inc").read_text()
    i = src.index(name + "[")
    body = src[src.index("{", i) + 1: src.index("};", i)]
    toks = [t.strip().rstrip("f") for t in body.replace("{", "").replace("}", "").split(",") if t.strip()]
    return np.array([float.fromhex(t) if "x" in t else float(t) for t in toks], np.float32)

dct = np.concatenate([table("JAAD_DCT4_64_TAB"), table("JAAD_DCT_W_RE"), table("JAAD_DCT_W_IM")])
n = 64
rng = np.random.default_rng(0)
re = (rng.standard_normal((n, 32)) * 100).astype(np.float32)
im = (rng.standard_normal((n, 32)) * 100).astype(np.float32)
d = {k: torch.from_numpy(v).cuda() for k, v in dict(dct=dct, re=re, im=im).items()}
ore = torch.zeros(n, 32, device="cuda"); oim = torch.zeros(n, 32, device="cuda")
L = N.lib()
L.jaad__sbr_dct_test.argtypes = [C.c_void_p] * 5 + [C.c_int]
rc = L.jaad__sbr_dct_test(d["dct"].data_ptr(), d["re"].data_ptr(), d["im"].data_ptr(), ore.data_ptr(), oim.data_ptr(), n)
print("rc", rc)
gre, gim = ore.cpu().numpy(), oim.cpu().numpy()
bad = 0
for v in range(n):
    wre, wim = O.sbr_dct4(re[v], im[v])
    dr = np.nonzero(gre[v].view(np.uint32) != wre.view(np.uint32))[0]
    di = np.nonzero(gim[v].view(np.uint32) != wim.view(np.uint32))[0]
    if len(dr) or len(di):
        bad += 1
        if bad <= 3:
            print("vec", v, "re idx", dr, "im idx", di)
            print("  got", gre[v][dr][:4], "want", wre[dr][:4])
print("vectors differing:", bad, "of", n)
