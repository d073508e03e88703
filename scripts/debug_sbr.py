"""SBR GPU-vs-oracle float diff statistics (debug helper, run on the GPU box)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
from jaadec_amd import native as N
from oracle import oracle as O

p = N.synth_params(4, n_streams=4, frames_per_stream=40)
b = N.synth_batch(p)
cfg = N.cfg_for(p)
with N.Context(cfg, 4) as ctx:
    got = ctx.decode(b, N.PCM_FLOAT32).view(np.float32).reshape(b.n_frames, 2048, 2)
want = O.decode_batch(cfg, b, O.Streams(4), N.PCM_FLOAT32).view(np.float32).reshape(b.n_frames, 2048, 2)
d = got != want
print("differing floats:", d.sum(), "of", d.size)
fr, smp, ch = np.nonzero(d)
print("frames:", np.unique(fr)[:40])
print("per-frame counts:", np.bincount(fr, minlength=b.n_frames)[:80])
print("channels:", np.bincount(ch, minlength=2))
if d.sum():
    g, w = got[d], want[d]
    ulp = np.abs(g.view(np.int32).astype(np.int64) - w.view(np.int32).astype(np.int64))
    print("max ulp", ulp.max(), "median", np.median(ulp), "max abs", np.abs(g - w).max())
    f0 = fr[0]
    print("first frame", f0, "samples", smp[fr == f0][:20], "slots", np.unique(smp[fr == f0] // 64))
    print("frame-in-stream:", np.unique(fr % 40))
