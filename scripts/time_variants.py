"""Time experimental library variants (JAAD_LIB=...) on the C2 workload; prints ms per batch."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CHILD = r'''
import sys, time, numpy as np, torch
sys.path.insert(0, "%s")
from jaadec_amd import native as N
cfgid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # streams (0: the config's default)
p = N.synth_params(cfgid, n_streams=ns) if ns else N.synth_params(cfgid); b = N.synth_batch(p); cfg = N.cfg_for(p)
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
d = {"q": t(b.q), "sf": t(b.sf), "cb": t(b.cb), "ics": t(b.ics)}
if b.ms_used is not None: d["ms_used"] = t(b.ms_used)
ptr = {k: v.data_ptr() for k, v in d.items()}
ptr.setdefault("ms_used", None); ptr["tns"] = None
pcm = torch.empty(b.n_frames * N.pcm_frame_bytes(0, bool(p.sbr)), dtype=torch.uint8, device=dev)
ctx = N.Context(cfg, int(b.stream_slot.max()) + 1)
s = torch.cuda.Stream(dev); torch.cuda.set_stream(s)
for _ in range(5): ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(s)
for _ in range(30): ctx.decode_device(ptr, b, pcm.data_ptr(), pcm.numel(), 0, s.cuda_stream)
ev[1].record(s); torch.cuda.synchronize()
import hashlib
print("%%.4f %%s" %% (ev[0].elapsed_time(ev[1]) / 30, hashlib.blake2b(pcm.cpu().numpy().tobytes(), digest_size=6).hexdigest()))
''' % ROOT

def main():
    libs = sorted((ROOT / ".tmp/exp").glob("lib_*.so"))
    cfgid = sys.argv[1] if len(sys.argv) > 1 else "2"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    streams = sys.argv[3] if len(sys.argv) > 3 else "0"
    for lib in [l for _ in range(rounds) for l in libs]:  # alternate: clock drift hits all alike
        env = dict(os.environ, JAAD_LIB=str(lib))
        r = subprocess.run([sys.executable, "-c", CHILD, cfgid, streams], env=env, capture_output=True, text=True,
                           timeout=300)
        out = r.stdout.strip().splitlines()
        print(f"{lib.stem:28s} {out[-1] if out else 'ERR ' + r.stderr[-300:]} ms", flush=True)

if __name__ == "__main__":
    main()
