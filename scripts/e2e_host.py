"""Host-buffer entry (jaad_decode_batch) on the C2 batch: frames/s with pageable and with
registered caller buffers and with buffers from jaad_host_alloc; JAAD_E2E_ITERS calls each (run under rocprofv3 for the copy/kernel
overlap trace: scripts/gpu_e2e_trace.sh)."""
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from jaadec_amd import native as N  # noqa: E402

p = N.synth_params(int(os.environ.get("JAAD_E2E_CONFIG", "2")))
b = N.synth_batch(p)
cfg = N.cfg_for(p)
iters = int(os.environ.get("JAAD_E2E_ITERS", "5"))
with N.Context(cfg, int(b.stream_slot.max()) + 1) as ctx:
    out = np.empty((b.n_frames, N.pcm_frame_bytes(N.PCM_BIG_ENDIAN, bool(cfg.sbr))), np.uint8)
    for mode in ("pageable", "registered", "hostalloc"):
        arrays = [b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, out]
        bb, o = b, out
        if mode == "registered":
            ctx.register(*arrays)
        if mode == "hostalloc":  # batch and PCM in jaad_host_alloc memory (hipHostMalloc)
            bb = ctx.host_batch(b)
            o = ctx.host_array(out.shape, np.uint8)
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            ctx.decode(bb, N.PCM_BIG_ENDIAN, out=o)
            ts.append(time.perf_counter() - t0)
        import hashlib
        digest = hashlib.blake2b(np.asarray(o).tobytes(), digest_size=6).hexdigest()  # PCM of the last call
        if mode == "registered":
            ctx.unregister(*arrays)
        if mode == "hostalloc":
            ctx.free_host(bb.q, bb.sf, bb.cb, bb.ics, bb.ms_used, bb.tns, o)
        print(f"{mode:10s} best {b.n_frames / min(ts):.4g} frames/s  median {b.n_frames / np.median(ts):.4g}  "
              f"({min(ts) * 1e3:.2f} ms per {b.n_frames} frames)  pcm {digest}", flush=True)
