#!/usr/bin/env python3
"""Benchmark: AAC frames/s of the MI355X DSP path on BASELINE.json's C2 workload.

One "step" = one pass of the hot path (jaad_decode_batch_device: IQ + M/S + IMDCT + window/OLA +
PCM packing) over one 65 536-frame batch (256 streams x 256 frames, AAC-LC 48 kHz stereo, long
windows) with inputs already resident in HBM.  Multi-GPU: one process per GPU, each rank decodes
its own 65 536-frame shard of independent streams (weak scaling, no collectives on the data
path; the only collectives are the barrier and the max-over-ranks timing reduction).

    python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5] [--no-cpu]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "AAC frames/sec (batched) at 1/2/4/8 MI355X; PCM ±1 LSB vs Java ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes per frame.  C2/C3 long stereo frame = 2 x 4308 + 8 (q, gains,
# side info, PCM); C4 (core + SBR, stereo) = 2 x (2048 q + 188 gains + 16 side + 1300 SBR params
# + 4096 PCM) = 15296; C5 (mono core + SBR + PS -> stereo) = 2048 q + 188 gains + 16 side + 1300 SBR
# params + 352 PS params + 8192 PCM = 12096
ALGO_BYTES = {2: 8624, 3: 8624, 4: 15296, 5: 12096}

WORKLOADS = {
    2: "C2: 65536 AAC-LC 48 kHz stereo frames (256 streams x 256), ONLY_LONG windows",
    3: "C3: 65536 AAC-LC 48 kHz stereo frames (256 streams x 256), LONG/START/SHORT/STOP + TNS data (compat)",
    4: "C4: 32768 HE-AAC v1 frames, 24 kHz AAC-LC stereo core + SBR to 48 kHz (128 streams x 256)",
    5: "C5: HE-AAC v2, 24 kHz mono core + SBR + PS to 48 kHz stereo; 32768 frames per GPU (256 streams x 128), "
       "the 8-GPU job is the 262144-frame batch",
}
SHARD_OVERRIDES = {5: {"n_streams": 256}}  # C5 is quoted for 8 GPUs: each rank decodes 1/8 of it


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-streams", type=int, default=256, help="streams in the CPU baseline sample")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from jaadec_amd import native as N

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    # ---- this rank's shard: its own 256 independent streams (seeded by rank)
    p = N.synth_params(args.config, **SHARD_OVERRIDES.get(args.config, {}))
    p.seed = p.seed + 0x1000 * rank
    batch = N.synth_batch(p)
    cfg = N.cfg_for(p)
    sbr = bool(p.sbr)
    n_frames = batch.n_frames
    flags = N.PCM_BIG_ENDIAN
    pcm_bytes = n_frames * N.pcm_frame_bytes(flags, sbr)
    ALGO_BYTES_PER_FRAME = ALGO_BYTES[args.config]

    def to_dev(a):
        if a is None:
            return None
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
        return t

    dq, dsf, dcb, dics, dms = (to_dev(batch.q), to_dev(batch.sf), to_dev(batch.cb), to_dev(batch.ics),
                               to_dev(batch.ms_used))
    dtns = to_dev(batch.tns)
    dptr = {"q": dq.data_ptr(), "sf": dsf.data_ptr(), "cb": dcb.data_ptr(), "ics": dics.data_ptr(),
            "ms_used": dms.data_ptr() if dms is not None else None, "tns": dtns.data_ptr() if dtns is not None else None}
    pcm = torch.empty(pcm_bytes, dtype=torch.uint8, device=dev)
    ctx = N.Context(cfg, int(batch.stream_slot.max()) + 1, device=dev.index)
    # a real (non-null) stream: the kernels and the timing events must share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    # ---- parity sample: the first call decodes every stream from a fresh state
    ctx.decode_device(dptr, batch, pcm.data_ptr(), pcm_bytes, flags, sptr)
    torch.cuda.synchronize(dev)
    parity = None
    if rank == 0:
        from oracle import oracle as O
        sub = batch.select_runs([0, len(batch.stream_slot) - 1])
        want = O.decode_batch(cfg, sub, O.Streams(ctx.n_slots), flags, threads=2)
        got_all = pcm.cpu().numpy().reshape(n_frames, -1)
        fb = batch.frame_begin
        got = np.concatenate([got_all[fb[0]:fb[1]], got_all[fb[-2]:fb[-1]]])
        d = np.abs(got.view(">i2").astype(np.int32) - want.view(">i2").astype(np.int32))
        parity = {"frames_checked": int(want.shape[0]), "max_abs_lsb": int(d.max()),
                  "samples_off_by_1": int((d == 1).sum())}

    for _ in range(max(0, args.warmup - 1)):
        ctx.decode_device(dptr, batch, pcm.data_ptr(), pcm_bytes, flags, sptr)
    torch.cuda.synchronize(dev)

    # ---- timed region: exactly K steps between barrier + synchronize
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        ctx.decode_device(dptr, batch, pcm.data_ptr(), pcm_bytes, flags, sptr)
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # ---- PCIe-inclusive rate (host buffers in, host PCM out), reported beside, never as value
    e2e_fps = None
    if rank == 0:
        t1 = time.perf_counter()
        ctx.decode(batch, flags)
        e2e_fps = n_frames / (time.perf_counter() - t1)

    cpu = None
    if rank == 0 and not args.no_cpu:
        from oracle import oracle as O
        ns = min(args.cpu_streams if not sbr else min(args.cpu_streams, 16), len(batch.stream_slot))
        sub = batch.select_runs(range(ns))
        t1 = time.perf_counter()
        O.decode_batch(cfg, sub, O.Streams(ctx.n_slots), flags, threads=1)
        dt1 = time.perf_counter() - t1
        ncores = os.cpu_count() or 1
        thr = min(ncores, 64)
        t1 = time.perf_counter()
        O.decode_batch(cfg, sub, O.Streams(ctx.n_slots), flags, threads=thr)
        dtn = time.perf_counter() - t1
        cpu = {"value": round(sub.n_frames / dt1, 1), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"{sub.n_frames} frames ({ns} streams x {p.frames_per_stream}) of the same workload, "
                         f"C restatement of the JAAD Java DSP (oracle/, -O2 -ffp-contract=off), 1 thread, "
                         f"parse excluded on both sides",
               "multicore_value": round(sub.n_frames / dtn, 1), "multicore_threads": thr}

    # HBM bytes per launch measured by rocprofv3 PMC passes of this same command
    # (scripts/gpu_prof.sh -> scripts/summarize_prof.py -> profiles/current.json)
    traffic, traffic_src = None, None
    cur = ROOT / "profiles" / "current.json"
    if cur.exists() and args.config == 2:
        prof = json.loads(cur.read_text())
        traffic = prof.get("hbm_traffic_bytes_per_launch")
        traffic_src = f"profiles/{prof.get('tag')}.json ({prof.get('hbm_traffic_note')})" if traffic else None

    if rank == 0:
        steps = args.steps
        total_frames = n_frames * world * steps
        value = total_frames / elapsed
        achieved = ALGO_BYTES_PER_FRAME * n_frames / (kern_ms * 1e-3) / 1e9
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": WORKLOADS[args.config], "frames_per_gpu": n_frames,
                       "parallelism": f"stream-sharded x{world} (no collectives)", "pcm": "int16 big-endian",
                       "samples_per_frame": 2048 if sbr else 1024},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": ALGO_BYTES_PER_FRAME * n_frames,
                         "kernel_ms": round(kern_ms, 4)},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "e2e_pcie_frames_per_s": round(e2e_fps, 1) if e2e_fps else None,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
