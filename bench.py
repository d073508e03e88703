#!/usr/bin/env python3
"""Benchmark: AAC frames/s of the MI355X DSP path on BASELINE.json's C2 workload.

One "step" = one pass of the hot path (jaad_decode_batch_device: IQ + M/S + IMDCT + window/OLA +
PCM packing) over one 65 536-frame batch (256 streams x 256 frames, AAC-LC 48 kHz stereo, long
windows) with inputs already resident in HBM.

Multi-GPU: one process per GPU.  The job is ONE global batch of N x (per-GPU streams) independent
streams; rank r decodes its shard_runs() slice of it (jaadec_amd/shard.py), generated on the rank
itself (the synthetic generator seeds every stream by its global index, so a rank's slice equals
the same streams of the whole batch).  Weak scaling, no collectives on the data path: the only
collectives are the barrier around the timed region and the max-over-ranks time reduction.

    python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5] [--no-cpu]

`--gpus N` with N > 1 and no torch.distributed environment launches N ranks itself
(torch.distributed.run, before this process touches the GPU) and exits with their status; under
a launcher, WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
# C4 / C5 are compute-leaning: graded against the FP32 VALU roof (MFMA unused) with
# the binary32 operations the reference performs per frame, counted from its loops (round 4, from
# the restatement oracle/jaad_oracle*.c, which follows them operation for operation; C4/C5 headers:
# kx 13, M 32, 2 envelopes, interpol_freq on, smoothing off):
#   core (24 kHz, per channel): IQ 1k + IMDCT (pre/post twiddle 2 x 3.1k, 512-point IFFT 20k) +
#       window/OLA 3.1k                                                             = 30k
#   QMF analysis, 32 slots: 64 x 5-tap window (576) + DCT-IV (pre 192, 32-point FFT 544,
#       post 192) + output scaling (64)                                 = 1.57k/slot = 50k
#   HF generation, 32 high bands: autocorrelation over 38 slots (790) + prediction
#       coefficients (30) + 32 slots of the 2nd-order predictor (516)   = 1.34k/band = 43k
#   HF adjustment: envelope estimate (4.1k) + gains/limiter/boost incl. 3 square roots per band
#       and envelope (1.6k) + assembly (32 x 32 x 10)                               = 16k
#   64-band synthesis, 32 slots: 2 DCT-IV (1.86k) + v-block butterflies (128) + 64 x 10-tap
#       window (1.22k) + input scaling (64)                             = 3.26k/slot = 104k
#   PS (C5): hybrid analysis 10k, decorrelation (all-pass chains of 23 QMF bands + 10 hybrid
#       groups, 48 per slot each: 51k; transient detector 11k), parameter scan 5k, mixing incl.
#       IPD/OPD rotation (71 bands x 24 per slot: 55k), hybrid synthesis 1k          = 133k
# C4 = 2 channels x 243k = 486k; C5 = one core/SBR channel (139k) + PS + two synthesis channels
ALGO_FLOPS = {4: 2 * (30e3 + 50e3 + 43e3 + 16e3 + 104e3), 5: (30e3 + 50e3 + 43e3 + 16e3) + 133e3 + 2 * 104e3}
VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak

WORKLOADS = {
    2: "C2: 65536 AAC-LC 48 kHz stereo frames (256 streams x 256), ONLY_LONG windows",
    3: "C3: 65536 AAC-LC 48 kHz stereo frames (256 streams x 256), LONG/START/SHORT/STOP + TNS data (compat)",
    4: "C4: 32768 HE-AAC v1 frames, 24 kHz AAC-LC stereo core + SBR to 48 kHz (128 streams x 256)",
    5: "C5: HE-AAC v2, 24 kHz mono core + SBR + PS to 48 kHz stereo; 32768 frames per GPU (256 streams x 128), "
       "the 8-GPU job is the 262144-frame batch",
}
PER_GPU_STREAMS = {5: 256}  # C5 is quoted for 8 GPUs: each rank decodes 1/8 of the 2048-stream job


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=sorted(WORKLOADS))
    ap.add_argument("--precision", choices=("lsb1", "exact"), default="lsb1",
                    help="jaad_stream_cfg.precision of the AAC-LC kernel: lsb1 = PCM within +-1 LSB of the "
                         "reference (BASELINE.json's bar; fused multiply-adds in the IMDCT), exact = "
                         "bit-identical; SBR/PS configs (4, 5) always decode exactly")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) leg")
    ap.add_argument("--no-host", action="store_true", help="skip the host front-end (bitstream parse) leg")
    ap.add_argument("--cpu-streams", type=int, default=256, help="streams in the CPU baseline sample")
    ap.add_argument("--settle", type=float, default=0.25,
                    help="seconds of untimed back-to-back steps before the warmup: the GPU's power management "
                         "takes ~60 ms of continuous load to leave its load-onset transient (DESIGN.md 5)")
    # diagnostics / CPU tests only: a smaller job than the config's (the line's config says so)
    ap.add_argument("--streams-per-gpu", type=int, default=0)
    ap.add_argument("--frames-per-stream", type=int, default=0)
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv) -> int:
    """Run this script as args.gpus ranks (one per GPU) and return their exit status.  The parent
    never touches the GPU: it only starts the launcher as a child process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve())] + list(argv)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def shard_params(N, config: int, world: int, rank: int, streams_per_gpu: int = 0, frames_per_stream: int = 0):
    """Synthetic-generator parameters of rank `rank`'s slice of the global job (world x the per-GPU
    stream count), the slice being shard_runs() of the global batch."""
    from jaadec_amd.shard import shard_runs

    over = {}
    if frames_per_stream:
        over["frames_per_stream"] = frames_per_stream
    g = N.synth_params(config, **over)
    per_gpu = streams_per_gpu or PER_GPU_STREAMS.get(config, g.n_streams)
    n_global = per_gpu * world
    fps = g.frames_per_stream
    begin = np.arange(n_global + 1, dtype=np.uint64) * fps  # stream-major, one run per stream
    runs = shard_runs(begin, world, rank)
    p = N.synth_params(config, n_streams=len(runs), first_stream=runs.start if len(runs) else 0, **over)
    return p, n_global


class HipEngine:
    """The product path on one GPU: the batch resident in HBM, jaad_decode_batch_device on a
    non-default stream, HIP events around every timed step."""

    def __init__(self, cfg, batch, flags: int, device: int, n_slots: int):
        import torch

        from jaadec_amd import native as N

        self.torch, self.N = torch, N
        self.dev = torch.device("cuda", device)
        torch.cuda.set_device(self.dev)
        self.batch, self.flags = batch, flags
        self.pcm_bytes = batch.n_frames * N.pcm_frame_bytes(flags, bool(cfg.sbr), N.sbr_downsampled(cfg))

        def to_dev(a):
            if a is None:
                return None
            return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(self.dev)

        self.bufs = {k: to_dev(getattr(batch, k)) for k in ("q", "sf", "cb", "ics", "ms_used", "tns")}
        self.ptr = {k: (v.data_ptr() if v is not None else None) for k, v in self.bufs.items()}
        self.pcm_dev = torch.empty(self.pcm_bytes, dtype=torch.uint8, device=self.dev)
        self.ctx = N.Context(cfg, n_slots, device=device)
        # a real (non-null) stream: the kernels and the timing events must share it
        self.stream = torch.cuda.Stream(self.dev)
        torch.cuda.set_stream(self.stream)
        self.ev = []

    def step(self, timed: bool = False):
        s = self.stream
        if timed:
            a, b = self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True)
            a.record(s)
        self.ctx.decode_device(self.ptr, self.batch, self.pcm_dev.data_ptr(), self.pcm_bytes, self.flags,
                               s.cuda_stream)
        if timed:
            b.record(s)
            self.ev.append((a, b))

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def kernel_ms(self) -> float:
        return float(np.mean([a.elapsed_time(b) for a, b in self.ev])) if self.ev else float("nan")

    def pcm(self) -> np.ndarray:
        return self.pcm_dev.cpu().numpy().reshape(self.batch.n_frames, -1)

    def decode_host(self) -> dict:
        """The drop-in entry (host buffers in, host PCM out): frames/s with the caller's buffers
        page-locked once (jaad_host_register, as a JNI caller pins its direct buffers) and with
        plain pageable buffers (staged).  Best of 5 calls each (PCIe rates vary from call to call)."""
        b = self.batch
        out = np.empty((b.n_frames, self.pcm_bytes // max(b.n_frames, 1)), np.uint8)
        arrays = [b.q, b.sf, b.cb, b.ics, b.ms_used, b.tns, out]

        def best():
            ts = []
            for _ in range(5):
                t1 = time.perf_counter()
                self.ctx.decode(b, self.flags, out=out)
                ts.append(time.perf_counter() - t1)
            return b.n_frames / min(ts)

        pageable = best()
        self.ctx.register(*arrays)
        try:
            registered = best()
        finally:
            self.ctx.unregister(*arrays)
        return {"registered": registered, "pageable": pageable}

    def close(self):
        self.ctx.close()


def run(args, engine_cls=HipEngine):
    """One rank of the benchmark; returns the JSON line on rank 0 (None elsewhere) and this
    rank's PCM after the timed steps.

    The ranks share nothing on the data path (north_star: "RCCL over xGMI not
    required"): the only collectives are the barrier around the timed region, the max-over-ranks
    time and the frame count, three host-side scalars.  They go through a gloo group for every
    world size (round 6), so the code an 8-GPU run executes is exactly the code the
    world-2 gloo tests run (tests/test_bench_multirank.py)."""
    import torch.distributed as dist

    from jaadec_amd import native as N
    from jaadec_amd.shard import reduce_max_time

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("gloo")

    # ---- this rank's slice of the global job
    p, n_global_streams = shard_params(N, args.config, world, rank, args.streams_per_gpu, args.frames_per_stream)
    batch = N.synth_batch(p)
    precision = N.PRECISION_LSB1 if args.precision == "lsb1" and not p.sbr else N.PRECISION_EXACT
    cfg = N.cfg_for(p, precision=precision)
    sbr = bool(p.sbr)
    n_frames = batch.n_frames
    flags = N.PCM_BIG_ENDIAN
    # the host knows its batch's window sequences (a parser writes them): with EIGHT_SHORT frames in a
    # CPE stream the device-entry call says so (JAAD_HINT_SHORT_WINDOWS: the mixed-window kernel
    # instantiation; jaad_decode_batch scans for itself)
    short = bool(n_frames) and cfg.channel_config == 2 and bool((batch.ics["window_sequence"] == N.EIGHT_SHORT_SEQUENCE).any())
    dev_flags = flags | (N.HINT_SHORT_WINDOWS if short else 0)
    eng = engine_cls(cfg, batch, dev_flags, local, int(batch.stream_slot.max()) + 1 if n_frames else 1)

    # ---- parity sample: the first call decodes every stream from a fresh state
    eng.step()
    eng.sync()
    parity = None
    if rank == 0 and n_frames:
        from oracle import oracle as O
        sub = batch.select_runs(sorted({0, len(batch.stream_slot) - 1}))
        want = O.decode_batch(cfg, sub, O.Streams(int(batch.stream_slot.max()) + 1), flags, threads=2)
        got_all = eng.pcm()
        fb = batch.frame_begin
        runs = sorted({0, len(batch.stream_slot) - 1})
        got = np.concatenate([got_all[fb[r]:fb[r + 1]] for r in runs])
        d = np.abs(got.view(">i2").astype(np.int32) - want.view(">i2").astype(np.int32))
        parity = {"frames_checked": int(want.shape[0]), "max_abs_lsb": int(d.max()),
                  "samples_off_by_1": int((d == 1).sum())}

    # ---- load onset: the first steps after the GPU idled (here: while the CPU checked the parity
    # sample) run in the power manager's transient -- reported beside, never as value
    cold = None
    if args.settle > 0 and args.steps:
        t1 = time.perf_counter()
        for _ in range(args.steps):
            eng.step()
        eng.sync()
        cold = (time.perf_counter() - t1) / args.steps * 1e3
    # ---- settle: untimed back-to-back steps until the clock has left that transient
    n_settle, t_settle = 0, time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        for _ in range(10):
            eng.step()
        eng.sync()
        n_settle += 10
    t_settle = time.perf_counter() - t_settle
    for _ in range(max(0, args.warmup - 1)):
        eng.step()
    eng.sync()

    # ---- timed region: exactly K steps between barrier + synchronize
    if world > 1:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step(timed=True)
    eng.sync()
    if world > 1:
        dist.barrier()
    elapsed = reduce_max_time(time.perf_counter() - t0)
    kern_ms = eng.kernel_ms()
    frames_all = n_frames
    if world > 1:
        import torch

        t = torch.tensor([n_frames], dtype=torch.int64)  # (a host scalar: gloo)
        dist.all_reduce(t)
        frames_all = int(t.item())
    pcm = eng.pcm()

    # ---- PCIe-inclusive rate (host buffers in, host PCM out), reported beside, never as value
    e2e = None
    if rank == 0 and not args.no_e2e:
        e2e = eng.decode_host()

    cpu = None
    if rank == 0 and not args.no_cpu:
        from oracle import oracle as O
        ns = min(args.cpu_streams if not sbr else min(args.cpu_streams, 16), len(batch.stream_slot))
        sub = batch.select_runs(range(ns))
        nsl = int(batch.stream_slot.max()) + 1
        t1 = time.perf_counter()
        O.decode_batch(cfg, sub, O.Streams(nsl), flags, threads=1)
        dt1 = time.perf_counter() - t1
        ncores = os.cpu_count() or 1
        # the box's CPU share, not the whole machine's CPUs (os.cpu_count() shows all of them there;
        # the GPU pool sets OMP_NUM_THREADS to the share of one GPU)
        thr = max(1, min(ncores, len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "64") or 64)))
        t1 = time.perf_counter()
        O.decode_batch(cfg, sub, O.Streams(nsl), flags, threads=thr)
        dtn = time.perf_counter() - t1
        cpu = {"value": round(sub.n_frames / dt1, 1), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"{sub.n_frames} frames ({ns} streams x {p.frames_per_stream}) of the same workload, "
                         f"C restatement of the JAAD Java DSP (oracle/, -O2 -ffp-contract=off), 1 thread, "
                         f"parse excluded on both sides",
               "multicore_value": round(sub.n_frames / dtn, 1), "multicore_threads": thr,
               "nproc": ncores, "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_model": cpu_model()}

    host = None
    if rank == 0 and world == 1 and not args.no_host:
        ncores = os.cpu_count() or 1
        thr = max(1, min(ncores, len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "64") or 64)))
        host = host_front_end(args.config, thr, frames_all * args.steps / elapsed)

    # HBM bytes per step measured by rocprofv3 PMC passes of this same command at the same config
    # (scripts/gpu_prof.sh [config] -> scripts/summarize_prof.py -> profiles/current_c<config>.json)
    traffic, traffic_src = None, None
    cur = ROOT / "profiles" / f"current_c{args.config}.json"
    if cur.exists():
        prof = json.loads(cur.read_text())
        if prof.get("frames_per_step", n_frames) == n_frames:  # the profile's workload is this one
            traffic = prof.get("hbm_traffic_bytes_per_launch")
            traffic_src = f"profiles/{prof.get('tag')}.json ({prof.get('hbm_traffic_note')})" if traffic else None

    line = None
    if rank == 0:
        steps = args.steps
        value = frames_all * steps / elapsed
        achieved = ALGO_BYTES[args.config] * n_frames / (kern_ms * 1e-3) / 1e9
        workload = WORKLOADS[args.config]
        if args.streams_per_gpu or args.frames_per_stream:
            workload += f" [reduced: {n_global_streams} streams x {p.frames_per_stream} frames]"
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": workload, "frames_per_gpu": n_frames, "frames_per_job": frames_all,
                       "streams_per_job": n_global_streams,
                       "parallelism": f"stream-sharded x{world} (no collectives)", "pcm": "int16 big-endian",
                       "samples_per_frame": 2048 if sbr else 1024,
                       "lc_kernel": ("mixed-window instantiation (JAAD_HINT_SHORT_WINDOWS: the batch holds EIGHT_SHORT frames)"
                                     if short else "long-window instantiation"),
                       "precision": ("lsb1: PCM within +-1 LSB of the reference (jaad_stream_cfg.precision = "
                                     "JAAD_PRECISION_LSB1, fused multiply-adds in the IMDCT; parity_sample checks it)"
                                     if precision == N.PRECISION_LSB1 else
                                     "exact: PCM bit-identical to the reference's binary32 arithmetic")},
            "roofline": roofline(args.config, n_frames, kern_ms, achieved, traffic, traffic_src),
            "settle": {"steps": n_settle, "seconds": round(t_settle, 3),
                       "cold_ms_per_step": round(cold, 4) if cold is not None else None,
                       "note": "untimed steps before the warmup; cold_ms_per_step = the first K steps after "
                               "the GPU idled (load-onset clock transient), beside the timed steady state"},
            "cpu_baseline": cpu,
            "parity_sample": parity,
            "e2e_pcie_frames_per_s": round(e2e["registered"], 1) if e2e else None,
            "e2e_pcie_pageable_frames_per_s": round(e2e["pageable"], 1) if e2e else None,
            "host_front_end": host,
        }
    eng.close()
    return line, pcm


def host_front_end(config: int, threads: int, gpu_value: float) -> dict | None:
    """The bitstream half of the drop-in (include/jaad_parse.h) on this host, with tools/bench_parse
    over the config's corpus (tests/golden/parse_c<config>.bin: the same synthetic frames, written
    as raw_data_blocks): parse frames/s on 1 and `threads` cores, the cores that would keep one GPU
    fed at `value`, and a measured bitstream -> PCM pipeline (parse threads fill the next batch while
    jaad_decode_batch decodes the current one through host buffers).  Reported beside, never as value."""
    tool, corpus = ROOT / "tools" / "bench_parse", ROOT / "tests" / "golden" / f"parse_c{config}.bin"
    if not tool.exists() or not corpus.exists():
        return None

    def run_tool(*a):
        r = subprocess.run([str(tool), str(corpus), *map(str, a)], capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout) if r.returncode == 0 and r.stdout.strip() else None

    one, many = run_tool(1, 1.0), run_tool(threads, 1.0)
    pipe = run_tool(threads, 2.0, 128 if config == 4 else 256)
    if not one:
        return None
    return {"parse_frames_per_s_1core": one["frames_per_s"], "parse_frames_per_s": many["frames_per_s"] if many else None,
            "parse_threads": threads, "bitstream_bytes_per_frame": one["bytes_per_frame"],
            "bitstream_MB_per_s_1core": one["bitstream_MB_per_s"],
            "cores_to_feed_one_gpu": round(gpu_value / one["frames_per_s"], 1),
            "bitstream_to_pcm_frames_per_s": pipe["bitstream_to_pcm_frames_per_s"] if pipe else None,
            "pipeline": pipe,
            "note": "tools/bench_parse: jaad_parse_frame over tests/golden/parse_c<config>.bin (synthetic frames "
                    "at ~1.4 KB = 530 kb/s stereo: a dense, high-rate workload); pipeline = parse on the threads "
                    "+ jaad_decode_batch (registered host buffers, PCIe both ways), measured"}


def roofline(config: int, n_frames: int, kern_ms: float, gbs: float, traffic, traffic_src) -> dict:
    """The dominant roof of the workload: HBM for the AAC-LC core (C2/C3), FP32 VALU for SBR/PS."""
    common = {"traffic": traffic, "traffic_source": traffic_src,
              "algorithmic_bytes_per_launch": ALGO_BYTES[config] * n_frames, "kernel_ms": round(kern_ms, 4)}
    if config in ALGO_FLOPS:
        tf = ALGO_FLOPS[config] * n_frames / (kern_ms * 1e-3) / 1e12
        return {"bound": "valu", "achieved": round(tf, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(tf / VALU_PEAK_TFLOPS, 4), "flop_per_frame": ALGO_FLOPS[config],
                "hbm_gbs": round(gbs, 1), **common}
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), **common}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    if int(env_world or 1) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    line, _ = run(args)
    if line is not None:
        print(json.dumps(line), flush=True)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
