"""bench.py's N>1 path on CPU: world-size-2 gloo ranks through bench.run() (rank env, shard of the
global job, barrier + max-over-ranks timing, the JSON line), with the decode engine swapped for
the CPU restatement (test infrastructure; on the GPU box the same code drives HipEngine over RCCL).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import bench
from jaadec_amd import native as N

SMALL = ["--config", "2", "--steps", "2", "--warmup", "2", "--settle", "0.02", "--no-cpu", "--no-e2e", "--no-host", "--streams-per-gpu", "3",
         "--frames-per-stream", "6"]


class OracleEngine:
    """bench.HipEngine's interface over oracle.decode_batch (stream state carried across steps,
    as the GPU context carries it)."""

    def __init__(self, cfg, batch, flags, device, n_slots):
        from oracle import oracle as O

        self.O, self.cfg, self.batch, self.flags = O, cfg, batch, flags
        self.streams = O.Streams(n_slots)
        self.out = None
        self.n_timed = 0

    def step(self, timed=False):
        self.out = self.O.decode_batch(self.cfg, self.batch, self.streams, self.flags)
        self.n_timed += bool(timed)

    def sync(self):
        pass

    def kernel_ms(self):
        return 1.0

    def pcm(self):
        return self.out.reshape(self.batch.n_frames, -1)

    def decode_host(self):
        return self.pcm()

    def close(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    try:
        line, pcm = bench.run(bench.parse(SMALL + ["--gpus", str(world)]), engine_cls=OracleEngine)
        got = [None] * world
        dist.all_gather_object(got, pcm.tobytes())
        if rank == 0:
            q.put((line, got))
    finally:
        dist.destroy_process_group()


def test_shard_params_slices_the_global_job():
    for config in (2, 4):
        g = N.synth_params(config, n_streams=6, frames_per_stream=3)
        full = N.synth_batch(g)
        for world in (2, 3):
            parts = []
            for r in range(world):
                p, n_glob = bench.shard_params(N, config, world, r, streams_per_gpu=6 // world, frames_per_stream=3)
                assert n_glob == 6
                parts.append(N.synth_batch(p))
            for k in ("q", "sf", "cb", "ics", "ms_used", "sbr"):
                a = getattr(full, k)
                if a is None:
                    continue
                b = np.concatenate([getattr(x, k) for x in parts])
                assert a.tobytes() == b.tobytes(), (config, world, k)


def test_world_size_mismatch_exits_nonzero(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2"])
    assert e.value.code == 2


def test_launcher_command(monkeypatch):
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env):
        seen["cmd"] = cmd
        return R()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "4", "--steps", "3"])
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "3"][-3:]


def test_gloo_world2_bench_line_and_pcm_match_world1(monkeypatch):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    line, got = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["scaling"] == "weak"
    assert line["config"]["frames_per_job"] == 2 * 3 * 6 and line["config"]["frames_per_gpu"] == 3 * 6
    assert line["parity_sample"]["max_abs_lsb"] == 0
    assert line["value"] > 0
    # world 1 over the same global job (6 streams) decodes byte-identically to the two shards
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    args = bench.parse(["--config", "2", "--steps", "2", "--warmup", "2", "--settle", "0.02", "--no-cpu", "--no-e2e", "--no-host",
                        "--streams-per-gpu", "6", "--frames-per-stream", "6"])
    line1, pcm1 = bench.run(args, engine_cls=OracleEngine)
    assert line1["n_gpus"] == 1
    assert b"".join(got) == pcm1.tobytes()


def _gpu_worker(rank, world, port, q):
    # both ranks on the one GPU of the box (LOCAL_RANK 0), gloo for the barrier / reductions
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0")
    import torch.distributed as dist

    try:
        line, pcm = bench.run(bench.parse(SMALL + ["--gpus", str(world)]))
        got = [None] * world
        dist.all_gather_object(got, pcm.tobytes())
        if rank == 0:
            q.put((line, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_world2_bench_path_on_the_hip_engine(monkeypatch):
    """bench.run() on two ranks with the product engine (HipEngine: jaad_decode_batch_device on the
    GPU): the ranks' PCM concatenates to the world-1 PCM of the same global job."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    line, got = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    # (the bench's default precision is lsb1: within 1 LSB of the restatement, byte-identical across ranks)
    assert line["n_gpus"] == 2 and line["parity_sample"]["max_abs_lsb"] <= 1
    assert line["config"]["precision"].startswith("lsb1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    args = bench.parse(["--config", "2", "--steps", "2", "--warmup", "2", "--settle", "0.02", "--no-cpu", "--no-e2e", "--no-host",
                        "--streams-per-gpu", "6", "--frames-per-stream", "6"])
    _, pcm1 = bench.run(args)
    assert b"".join(got) == pcm1.tobytes()
