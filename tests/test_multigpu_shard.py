"""N>1 path on CPU: world_size-2 gloo processes, stream-sharded decode, byte-identical PCM.

The per-rank decode here is the CPU restatement (test infrastructure); on the GPU box the same
sharding feeds jaad_decode_batch_device on each rank's own device (bench.py).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from jaadec_amd import native as N
from jaadec_amd.shard import rank_batch, reduce_max_time, shard_runs


def test_shard_runs_partition_and_balance():
    begin = np.cumsum([0] + [7, 3, 12, 1, 9, 5, 8, 2, 11, 6]).astype(np.uint32)
    for world in (1, 2, 3, 4, 8):
        parts = [shard_runs(begin, world, r) for r in range(world)]
        flat = [i for p in parts for i in p]
        assert flat == list(range(10))  # contiguous, disjoint, complete, in order
    p = [shard_runs(np.arange(0, 2049, 8, dtype=np.uint32), 8, r) for r in range(8)]
    assert all(len(x) == 32 for x in p)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        p = N.synth_params(3, n_streams=6, frames_per_stream=9, pns_percent=3)
        full = N.synth_batch(p)
        mine = rank_batch(full, world, rank)
        cfg = N.make_cfg()
        pcm = O.decode_batch(cfg, mine, O.Streams(6), N.PCM_BIG_ENDIAN)
        t = reduce_max_time(0.5 + rank)
        got = [None] * world
        dist.all_gather_object(got, (list(mine.stream_slot), pcm.tobytes()))
        if rank == 0:
            q.put((got, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_world2_sharded_decode_is_byte_identical(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got, tmax = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert tmax == 0.5 + (world - 1)  # max over ranks
    from oracle import oracle as O
    p = N.synth_params(3, n_streams=6, frames_per_stream=9, pns_percent=3)
    full = N.synth_batch(p)
    want = O.decode_batch(N.make_cfg(), full, O.Streams(6), N.PCM_BIG_ENDIAN).tobytes()
    slots = [s for g in got for s in g[0]]
    assert slots == list(range(6))
    assert b"".join(g[1] for g in got) == want


@pytest.mark.gpu
def test_gpu_c5_whole_job_as_eight_shards():
    """the whole C5 job (HE-AAC v2, 2048 streams x 128 frames = 262 144 frames) on
    the HIP engine, once in one context and once as the 8 shard_runs slices of an 8-GPU run (each
    slice in its own context, one after the other on this GPU): the slices' PCM concatenates to the
    single-context PCM, and a sample of streams equals the restatement (0 LSB)."""
    from oracle import oracle as O
    p = N.synth_params(5)  # 2048 streams x 128 frames
    full = N.synth_batch(p)
    assert full.n_frames == 262144
    cfg = N.cfg_for(p)
    with N.Context(cfg, len(full.stream_slot)) as ctx:
        one = ctx.decode(full, N.PCM_BIG_ENDIAN)
    parts = []
    for r in range(8):
        mine = rank_batch(full, 8, r)
        assert len(mine.stream_slot) == 256
        with N.Context(cfg, len(full.stream_slot)) as ctx:
            parts.append(ctx.decode(mine, N.PCM_BIG_ENDIAN))
    assert np.array_equal(np.concatenate(parts), one)
    sample = [0, 511, 1024, 2047]
    want = O.decode_batch(cfg, full.select_runs(sample), O.Streams(len(full.stream_slot)), N.PCM_BIG_ENDIAN, threads=4)
    fb = full.frame_begin
    got = np.concatenate([one[fb[r]:fb[r + 1]] for r in sample])
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_two_contexts_from_two_threads():
    """INTEGRATION s6 "(or thread)": two contexts on one GPU driven from two host threads at once
    (AAC-LC and HE-AAC v1), five calls each; every call's PCM equals the single-threaded decode."""
    import threading
    jobs = []
    for config, ns in ((2, 64), (4, 16)):
        p = N.synth_params(config, n_streams=ns, frames_per_stream=64)
        b = N.synth_batch(p)
        with N.Context(N.cfg_for(p), ns) as ctx:
            want = [ctx.decode(c, N.PCM_BIG_ENDIAN) for c in b.split_frames(32)]
        jobs.append((N.cfg_for(p), ns, b, want))
    errors = []

    def run(cfg, ns, b, want):
        try:
            a1, a2 = b.split_frames(32)
            with N.Context(cfg, ns) as ctx:
                for _ in range(5):
                    for s in range(ns):
                        ctx.state_reset(s)
                    g1 = ctx.decode(a1, N.PCM_BIG_ENDIAN)
                    g2 = ctx.decode(a2, N.PCM_BIG_ENDIAN)
                    if not (np.array_equal(g1, want[0]) and np.array_equal(g2, want[1])):
                        errors.append("PCM differs")
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    th = [threading.Thread(target=run, args=j) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th)
    assert not errors, errors
