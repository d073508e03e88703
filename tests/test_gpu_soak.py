"""Randomised differential parity soak: random synthetic batches of every config family (AAC-LC
mono/stereo with window switching, TNS data, PNS, intensity, M/S variants, escapes; HE-AAC v1 with
coupling, frames before the first header and upsampled fallback frames; HE-AAC v2; multichannel AAC-LC
configurations 3-7; random sample rates and output formats) decoded through the C-ABI and compared byte for byte with the
restatement.  Opt-in (it runs for JAAD_SOAK_SECONDS), so the round-end `-m gpu` run is unchanged:

    JAAD_SOAK_SECONDS=240 python -m pytest tests/test_gpu_soak.py -m gpu -s
"""
import os
import time

import numpy as np
import pytest

from jaadec_amd import native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SECS = float(os.environ.get("JAAD_SOAK_SECONDS", "0"))


def _mc_case(rng):
    """A multichannel AAC-LC batch (channel configurations 3-7) from per-element batches."""
    cc = int(rng.integers(3, 8))
    ns, fps = int(rng.integers(1, 5)), int(rng.integers(1, 25))
    els = []
    for k, i in enumerate(N.MC_ELEMENTS[cc]):
        p = N.synth_params(3, n_streams=ns, frames_per_stream=fps, channel_config=2 if i == 1 else 1, pns_percent=0,
                           seed=int(rng.integers(1, 2 ** 62)), ms_mode=int(rng.integers(0, 3)))
        if i == 3:
            p.window_switching = 0
        els.append(N.synth_batch(p))
    return cc, N.mc_batch(els, N.MC_ELEMENTS[cc])


def _case(rng):
    cid = int(rng.choice([2, 3, 3, 4, 4, 5]))
    over = dict(n_streams=int(rng.integers(1, 9)), frames_per_stream=int(rng.integers(1, 41)),
                seed=int(rng.integers(1, 2 ** 62)))
    if cid in (2, 3):
        over.update(channel_config=int(rng.choice([1, 2, 2])), ms_mode=int(rng.integers(0, 3)),
                    pns_percent=int(rng.choice([0, 0, 6])), is_percent=int(rng.choice([0, 12])),
                    escape_permille=int(rng.choice([0, 4])), sf_index=int(rng.choice([3, 4, 5, 6, 8])),
                    common_window=int(rng.choice([0, 1, 1])))
        if over["channel_config"] == 1:
            over["is_percent"] = 0
    elif cid == 4:
        over.update(coupling_percent=int(rng.choice([0, 0, 40])), upsample_percent=int(rng.choice([0, 0, 10])),
                    nohdr_frames=int(rng.choice([0, 0, 3])))
    flags = int(rng.choice([N.PCM_BIG_ENDIAN, N.PCM_LITTLE_ENDIAN, N.PCM_FLOAT32]))
    tns = N.TNS_SPEC if cid == 3 and rng.random() < 0.25 else N.TNS_COMPAT
    return cid, over, flags, tns


@pytest.mark.skipif(SECS <= 0, reason="opt-in soak: set JAAD_SOAK_SECONDS")
def test_random_parity_soak():
    rng = np.random.default_rng(int(os.environ.get("JAAD_SOAK_SEED", "1")))
    t_end = time.time() + SECS
    n = frames = 0
    per = {}
    while time.time() < t_end:
        if rng.random() < 0.15:
            cc, b = _mc_case(rng)
            flags = int(rng.choice([N.PCM_BIG_ENDIAN, N.PCM_LITTLE_ENDIAN, N.PCM_FLOAT32]))
            with N.Context(N.make_cfg(channel_config=cc), int(b.stream_slot.max()) + 1) as ctx:
                got = ctx.decode(b, flags)
            want = O.decode_batch_mc(3, b, N.MC_ELEMENTS[cc], flags)
            assert got.tobytes() == want.tobytes(), f"case {n}: multichannel {cc} flags {flags}"
            n += 1
            frames += b.n_frames
            per[f"mc{cc}"] = per.get(f"mc{cc}", 0) + 1
            continue
        cid, over, flags, tns = _case(rng)
        p = N.synth_params(cid, **over)
        b = N.synth_batch(p)
        cfg = N.cfg_for(p, tns)
        n_slots = int(b.stream_slot.max()) + 1
        with N.Context(cfg, n_slots) as ctx:
            got = ctx.decode(b, flags)
        want = O.decode_batch(cfg, b, O.Streams(n_slots), flags)
        assert got.tobytes() == want.tobytes(), f"case {n}: C{cid} {over} flags {flags} tns {tns}"
        n += 1
        frames += b.n_frames
        per[cid] = per.get(cid, 0) + 1
        if n % 25 == 0:  # progress (a silent GPU job looks hung)
            print(f"soak: {n} batches, {frames} frames", flush=True)
    print(f"\nsoak: {n} random batches ({frames} frames, per config {dict(sorted(per.items(), key=str))}) byte-identical to the restatement")
    assert n > 0
