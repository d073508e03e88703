"""Committed fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py)."""
import importlib.util
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

HERE = Path(__file__).resolve().parent
GOLD = sorted(g for g in (HERE / "golden").glob("*.npz") if not g.stem.endswith(("_raw_frame", "_adts_stream")))


def _load(path):
    spec = importlib.util.spec_from_file_location("make_golden", HERE / "golden" / "make_golden.py")
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg.load(path)


def test_fixtures_exist():
    assert len(GOLD) >= 5


@pytest.mark.parametrize("path", GOLD, ids=[p.stem for p in GOLD])
def test_oracle_reproduces_fixture(path):
    b, cfg, flags, pcm = _load(path)
    got = O.decode_batch(cfg, b, O.Streams(int(b.stream_slot.max()) + 1), flags)
    assert got.tobytes() == pcm.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLD, ids=[p.stem for p in GOLD])
def test_hip_path_reproduces_fixture(path):
    from jaadec_amd import native as N

    b, cfg, flags, pcm = _load(path)
    with N.Context(cfg, int(b.stream_slot.max()) + 1) as ctx:
        got = ctx.decode(b, flags)
    assert got.tobytes() == pcm.tobytes()


def test_c1_fixture_is_two_identical_channels():
    """A mono AAC-LC stream is emitted as 2 channels (A/DecoderConfig.java:108-115)."""
    p = [g for g in GOLD if g.stem.startswith("c1")][0]
    b, cfg, flags, pcm = _load(p)
    s = pcm.view(">i2").reshape(-1, 1024, 2)
    assert (s[..., 0] == s[..., 1]).all() and np.abs(s).max() > 0
