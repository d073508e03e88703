import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the native libraries exist (in-tree build; cheap when up to date)."""
    from jaadec_amd import build
    if not (build.LIB.exists() and build.ORACLE_LIB.exists() and build.SYNTH_LIB.exists()) or os.environ.get("JAAD_REBUILD"):
        build.build_all()
    # torch ships its own HIP runtime: bring it up before libjaadgpu's (/opt/rocm) runtime opens
    # the device, as bench.py does, so tests that use both see the GPU whatever their order
    if config_has_gpu_marker():
        try:
            import torch
            if torch.cuda.device_count() > 0:
                torch.cuda.init()
        except Exception:
            pass
    yield


def config_has_gpu_marker() -> bool:
    return "gpu" in " ".join(sys.argv) and "not gpu" not in " ".join(sys.argv)


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
