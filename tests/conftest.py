import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# every swarm node of the suite -- in this process, in its threads and in the bench / example
# subprocesses it starts (they inherit the environment) -- checks its replicated-state
# invariants after every launch_round / complete_round (agent/audit.py; round-5 VERDICT Next 4).
# HLSP2P_AUDIT=0 on the pytest command line turns it off.
os.environ.setdefault("HLSP2P_AUDIT", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native _C kernels")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def rt():
    from hlsjs_p2p_wrapper_amd.ops._native import runtime

    return runtime()


@pytest.fixture(scope="session")
def cuda():
    import torch

    from hlsjs_p2p_wrapper_amd.ops._native import device

    device()  # native kernels must load: no silent fallback
    return torch.device("cuda:0")
