import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# the pre-warmed zygote (kubelet launch-delay optimisation) imports torch in a
# side process; tests opt in explicitly (tests/test_zygote.py)
os.environ.setdefault("KDL_ZYGOTE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "multigpu: ranks on distinct GPUs; skips itself below its world size "
                                       "(tests/test_multigpu.py)")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU on this host")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
