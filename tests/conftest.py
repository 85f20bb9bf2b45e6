import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libmde_hip.so")


def load_golden(name):
    path = os.path.join(GOLDEN, name)
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]

    return get


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_sessionstart(session):
    """Build libmde_hip.so if this checkout has not built it yet (hipcc cross-compiles)."""
    import subprocess
    lib = os.path.join(REPO, "monocular_depth_estimation_amd", "libmde_hip.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(REPO, "monocular_depth_estimation_amd", "csrc"),
                        "-j8"], check=True)
