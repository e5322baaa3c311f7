import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmraft_hip.so)")
    config.addinivalue_line("markers", "slow: long CPU test")


def _ensure_built():
    libs = [os.path.join(ROOT, "multiraft_amd", "libmraft_synth.so"),
            os.path.join(ROOT, "oracle", "liboracle.so")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "multiraft_amd", "csrc"),
                               os.path.join("..", "libmraft_synth.so")])


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
