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


# MRAFT_TEST_TICK_MODE=light runs every engine the tests create in
# MRAFT_TICK_LIGHT (mraft_set_tick_mode): the whole GPU suite then checks the
# light tick against the oracle wherever it checks the full one.
if os.environ.get("MRAFT_TEST_TICK_MODE") == "light":
    from multiraft_amd import engine as _engine_mod

    _engine_init = _engine_mod.Engine.__init__

    def _light_init(self, *a, **k):
        _engine_init(self, *a, **k)
        self.set_tick_mode(1)

    _engine_mod.Engine.__init__ = _light_init
