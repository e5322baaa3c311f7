"""The top of the engine's Index domain on the GPU (include/mraft.h: every
Raft Index up to 2^31 - 2, so that nextIndex = Index + 1 is an int32): the
fused tick with its highest Index 0, 3 and 7 below that bound, and the
malformed items just past it, GPU == oracle (tests/index_domain_cases.py).
The streaming pass runs on Indexes relative to its first one (mraft_pass.h
pass_bias), so chunk ends (c + 256) never overflow there; the message path's
cases are test_message_path_gpu.py::test_handle_high_indices_gpu."""
import pytest

from index_domain_cases import malformed_case, tick_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("j", [0, 3, 7])
def test_tick_top_of_index_domain_gpu(j):
    assert tick_case(j) > 0  # some group committed at those Indexes


def test_past_index_domain_gpu():
    malformed_case()
