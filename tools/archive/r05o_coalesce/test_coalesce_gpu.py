"""Group-committed Token calls on the kernels: 16 threads of mixed
encrypt / decrypt / verify_hmac with their own keys (AES-256 and -128), every
result against the C oracle and every failure with Token's message
(tests/test_coalesce.py has the CPU half)."""
import pytest

pytestmark = pytest.mark.gpu


def test_coalesced_threads_on_the_gpu():
    import test_coalesce as tc
    from reticulum_amd import coalesce
    coalesce._coalescers.clear()
    tc._run_threads(coalesce.CoalescingToken, 16, 25)
    st = coalesce.coalescer().stats
    assert st["calls"] == 16 * 25 * 5 and st["batches"] < st["calls"]
