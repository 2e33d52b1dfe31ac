"""The driver's round-end smoke() (one small forward + backward against the CPU oracles) as a GPU
test, so the suite catches a smoke regression before the driver does."""
import pytest


@pytest.mark.gpu
def test_graft_smoke():
    import __graft_entry__ as g
    g.smoke()
