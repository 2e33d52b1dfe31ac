"""Shared test setup.

Markers: `gpu` = needs a HIP device (run on the MI355X box with `pytest -m gpu`); everything else
runs on CPU.  The oracle (oracle/dladmm_oracle.py) is imported here only as the checker.
"""
import importlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def pytest_collection_modifyitems(config, items):
    if has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def dl():
    """The product package (directory name is not an identifier)."""
    return importlib.import_module("d-ladmm_amd")


@pytest.fixture(scope="session")
def oracle():
    from oracle import dladmm_oracle
    return dladmm_oracle


@pytest.fixture(scope="session")
def problems():
    import problems as P
    return P


class _PlanFlags:
    """Plan options (include/dladmm.h dladmm_flags) for the rest of a test, the way
    monkeypatch.setenv sets a variable: `flags.set(per_layer=True)` ... `flags.set(per_layer=False)`;
    everything is undone at teardown (d-ladmm_amd.ops.plan_flags' context variable)."""

    def __init__(self):
        self.ops = importlib.import_module("d-ladmm_amd.ops")
        self.first = None

    def set(self, **opts):
        var = self.ops._PLAN_FLAGS
        cur = var.get()
        for k, v in opts.items():
            f = self.ops._FLAG_NAMES[k]
            cur = (cur | f) if v else (cur & ~f)
        tok = var.set(cur)
        if self.first is None:
            self.first = tok

    def undo(self):
        if self.first is not None:
            self.ops._PLAN_FLAGS.reset(self.first)
            self.first = None


@pytest.fixture
def flags():
    f = _PlanFlags()
    yield f
    f.undo()


def load_golden(name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = json.loads(str(g["meta"]))
    return g, meta


def pytest_sessionfinish(session, exitstatus):
    """DLADMM_PARITY_JSON=<path>: write every error the parity tests checked (tests/parity.py)."""
    path = os.environ.get("DLADMM_PARITY_JSON")
    if not path:
        return
    import parity
    if parity.LOG:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(parity.LOG, f)
