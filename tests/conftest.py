import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True


@pytest.fixture
def knob():
    """Set library tuning knobs (pfscdc_set_knob) for one test; restored afterwards.
    knob("PFSCDC_SCAN_GRID", 1); a value of None restores the knob's default."""
    from pfs_amd import _lib

    old = {}
    info = _lib.knob_info()

    def set_(name, value):
        if name not in old:
            old[name] = _lib.get_knob(name)
        _lib.set_knob(name, info[name][2] if value is None else int(value))

    yield set_
    for k, v in old.items():
        _lib.set_knob(k, v)


def fuzz_cases(default: int):
    """Seeds of a randomised parity test: range(default), or PFS_FUZZ_CASES seeds from
    PFS_FUZZ_FIRST (default 0) for a longer soak
    (PFS_FUZZ_CASES=60 PFS_FUZZ_FIRST=1000 python -m pytest -m gpu -k random ...)."""
    import os

    n = os.environ.get("PFS_FUZZ_CASES")
    first = int(os.environ.get("PFS_FUZZ_FIRST", "0"))
    return range(first, first + (int(n) if n else default))
