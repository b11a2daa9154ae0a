import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "rl-k8s-scheduler_amd"
for p in (str(ROOT), str(PKG), str(ROOT / "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden_table():
    t = np.load(GOLDEN / "table.npz")["table"]
    return t


@pytest.fixture(scope="session")
def golden_cost_lat(golden_table):
    t = golden_table
    cost = np.ascontiguousarray(t[:, [1, 2]])
    lat = np.ascontiguousarray(t[:, [3, 4]])
    return cost, lat


@pytest.fixture(scope="session")
def traces():
    return np.load(GOLDEN / "traces.npz")


@pytest.fixture(scope="session")
def traces_meta():
    return json.loads((GOLDEN / "traces_meta.json").read_text())


@pytest.fixture(scope="session")
def mt_draws():
    return np.load(GOLDEN / "mt_draws.npz")


@pytest.fixture(autouse=True)
def _device_bounds_checks(request):
    """with RLKS_LIB pointing at librlks_debug.so (make -C csrc debug), every GPU test must end
    with no device-side bounds-check violation (rlks_debug_checks; rlks_internal.h DcheckSite)"""
    yield
    import os

    if "debug" not in os.environ.get("RLKS_LIB", "") or request.node.get_closest_marker("gpu") is None:
        return
    import ctypes as C

    from rlks import _lib

    out = (C.c_ulonglong * 3)()
    _lib.call("rlks_debug_checks", out)
    assert out[0] == 0, f"{out[0]} device bounds-check violations; first at site {out[1]} (value {out[2]})"
