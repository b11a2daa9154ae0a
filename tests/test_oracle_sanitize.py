"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer: every entry
point of oracle/rlks_oracle.c driven by oracle/oracle_selftest.c, built by `make -C oracle
sanitize` with -fno-sanitize-recover=all, so any report fails the run."""
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def test_oracle_clean_under_asan_ubsan(tmp_path, golden_cost_lat):
    r = subprocess.run(["make", "-C", str(ROOT / "oracle"), "sanitize"], capture_output=True, text=True)
    if r.returncode != 0 and "asan" in (r.stderr + r.stdout).lower():
        pytest.skip("this toolchain has no libasan")
    assert r.returncode == 0, r.stderr
    cost, lat = golden_cost_lat
    tab = tmp_path / "table.bin"
    np.concatenate([cost.ravel(), lat.ravel()]).astype(np.float64).tofile(tab)
    out = subprocess.run([str(ROOT / "oracle/_build/oracle_selftest_san"), str(tab)], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    # the round-robin episode return of the reference (train_and_compare.py:65)
    assert "round_robin_return 4765.215199784463" in out.stdout
