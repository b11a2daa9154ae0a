"""CPU checks of the c5 arrival model: the packaged MMPP (rlks/data/locust_mmpp.json) is exactly
what tools/fit_locust_mmpp.py derives from the reference's Locust history (committed as the data
fixture tests/golden/locust_history.npz), and bursty_trace() follows it."""
import json
import sys

import numpy as np

from conftest import GOLDEN, ROOT


def _fit():
    sys.path.insert(0, str(ROOT / "tools"))
    import fit_locust_mmpp

    z = np.load(GOLDEN / "locust_history.npz")
    series = {c: {k: z[f"{c}_{k}"] for k in ("users", "total", "ts")} for c in ("aws", "azure")}
    return fit_locust_mmpp.fit(series), series


def test_packaged_mmpp_is_the_fit_of_the_locust_history():
    from rlks.env import locust_mmpp

    fitted, series = _fit()
    assert json.loads(json.dumps(fitted)) == locust_mmpp()
    # the history itself: a 5 users/s ramp to 20 users, then ~10 requests/s
    u = series["aws"]["users"]
    assert list(u[:6]) == [0, 5, 10, 15, 20, 20] and u.max() == 20
    m = locust_mmpp()
    assert m["states"] == [0, 5, 10, 15, 20]
    assert abs(m["rate"]["pooled"]["20"] - 9.94) < 0.05
    # under-dispersed plateau: no hidden (burst) rate state is identifiable
    assert all(d["index"] < 1 for d in m["dispersion"].values())


def test_bursty_trace_follows_the_chain():
    from rlks.env import NodeSpec, bursty_trace, locust_mmpp

    lam = bursty_trace(100, base=1.0)
    r = locust_mmpp()["rate"]["pooled"]
    top = r["20"]
    np.testing.assert_allclose(lam[:5], [0.0, r["5"] / top, r["10"] / top, r["15"] / top, 1.0], rtol=0, atol=0)
    assert np.all(lam[4:] == 1.0) and np.all(np.diff(lam[:5]) > 0)
    assert np.array_equal(bursty_trace(100, base=3.0), 3.0 * lam)
    # the stationary departure probability balances the trace's mean rate
    spec = NodeSpec(64, 1024, arrival_trace=lam, depart_prob="stationary")
    assert abs(spec.depart_prob - lam.mean() / spec.expected_initial_pods()) < 1e-15
