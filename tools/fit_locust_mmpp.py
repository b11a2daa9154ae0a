#!/usr/bin/env python3
"""Derive the c5 arrival model (BASELINE configs[4], "bursty Locust-style load traces") from the
reference's Locust runs and write it as a package fixture.

Input (read-only, this container only): /root/reference/data/local_{aws,azure}_load_stats_history.csv
— one row per second: Timestamp, User Count, ..., Total Request Count.

Model: a Markov-modulated Poisson process whose modulating state is Locust's active user count.
  * states      = the user counts observed (0, 5, 10, 15, 20: the 5 users/s spawn ramp, then 20);
  * transitions = maximum-likelihood estimate from consecutive rows (counts of u_i -> u_{i+1},
                  row-normalised);
  * state rate  = mean requests per second over the intervals that end in that state
                  (increments of Total Request Count / elapsed seconds), per cloud and pooled;
  * dispersion  = variance / mean of the per-second counts on the plateau.  An MMPP is
                  over-dispersed (index >= 1) whenever a hidden rate switch exists; the runs show
                  0.47-0.50 (Locust users wait U(1, 3) s, a renewal process more regular than
                  Poisson), so no hidden burst state is identifiable and the fitted chain is the
                  observed ramp + plateau.
The env consumes it through rlks.env.bursty_trace(): lambda[t] = base * rate(state(t)) /
rate(plateau), state(t) the chain's state t steps after a reset (one env step = one Locust second;
the fitted chain is deterministic, so its per-lane realisation is this one sequence).

Writes rl-k8s-scheduler_amd/rlks/data/locust_mmpp.json and the per-second series it was fitted on
to tests/golden/locust_history.npz (data, so that tests re-derive the fit without the reference).
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/data")


def fit(series: dict) -> dict:
    """series: cloud -> dict(users [n], total [n], ts [n]) per-second rows -> the MMPP dict"""
    out = {"states": None, "transitions": None, "rate": {}, "dispersion": {}, "source": {}}
    trans = {}
    per_state = {}
    pooled = {}
    for cloud, s in series.items():
        u, tot, ts = (np.asarray(s[k], np.int64) for k in ("users", "total", "ts"))
        dt = np.diff(ts)
        inc = np.diff(tot)
        for a, b in zip(u[:-1], u[1:]):
            trans[(int(a), int(b))] = trans.get((int(a), int(b)), 0) + 1
        rates = {}
        for st in np.unique(u[1:]):
            m = u[1:] == st
            rates[int(st)] = float(inc[m].sum() / dt[m].sum())
            pooled.setdefault(int(st), [0.0, 0.0])
            pooled[int(st)][0] += float(inc[m].sum())
            pooled[int(st)][1] += float(dt[m].sum())
        per_state[cloud] = rates
        top = int(u.max())
        plateau = (u[1:] == top) & (dt == 1)
        c = inc[plateau].astype(np.float64)
        out["dispersion"][cloud] = {"mean": float(c.mean()), "var": float(c.var()), "index": float(c.var() / c.mean()),
                                    "seconds": int(plateau.sum())}
        out["source"][cloud] = f"data/local_{cloud}_load_stats_history.csv ({len(u)} rows)"
    states = sorted({a for a, _ in trans} | {b for _, b in trans})
    P = np.zeros((len(states), len(states)))
    for (a, b), n in trans.items():
        P[states.index(a), states.index(b)] += n
    P /= np.maximum(P.sum(1, keepdims=True), 1)
    out["states"] = states
    out["transitions"] = P.tolist()
    out["rate"] = {c: {str(k): v for k, v in r.items()} for c, r in per_state.items()}
    out["rate"]["pooled"] = {str(k): v[0] / v[1] for k, v in pooled.items()}
    out["rate"]["pooled"].setdefault(str(states[0]), 0.0)
    for c in out["rate"]:
        out["rate"][c].setdefault(str(states[0]), 0.0)
    out["initial_state"] = states[0]
    return out


def load_reference():
    import pandas as pd

    series = {}
    for cloud in ("aws", "azure"):
        df = pd.read_csv(REF / f"local_{cloud}_load_stats_history.csv")
        series[cloud] = {"users": df["User Count"].to_numpy(np.int64), "total": df["Total Request Count"].to_numpy(np.int64),
                         "ts": df["Timestamp"].to_numpy(np.int64)}
    return series


def main():
    series = load_reference()
    model = fit(series)
    (ROOT / "rl-k8s-scheduler_amd/rlks/data/locust_mmpp.json").write_text(json.dumps(model, indent=1) + "\n")
    np.savez(ROOT / "tests/golden/locust_history.npz",
             **{f"{c}_{k}": v for c, s in series.items() for k, v in s.items()})
    print(json.dumps(model["rate"]["pooled"]), model["dispersion"])


if __name__ == "__main__":
    main()
