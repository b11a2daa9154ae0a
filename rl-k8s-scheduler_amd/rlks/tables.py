"""Price / latency tables consumed by the env kernel.

Reference: k8s_multi_cloud_env.py:22-27 resolves DATA_PATH = <project root>/data/processed/
normalized_rl_data.csv with a CWD-relative fallback, then `pd.read_csv(DATA_PATH)` (:58) and
`max_steps = len(df) - 1` (:66).  Missing file -> FileNotFoundError with a fix-it hint (:56-64).

Here the table is resolved in this order:
  1. an explicit `path` argument (CSV read with pandas' default parser, exactly as the reference);
  2. the RLKS_DATA_PATH environment variable;
  3. `data/processed/normalized_rl_data.csv` relative to the current directory (the reference's
     fallback, so running from a checkout of the reference project picks up its CSV);
  4. the packaged copy `rlks/data/normalized_rl_data.npz`: the float64 bits pandas parsed from the
     reference CSV (pandas' default parser is not correctly rounded, SURVEY.md §7.3, so the bits
     are shipped rather than re-parsed).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path

import numpy as np

PACKAGED = Path(__file__).resolve().parent / "data" / "normalized_rl_data.npz"
DEFAULT_CSV = Path("data/processed/normalized_rl_data.csv")
CLOUDS = ("aws", "azure")


@dataclass
class Table:
    cost: np.ndarray      # [T][C] float64
    latency: np.ndarray   # [T][C] float64
    columns: list
    raw: np.ndarray       # [T][ncols] float64, the whole parsed table
    source: str

    @property
    def n_rows(self) -> int:
        return int(self.cost.shape[0])

    @property
    def n_clouds(self) -> int:
        return int(self.cost.shape[1])

    def dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.raw, columns=self.columns)

    def save(self, path) -> None:
        """npz of the exact float64 bits (checkpoints); load with Table.load (no pickle)"""
        np.savez(path, cost=self.cost, latency=self.latency, raw=self.raw,
                 columns=np.array([str(c) for c in self.columns]), source=np.array(self.source))

    @classmethod
    def load(cls, path) -> "Table":
        z = np.load(path, allow_pickle=False)
        return cls(np.ascontiguousarray(z["cost"]), np.ascontiguousarray(z["latency"]),
                   [str(c) for c in z["columns"]], z["raw"], str(z["source"]))


def _from_columns(raw: np.ndarray, columns: list, source: str, clouds=CLOUDS) -> Table:
    idx = {c: i for i, c in enumerate(columns)}
    cost = np.stack([raw[:, idx[f"cost_{c}"]] for c in clouds], axis=1).astype(np.float64)
    lat = np.stack([raw[:, idx[f"latency_{c}"]] for c in clouds], axis=1).astype(np.float64)
    return Table(np.ascontiguousarray(cost), np.ascontiguousarray(lat), list(columns), raw, source)


def read_csv(path) -> Table:
    import pandas as pd

    df = pd.read_csv(path)
    return _from_columns(df.to_numpy(dtype=np.float64), list(df.columns), str(path))


def load_table(path=None) -> Table:
    if path is not None:
        p = Path(path)
        if not p.exists():
            raise FileNotFoundError(
                f"Cannot find normalized data at:\n  {p}\n"
                "Run `python normalize_data.py` from the project root first!")
        return read_csv(p)
    env = os.environ.get("RLKS_DATA_PATH")
    if env:
        return load_table(env)
    if DEFAULT_CSV.exists():
        return read_csv(DEFAULT_CSV)
    z = np.load(PACKAGED, allow_pickle=False)
    return _from_columns(z["table"], [str(c) for c in z["columns"]], str(PACKAGED))


def minmax_scale(x: np.ndarray) -> np.ndarray:
    """sklearn MinMaxScaler().fit_transform per column (normalize_data.py:25-26), in its own
    arithmetic: scale = 1 / range (a zero range counts as 1), min = -data_min * scale,
    x * scale + min; NaNs are ignored by the fit and kept"""
    x = np.asarray(x, dtype=np.float64)
    lo, hi = np.nanmin(x, axis=0), np.nanmax(x, axis=0)
    rng = hi - lo
    scale = 1.0 / np.where(rng == 0.0, 1.0, rng)
    return x * scale + (0.0 - lo * scale)


def build_reference_table(steps: int = 100, seed: int = 42, cpu_aws=None, cpu_azure=None) -> Table:
    """generate_real_pricing.py:3-18 + normalize_data.py:5-29 restated.

    np.random.seed(seed); cost_aws = 0.0104 + U(-0.001, 0.001), cost_azure = 0.0208 + U(...),
    latency_aws = 70 + U(-10, 10), latency_azure = 60 + U(-10, 10) (draws in that order); the cpu
    columns hold one value in row 0 (the mean Locust 'Average Response Time', :14-15, None = NaN)
    and NaN below; every column min-max scaled.  The result differs from the committed CSV by
    < 5e-14 (its writer's platform and pandas' CSV round trip), so the committed bits stay the
    env's source of truth (load_table); this builder feeds tables of other lengths and seeds."""
    rs = np.random.RandomState(seed)
    cols = {"step": np.arange(steps, dtype=np.float64)}
    cols["cost_aws"] = 0.0104 + rs.uniform(-0.001, 0.001, steps)
    cols["cost_azure"] = 0.0208 + rs.uniform(-0.001, 0.001, steps)
    cols["latency_aws"] = 70 + rs.uniform(-10, 10, steps)
    cols["latency_azure"] = 60 + rs.uniform(-10, 10, steps)
    for name, v in (("cpu_aws", cpu_aws), ("cpu_azure", cpu_azure)):
        c = np.full(steps, np.nan)
        c[0] = np.nan if v is None else float(v)
        cols[name] = c
    names = list(cols)
    raw = np.stack([cols[n] for n in names], axis=1)
    with np.errstate(invalid="ignore"):
        norm = np.column_stack([minmax_scale(raw[:, j]) if not np.all(np.isnan(raw[:, j])) else raw[:, j]
                                for j in range(raw.shape[1])])
    return _from_columns(norm, names, f"build_reference_table(steps={steps}, seed={seed})")


def synthetic_table(n_clouds: int, n_rows: int = 100, seed: int = 42) -> Table:
    """C-cloud table in the style of generate_real_pricing.py:3-18 + normalize_data.py:18-29.

    Per cloud c: cost = base_c + U(-0.001, 0.001) with base_c ~ U(0.009, 0.022), latency =
    lat_c + U(-10, 10) with lat_c ~ U(50, 80); every column then min-max scaled to [0, 1]
    (minmax_scale: sklearn MinMaxScaler arithmetic).  At C = 2 the bases are the reference's
    (0.0104 / 0.0208 and 70 / 60) and the cost / latency columns equal build_reference_table's.
    """
    rng = np.random.RandomState(seed)
    if n_clouds == 2:
        cbase, lbase = np.array([0.0104, 0.0208]), np.array([70.0, 60.0])
    else:
        cbase = rng.uniform(0.009, 0.022, n_clouds)
        lbase = rng.uniform(50.0, 80.0, n_clouds)
    cost = np.stack([cbase[c] + rng.uniform(-0.001, 0.001, n_rows) for c in range(n_clouds)], axis=1)
    lat = np.stack([lbase[c] + rng.uniform(-10, 10, n_rows) for c in range(n_clouds)], axis=1)
    cost, lat = minmax_scale(cost), minmax_scale(lat)
    names = [f"c{c}" for c in range(n_clouds)]
    cols = ["step"] + [f"cost_{n}" for n in names] + [f"latency_{n}" for n in names]
    raw = np.concatenate([minmax_scale(np.arange(n_rows, dtype=np.float64)[:, None]), cost, lat], axis=1)
    return Table(np.ascontiguousarray(cost), np.ascontiguousarray(lat), cols, raw, f"synthetic(C={n_clouds})")
