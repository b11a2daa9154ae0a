"""CPU tests of the table builder (generate_real_pricing.py + normalize_data.py restated) and the
evaluation harness's host-side reporting (final_evaluation.py:54-82, train_and_compare.py:75-79)."""
import numpy as np
import pytest


def test_build_reference_table_reproduces_committed_csv():
    from rlks.tables import build_reference_table, load_table

    ref = load_table()                     # pandas-parsed bits of the reference's committed CSV
    b = build_reference_table()
    assert b.columns == ref.columns
    assert b.n_rows == ref.n_rows == 100
    # the committed CSV went through its writer's platform and a CSV round trip: < 5e-14 absolute
    assert np.abs(b.cost - ref.cost).max() < 5e-14
    assert np.abs(b.latency - ref.latency).max() < 5e-14
    assert np.abs(b.raw[:, 0] - ref.raw[:, 0]).max() < 5e-14  # step column 0..1
    assert np.isnan(b.raw[1:, 5:]).all() and np.isnan(ref.raw[1:, 5:]).all()


def test_minmax_scale_is_sklearn_bit_exact():
    sk = pytest.importorskip("sklearn.preprocessing")
    from rlks.tables import minmax_scale

    rng = np.random.default_rng(0)
    x = np.column_stack([rng.normal(size=300) * 17 + 3, rng.uniform(-1e-3, 1e-3, 300), np.full(300, 2.5)])
    assert np.array_equal(minmax_scale(x), sk.MinMaxScaler().fit_transform(x))
    y = x.copy()
    y[5:, 2] = np.nan                           # normalize_data.py's cpu columns: one value + NaN
    got, want = minmax_scale(y), sk.MinMaxScaler().fit_transform(y)
    assert np.array_equal(np.isnan(got), np.isnan(want)) and np.array_equal(got[~np.isnan(got)], want[~np.isnan(want)])


def test_synthetic_two_cloud_table_is_the_reference_builder():
    from rlks.tables import build_reference_table, synthetic_table

    s, b = synthetic_table(2, 100, seed=42), build_reference_table(100, 42)
    assert np.array_equal(s.cost, b.cost) and np.array_equal(s.latency, b.latency)
    t = synthetic_table(8, 64, seed=3)
    assert t.cost.shape == (64, 8) and t.cost.min() == 0.0 and abs(t.cost.max() - 1.0) <= 1e-15


def test_eval_result_reporting():
    from rlks.evaluation import BASELINE_COST, EvalResult, comparison_lines

    rewards = np.array([4765.0, 4700.5, 4800.25, 4750.0])
    actions = np.zeros((99, 4), np.int32)
    actions[::3] = 1
    r = EvalResult(rewards, actions)
    assert r.avg_cost == float(np.mean([-x for x in rewards]))
    ch = r.choices
    assert ch == {"AWS": int((actions == 0).sum()), "Azure": int((actions == 1).sum())}
    assert r.improvement == 100 * (BASELINE_COST - r.avg_cost) / BASELINE_COST
    txt = r.report()
    assert "FINAL EVALUATION RESULTS (4 episodes)" in txt
    assert f"Average cost per episode       : ${r.avg_cost:.4f}" in txt
    assert f"Agent chose AWS                : {ch['AWS']:4d} times" in txt
    assert r.summary_text().startswith(f"Avg cost: ${r.avg_cost:.4f} | Improvement:")
    assert r.progress_lines(2) == [f"Episode   2 → cost = ${-4700.5:6.3f}", f"Episode   4 → cost = ${-4750.0:6.3f}"]
    assert comparison_lines([1.0, 2.0], [3.0, 4.0]) == ["Iteration 1: RL = 1.00 | Baseline = 3.00",
                                                       "Iteration 2: RL = 2.00 | Baseline = 4.00"]
