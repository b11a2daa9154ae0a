"""CPU checks of the oracle's learner-side restatements (test infrastructure for the GPU parity
tests): the per-epoch Feistel minibatch order, its lane-group (world-size) invariance, the
Categorical sampler restatement and a tiny whole PPO iteration."""
import numpy as np
import pytest

import oracle


@pytest.mark.parametrize("S", [1, 5, 4096, 4000, 128 * 4096, 3 * 1000 + 7])
def test_epoch_permutation_is_a_bijection(S):
    for epoch in (0, 3):
        p = oracle.epoch_permutation(1234567, epoch, S)
        assert np.array_equal(np.sort(p), np.arange(S))
    if S > 16:
        assert not np.array_equal(oracle.epoch_permutation(1, 0, S), oracle.epoch_permutation(1, 1, S))


def test_lane_groups_make_minibatches_world_size_invariant():
    """a single rank with W lane groups draws the union of what W ranks (one group each) draw"""
    T, N, mb, W = 16, 512, 2048, 4
    single = oracle.minibatch_indices(9, 2, T, N * W, mb * W, groups=W)
    for r in range(W):
        part = oracle.minibatch_indices(9, 2, T, N, mb, groups=1, group0=r)
        t, n = np.divmod(part, N)
        ts, ns = np.divmod(single[:, r * mb:(r + 1) * mb], N * W)
        assert np.array_equal(t, ts) and np.array_equal(n + r * N, ns)
    # every minibatch row is a distinct sample
    assert np.unique(single).size == single.size


def test_sampler_restatement_follows_softmax():
    rng = np.random.default_rng(0)
    n = 200000
    lg = rng.standard_normal((n, 4)).astype(np.float32)
    act, margin = oracle.sample_actions(lg, np.arange(n), np.ones(n), np.zeros(n), 42)
    p = np.exp(lg - lg.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    for a in range(4):
        z = ((act == a).sum() - p[:, a].sum()) / np.sqrt((p[:, a] * (1 - p[:, a])).sum())
        assert abs(z) < 5
    assert (margin < 4).mean() < 1e-4


def test_tiny_ppo_iteration_lowers_the_loss():
    """the oracle iteration on a tiny net: the surrogate + value loss after the update is below the
    loss before it on the same batch"""
    rng = np.random.default_rng(1)
    D, H, A, T, N = 6, 8, 2, 8, 64
    shapes = [(H, D), (H,), (H, H), (H,), (A, H), (A,), (H, D), (H,), (H, H), (H,), (1, H), (1,)]
    off, o = [], 0
    for s in shapes:
        off.append(o)
        o += int(np.prod(s))
    flat = rng.standard_normal(o) * 0.3
    obs = rng.random((T + 1, N, D)).astype(np.float32)
    lg, v = oracle.mlp_forward(flat, off, D, H, A, obs.reshape(-1, D))
    lg = lg.reshape(T + 1, N, A)[:T].astype(np.float32)
    act = rng.integers(0, A, (T, N)).astype(np.int32)
    lsm = lg - np.log(np.exp(lg).sum(-1, keepdims=True))
    buf = {"obs": obs, "logits": lg, "values": v.reshape(T + 1, N).astype(np.float32), "actions": act,
           "logp": np.take_along_axis(lsm, act[..., None], -1)[..., 0], "rewards": rng.random((T, N)).astype(np.float32),
           "dones": np.zeros((T, N), np.uint8)}
    p, m, vv, klc, st = oracle.ppo_iteration(flat, off, D, H, A, buf, perm_seed=3, epochs=4, mb=128, lr=1e-2)
    assert len(st) == 4 * (T * N // 128)
    first = (st[0]["policy_loss"] + st[0]["vf_loss"]) / st[0]["rows"]
    last = (st[-1]["policy_loss"] + st[-1]["vf_loss"]) / st[-1]["rows"]
    assert last < first and np.all(np.isfinite(p)) and klc in (0.1, 0.2, 0.3)
