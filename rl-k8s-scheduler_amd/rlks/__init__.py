"""rlks — MI355X-native rollout-and-training engine for the rl_scheduler multi-cloud pod scheduler.

Public surface (mirrors the reference's gymnasium env and RLlib PPO call sites):
    K8sMultiCloudEnv, VecK8sMultiCloudEnv      rlks.env   (k8s_multi_cloud_env.py:36-157)
    PPO, PPOConfig                             rlks.ppo   (train_ppo.py:9-31, eval_ppo.py:17-27)
    evaluate, round_robin_baseline             rlks.evaluation (final_evaluation.py:39-82,
                                                               train_and_compare.py:53-79)
    build_reference_table, synthetic_table     rlks.tables (generate_real_pricing.py, normalize_data.py)
    latest_checkpoint, run_experiment          rlks.checkpoints (final_evaluation.py:13-25, train_final.py:22-35)
    JsonLinesReporter                          rlks.metrics (train_ppo.py:29-30 per-iteration report)
All compute runs in librlks.so (hand-written gfx950 HIP kernels); there is no CPU fallback.
"""
from .checkpoints import find_checkpoints, latest_checkpoint, results_root, run_experiment  # noqa: F401
from .metrics import JsonLinesReporter  # noqa: F401
from .tables import Table, build_reference_table, load_table, synthetic_table  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package must not require a GPU
    if name in ("K8sMultiCloudEnv", "VecK8sMultiCloudEnv"):
        from . import env

        return getattr(env, name)
    if name in ("PPO", "PPOConfig"):
        from . import ppo

        return getattr(ppo, name)
    if name in ("evaluate", "round_robin_baseline", "EvalResult"):
        from . import evaluation

        return getattr(evaluation, name)
    if name == "PolicyParams":
        from .policy import PolicyParams

        return PolicyParams
    raise AttributeError(name)
