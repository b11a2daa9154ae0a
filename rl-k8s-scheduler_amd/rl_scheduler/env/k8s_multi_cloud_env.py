"""Drop-in module path of the reference env (rl_scheduler/env/k8s_multi_cloud_env.py).

DATA_PATH resolution and the env class come from rlks (see rlks/tables.py, rlks/env.py).
"""
from pathlib import Path

from rlks.env import K8sMultiCloudEnv  # noqa: F401
from rlks.tables import DEFAULT_CSV as DATA_PATH  # noqa: F401

PROJECT_ROOT = Path.cwd()
