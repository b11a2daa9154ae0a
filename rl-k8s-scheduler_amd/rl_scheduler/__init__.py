"""Import-path shim: `from rl_scheduler.env.k8s_multi_cloud_env import K8sMultiCloudEnv` resolves to
the GPU-backed drop-in (rlks.env.K8sMultiCloudEnv)."""
