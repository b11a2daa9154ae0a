"""Agent surface: `from rl_scheduler.agent import PPO, PPOConfig` (RLlib's names, GPU engine)."""


def __getattr__(name):
    if name in ("PPO", "PPOConfig"):
        from rlks import ppo

        return getattr(ppo, name)
    raise AttributeError(name)
