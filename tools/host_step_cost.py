"""Host (CPU) cost of the multi-rank SGD step (RLKS_DDP_FORCE=1: a one-rank RCCL group takes the
multi-rank path): cProfile of PPO.update() at a size whose GPU work per step is small, so the host
calls bound the step; overlapped two-bucket all-reduce vs one bucket vs the one-rank fused step."""
import cProfile
import io
import os
import pstats
import socket
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))


def main():
    import torch
    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), RANK="0", WORLD_SIZE="1")
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from rlks.ppo import PPO, PPOConfig

    for mode in ("overlap", "onebucket", "one_rank"):
        os.environ["RLKS_DDP_FORCE"] = "0" if mode == "one_rank" else "1"
        cfg = (PPOConfig().environment("K8sMultiCloudEnv").framework("torch")
               .training(train_batch_size=1024 * 64, sgd_minibatch_size=4096, num_sgd_iter=10, lr=3e-4)
               .debugging(seed=3))
        cfg.num_envs, cfg.rollout_fragment_length = 1024, 64
        cfg.overlap_allreduce = mode == "overlap"
        algo = PPO(config=cfg, device=torch.device("cuda", 0))
        algo.train()
        torch.cuda.synchronize()
        algo.rollout()
        algo.advantages()
        torch.cuda.synchronize()
        steps = algo.config.num_sgd_iter * algo.n_mb
        t0 = time.perf_counter()
        pr = cProfile.Profile()
        pr.enable()
        algo.update()
        pr.disable()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"== {mode}: multi={algo.multi} overlap={algo._overlap}: {steps} SGD steps, host {1e6 * (t1 - t0) / steps:.1f} "
              f"us/step (GPU done {1e6 * (t2 - t0) / steps:.1f} us/step)", flush=True)
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(8)
        print("\n".join(out.getvalue().splitlines()[6:20]), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
