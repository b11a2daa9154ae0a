#!/bin/bash
# round 6 multi-GPU readiness on one GPU box: the strong-scaling anchor (--scaling strong --gpus 1: the
# whole 1,048,576-lane job on one GPU), and the launcher's own two-rank start (bench.py --gpus 2 with
# no torch.distributed launcher) in both scalings, gloo (both ranks share the one GPU)
O=gpurun_out/r06_launcher; mkdir -p $O
summ() {
  python3 -c "
import json
d=[json.loads(l) for l in open('$1') if l.startswith('{')][-1]
print('$2', d['n_gpus'], d['scaling'], round(d['value']/1e6,3), 'M env-steps/s', round(d['ms_per_step'],1), 'ms/it', d['config']['envs_per_gpu'], d['config']['minibatch_per_gpu'], json.dumps(d.get('allreduce')))"
}
timeout -k 10 500 python3 -u bench.py --gpus 1 --scaling strong --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/strong_gpus1.txt 2>&1 || { tail -20 $O/strong_gpus1.txt; exit 1; }
summ $O/strong_gpus1.txt strong_n1
RLKS_DIST_BACKEND=gloo timeout -k 10 500 python3 -u bench.py --gpus 2 --scaling strong --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/strong_gpus2_gloo.txt 2>&1 || { tail -20 $O/strong_gpus2_gloo.txt; exit 1; }
summ $O/strong_gpus2_gloo.txt strong_n2_gloo
RLKS_DIST_BACKEND=gloo timeout -k 10 500 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/weak_gpus2_gloo.txt 2>&1 || { tail -20 $O/weak_gpus2_gloo.txt; exit 1; }
summ $O/weak_gpus2_gloo.txt weak_n2_gloo
