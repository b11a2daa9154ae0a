#!/bin/bash
# round 6: whole GPU suite + smoke on the current tree, the multi-GPU readiness runs, fused-vs-split F1 A/B
O=gpurun_out/r06b2; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/r06_launcher.sh || exit 1
bash tools/ab_f1time.sh
