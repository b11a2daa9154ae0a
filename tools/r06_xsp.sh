#!/bin/bash
# round 6: F1a hands its Xa split to F2 (SfArgs::xsp): GPU suite + smoke, then same-box c4 / c3 bench
# lines against the previous commit's library (librlks_xp_head.so)
O=gpurun_out/r06_xsp; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/r06_libab.sh xsp c4 head && bash tools/r06_libab.sh xsp c3 head
