mkdir -p gpurun_out/red_tree
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/red_tree/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/red_tree/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/red_tree/pytest_gpu.log
bash tools/xp_f1a.sh red_xp4 c4 base t16 t64 base
