set -e
O=gpurun_out/ab_envgae; mkdir -p $O
for L in librlks.so librlks_g64.so librlks_gser.so librlks_envnt.so; do
  RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/$L timeout -k 10 120 python3 -u tools/step_gae_time.py >> $O/ab.txt 2>&1
done
cat $O/ab.txt | grep '{'
