#!/bin/bash
# librlks_xp_<name>.so: the working tree's sgd_sf16.hip built with extra flags, for same-box A/B
# timing (tools/ab_cfg.sh): build_xp_variant.sh <name> <hipcc flags...>
set -e
N=$1; shift
cd "$(dirname "$0")/../rl-k8s-scheduler_amd/csrc"
mkdir -p ../build/xp_$N
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -I../../include -munsafe-fp-atomics "$@" -c sgd_sf16.hip -o ../build/xp_$N/sgd_sf16.o
ls ../build/*.o | grep -v sgd_sf16 | xargs /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 ../build/xp_$N/sgd_sf16.o -o ../rlks/librlks_xp_$N.so
