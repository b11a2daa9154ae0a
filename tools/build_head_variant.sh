#!/bin/bash
# librlks_xp_head.so: the library with sgd_sf16.hip as committed (HEAD), for same-box A/B timing
set -e
cd "$(dirname "$0")/../rl-k8s-scheduler_amd/csrc"
git show HEAD:rl-k8s-scheduler_amd/csrc/sgd_sf16.hip > sgd_sf16_head.hip
mkdir -p ../build/xp_head
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -I../../include -munsafe-fp-atomics -c sgd_sf16_head.hip -o ../build/xp_head/sgd_sf16.o 2>/dev/null
rm sgd_sf16_head.hip
ls ../build/*.o | grep -v sgd_sf16 | xargs /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 ../build/xp_head/sgd_sf16.o -o ../rlks/librlks_xp_head.so
