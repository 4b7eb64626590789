#!/bin/bash
# Snapshot the committed kernels (HEAD) as the A/B baseline: ab/head_csrc (sources, for
# scripts/variant_counters.py head=@ab/head_csrc) and ab/libsrbd_mpc_old.so (for scripts/ab_bench.sh).
set -e
cd "$(dirname "$0")/.."
rm -rf ab/head_csrc /tmp/ab_snap && mkdir -p ab/head_csrc /tmp/ab_snap
git archive HEAD biped_pympc_amd/csrc include | tar -x -C /tmp/ab_snap
cp /tmp/ab_snap/biped_pympc_amd/csrc/* ab/head_csrc/
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I /tmp/ab_snap/include \
  -o ab/libsrbd_mpc_old.so /tmp/ab_snap/biped_pympc_amd/csrc/srbd_mpc.hip
echo "A/B baseline = $(git rev-parse --short HEAD)"
