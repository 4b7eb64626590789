#!/bin/bash
# Threshold sweep of the W-triggered affine refinement: fused / CCS kernel times of the product
# (tau = 1e3) against the builds before the trigger (5db84f), with the vote but no W trigger (w1e300:
# the vote's own cost) and tau = 1e4 (w1e4), alternating (scripts/ab_bench.sh); then the randomised
# parity campaign (same NC cases) on w1e4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
for v in 5db84f w1e300 w1e4; do
  { echo "# $v N=10"; AB_OLD=ab/libsrbd_mpc_$v.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller &&
    echo "# $v N=20" && AB_OLD=ab/libsrbd_mpc_$v.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller --horizon 20; } 2>&1 | grep -v amdgpu.ids
done > $O/ab_wsweep.txt
cat $O/ab_wsweep.txt
SRBD_LIB=ab/libsrbd_mpc_w1e4.so FUZZ_CASES=${NC:-1200} timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_w1e4.json > $O/fuzz_w1e4.log 2>&1; echo "fuzz rc=$?"; tail -1 $O/fuzz_w1e4.log | cut -c1-300
exit 0
