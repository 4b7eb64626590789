#!/bin/bash
# Affine-refinement A/B: the product build vs ab/libsrbd_mpc_affall.so (-DSRBD_REFINE_AFFINE_ALL=1: the
# register kernels refine the affine direction in every iteration, as the LDS-resident and general
# kernels do) -- the randomised parity campaign on the same FUZZ_CASES cases, then fused-step timings
# (scripts/ab_bench.sh: "old" = the variant).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
NC=${NC:-1200}
FUZZ_CASES=$NC timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_prod.json > $O/fuzz_prod.log 2>&1; echo "prod rc=$?"; tail -1 $O/fuzz_prod.log | cut -c1-600
SRBD_LIB=ab/libsrbd_mpc_affall.so FUZZ_CASES=$NC timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_affall.json > $O/fuzz_affall.log 2>&1; echo "affall rc=$?"; tail -1 $O/fuzz_affall.log | cut -c1-600
{ echo "# N=10 (old = affall variant)"; AB_OLD=ab/libsrbd_mpc_affall.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller &&
  echo "# N=20" && AB_OLD=ab/libsrbd_mpc_affall.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller --horizon 20; } 2>&1 | grep -v amdgpu.ids > $O/ab_affall.txt
cat $O/ab_affall.txt
