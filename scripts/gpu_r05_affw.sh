#!/bin/bash
# The W-triggered affine refinement (SRBD_AFFINE_REFINE_W) in the product build: the GPU suite, the
# randomised parity campaign on the same NC cases as before, and the fused / CCS kernels A/B'd against
# the build before the change (ab/libsrbd_mpc_5db84f.so; scripts/ab_bench.sh, "old" = that build).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
NC=${NC:-1200}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu3.txt 2>&1 || { tail -40 $O/pytest_gpu3.txt; exit 1; }
tail -1 $O/pytest_gpu3.txt
FUZZ_CASES=$NC timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_affw.json > $O/fuzz_affw.log 2>&1; echo "fuzz rc=$?"; tail -1 $O/fuzz_affw.log | cut -c1-600
{ echo "# N=10 (old = 5db84f661ca2f4db, before the W trigger)"; AB_OLD=ab/libsrbd_mpc_5db84f.so bash scripts/ab_bench.sh 3 --sustain-seconds 0 --no-config3 --no-controller &&
  echo "# N=20" && AB_OLD=ab/libsrbd_mpc_5db84f.so bash scripts/ab_bench.sh 3 --sustain-seconds 0 --no-config3 --no-controller --horizon 20; } 2>&1 | grep -v amdgpu.ids > $O/ab_affw.txt
cat $O/ab_affw.txt
