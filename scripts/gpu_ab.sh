#!/bin/bash
# One GPU call for a kernel change: the GPU test suite, then the A/B of the fused step against
# ab/libsrbd_mpc_old.so (scripts/ab_bench.sh) at N = 10 (3 rounds) and N = 20 (2 rounds).
#   gpurun -- bash scripts/gpu_ab.sh        -> gpurun_out/ab_pytest.log, gpurun_out/ab.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
{ echo "# N=10"; bash scripts/ab_bench.sh 3 && echo "# N=20" && bash scripts/ab_bench.sh 2 --horizon 20 --no-controller; } 2>&1 | grep -v amdgpu.ids > gpurun_out/ab.txt
cat gpurun_out/ab.txt
