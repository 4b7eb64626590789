#!/bin/bash
# Round-5 check on one GPU box: the GPU suite, the default bench line, and (with AB=1) the fused
# N = 10 / N = 20 steps A/B'd against ab/libsrbd_mpc_r04.so (the round-4 build), alternating runs.
#   gpurun -- bash scripts/gpu_r05.sh   -> gpurun_out/r05/{pytest_gpu.txt,bench.json,ab.txt}
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  tail -c 3000 $O/bench.json
fi
if [ -n "$AB" ]; then
  { echo "# N=10 (fused_ms pdipm_ms value max_rel_du)"; AB_OLD=${AB_LIB:-ab/libsrbd_mpc_r04.so} bash scripts/ab_bench.sh ${AB_ROUNDS:-2} --sustain-seconds 0 --no-config3 &&
    echo "# N=20" && AB_OLD=${AB_LIB:-ab/libsrbd_mpc_r04.so} bash scripts/ab_bench.sh ${AB_ROUNDS:-2} --sustain-seconds 0 --horizon 20 --no-controller; } 2>&1 | grep -v amdgpu.ids > $O/ab.txt
  cat $O/ab.txt
fi
exit 0
