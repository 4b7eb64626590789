#!/bin/bash
# Phase marginals of the fused N=10 step: each ab/lib_<variant>.so (scripts/ablate.py) runs one
# phase twice per Newton iteration; (variant - base) of the HIP-event time and of the SQ counters
# per wave is that phase's cost.  gpurun -- bash scripts/gpu_phase_marginals.sh VARIANT...
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
t() { SRBD_LIB=$1 timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-controller 2>/dev/null | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["kernels_ms"]["mpc_step_fused"])'; }
{
for r in 1 2; do
  echo "base $(t '')"
  for v in "$@"; do echo "$v $(t ab/lib_$v.so)"; done
done
} > gpurun_out/marg_time.txt || exit 1
cat gpurun_out/marg_time.txt
args="base="
for v in "$@"; do args="$args $v=ab/lib_$v.so"; done
bash scripts/gpu_sq_ab.sh $args > gpurun_out/marg_sq.txt 2>&1 || { tail gpurun_out/marg_sq.txt; exit 1; }
grep -E "^==|VALU  |INSTS_LDS|BANK|WAVE_CYCLES|INSTS_VALU " gpurun_out/marg_sq.txt
