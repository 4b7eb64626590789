#!/bin/bash
# Fused-step HIP-event time of several libraries, alternating ROUNDS times on one box:
#   gpurun -- bash scripts/gpu_multi_ab.sh ROUNDS "bench args" name=lib ...   (lib empty: product)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$1; A=$2; shift 2
for r in $(seq "$R"); do
  for v in "$@"; do
    n=${v%%=*}; l=${v#*=}
    ms=$(SRBD_LIB=$l timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-controller $A 2>/dev/null | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["kernels_ms"]["mpc_step_fused"])') || exit 1
    echo "$n $ms"
  done
done
