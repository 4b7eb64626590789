#!/bin/bash
# A/B of library variants on ONE GPU box, alternating ROUNDS times (fused step kernel time per launch):
#   scripts/ab_variants.sh ROUNDS "libA libB ..." [bench.py args...]     (run through gpurun)
set -o pipefail
cd "$(dirname "$0")/.."
ROUNDS=$1; LIBS=$2; shift 2
export TMPDIR=/tmp
for r in $(seq "$ROUNDS"); do
  for lib in $LIBS; do
    [ "$lib" = product ] && l= || l=$lib
    out=$(SRBD_LIB=$l timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-dropin --no-controller --no-config3 "$@") || exit 1
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["kernels_ms"]["mpc_step_fused"], d["kernels_ms"]["pdipm"], d["value"])')"
  done
done
