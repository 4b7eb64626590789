#!/bin/bash
# A/B of the fused step on ONE GPU box: the product library vs ab/libsrbd_mpc_old.so (or $AB_OLD; built here
# from an earlier tree), alternating old/new ROUNDS times so box drift hits both equally.
#   scripts/ab_bench.sh [ROUNDS] [extra bench.py args...]     (run through gpurun)
# Prints the fused kernel's and the CCS solver kernel's HIP-event time per launch of each run.
set -o pipefail
cd "$(dirname "$0")/.."
ROUNDS=${1:-2}
shift
export TMPDIR=/tmp
for r in $(seq "$ROUNDS"); do
  for v in old new; do
    if [ "$v" = old ]; then lib=${AB_OLD:-ab/libsrbd_mpc_old.so}; else lib=; fi
    out=$(SRBD_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-dropin "$@") || exit 1
    echo "$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["kernels_ms"]["mpc_step_fused"], d["kernels_ms"]["pdipm"], d["value"], (d.get("parity") or {}).get("max_rel_du"))')"
  done
done
