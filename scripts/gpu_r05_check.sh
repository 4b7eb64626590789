#!/bin/bash
# Round-5 check of the product build on one GPU box: the GPU suite, the default bench line, the drop-in
# memory probe and the fused N = 10 / 20 steps A/B'd against the round-4 library (ab/libsrbd_mpc_r04.so).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
AB=1 AB_ROUNDS=3 bash scripts/gpu_r05.sh || exit 1
timeout -k 10 300 python3 scripts/dropin_memory_probe.py 4096 > $O/dropin_memory.json 2> $O/dropin_memory.err || { tail -20 $O/dropin_memory.err; exit 1; }
cat $O/dropin_memory.json
