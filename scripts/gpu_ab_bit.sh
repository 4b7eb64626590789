#!/bin/bash
# scripts/gpu_ab.sh preceded by a bit-for-bit comparison of the fused step's outputs between
# ab/libsrbd_mpc_old.so and the product library (scripts/bitcmp.py) -> gpurun_out/bitcmp.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SRBD_LIB=ab/libsrbd_mpc_old.so timeout -k 10 200 python scripts/bitcmp.py dump /tmp/old.npz 2>/dev/null && \
timeout -k 10 200 python scripts/bitcmp.py dump /tmp/new.npz 2>/dev/null && \
python scripts/bitcmp.py cmp /tmp/old.npz /tmp/new.npz > gpurun_out/bitcmp.txt 2>&1 || exit 1
tail -3 gpurun_out/bitcmp.txt
bash scripts/gpu_ab.sh
