#!/bin/bash
# Instruction-cache behaviour of the fused step (rocprofv3 --pmc, SQC block): hits, misses, requests
# to L2 for instructions; summary per kernel into gpurun_out/icache.txt (run through gpurun).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAVES -d gpurun_out/icache -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-reps 2 "$@" > /dev/null 2> gpurun_out/icache.err || exit 1
python3 - <<'PY' > gpurun_out/icache.txt
import csv, glob
acc = {}
for f in glob.glob("gpurun_out/icache/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "mpc_step" in row["Kernel_Name"]:
            acc.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:32s} {sum(v) / len(v):14.0f} per launch")
PY
cat gpurun_out/icache.txt
