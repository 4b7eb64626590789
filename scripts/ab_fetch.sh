#!/bin/bash
# HBM read traffic (rocprofv3 FETCH_SIZE, one --pmc pass each) of the fused step, product library
# vs ab/libsrbd_mpc_old.so; summaries under gpurun_out/ab_fetch_{old,new}/ (run through gpurun).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in old new; do
  if [ "$v" = old ]; then export SRBD_LIB=ab/libsrbd_mpc_old.so; else unset SRBD_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ab_fetch_$v -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-reps 2 > /dev/null 2> gpurun_out/ab_fetch_$v.err || exit 1
  python3 - "$v" <<'PY'
import csv, glob, sys
acc = {}
for f in glob.glob(f"gpurun_out/ab_fetch_{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        acc.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
for k, v in acc.items():
    if "mpc_step" in k:
        print(sys.argv[1], k[:40], f"FETCH {2 * 1024 * sum(v) / len(v) / 1e6:.2f} MB/launch (x2 gfx950 corrected)")
PY
done
