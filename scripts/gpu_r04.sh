#!/bin/bash
# Round-4 check on one GPU box: the GPU suite, the fallback throughput probe, then the A/B of the
# fused step and the CCS solver kernel against ab/libsrbd_mpc_old.so (round-3 HEAD build).
#   gpurun -- bash scripts/gpu_r04.sh   -> gpurun_out/r04/{pytest_gpu.txt,fallback_probe.json,ab.txt}
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/r04/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/r04/pytest_gpu.txt
for v in ${PROBE_LIBS:-new slots old}; do
  case $v in new) lib=;; slots) lib=ab/libsrbd_mpc_slots.so;; old) lib=ab/libsrbd_mpc_old.so;; prev) lib=ab/libsrbd_mpc_prev.so;; esac
  [ -z "$lib" ] || [ -f "$lib" ] || continue
  SRBD_LIB=$lib timeout -k 10 400 python scripts/fallback_probe.py > gpurun_out/r04/fallback_probe_$v.json 2> gpurun_out/r04/fallback_probe_$v.err || { tail -20 gpurun_out/r04/fallback_probe_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/r04/fallback_probe_$v.json)"
done
[ -n "$SKIP_AB" ] && exit 0
{ echo "# N=10 (fused_ms pdipm_ms value max_rel_du)"; bash scripts/ab_bench.sh 3 && echo "# N=20" && bash scripts/ab_bench.sh 2 --horizon 20 --no-controller; } 2>&1 | grep -v amdgpu.ids > gpurun_out/r04/ab.txt
cat gpurun_out/r04/ab.txt
