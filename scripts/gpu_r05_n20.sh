#!/bin/bash
# Round-5 N = 20 experiment on one GPU box: phase profiles (wave 0 and wave 1, chain waits) of the
# instrumented variants, and SQ counters of the fused N = 20 step for the product library and a
# variant (ab/libsrbd_mpc_nopipe.so by default).  -> gpurun_out/r05/n20/
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05/n20
mkdir -p $O
for lib in ${PHASE_LIBS:-ab/libsrbd_mpc_prof20.so ab/libsrbd_mpc_prof20_nopipe.so}; do
  [ -f "$lib" ] || continue
  echo "# $lib" >> $O/phases.txt
  PHASE_LIB=$lib timeout -k 10 120 python scripts/phase_profile.py 20 4096 10 2>&1 | grep -v amdgpu.ids >> $O/phases.txt || { tail -20 $O/phases.txt; exit 1; }
done
cat $O/phases.txt
B20="python3 bench.py --horizon 20 --steps 3 --warmup 1 --no-cpu-baseline --no-controller --no-dropin --no-config3 --kernel-reps 2"
for v in new ${SQ_VARIANT:-nopipe}; do
  if [ "$v" = new ]; then export SRBD_LIB=; else export SRBD_LIB=ab/libsrbd_mpc_$v.so; fi
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $O/sq_$v -o run --output-format csv -- $B20 > $O/sq_$v.json 2> $O/sq_$v.err || { tail -20 $O/sq_$v.err; exit 1; }
done
ls -R $O | head -40
