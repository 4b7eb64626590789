#!/bin/bash
# End-of-round evidence in one GPU call (boxes are scarce): the GPU suite and the fallback probe
# (scripts/gpu_r04.sh without the A/B), the general solve's phase profile (needs
# ab/libsrbd_mpc_gprof5.so from `GPROF_LIB=libsrbd_mpc_gprof5.so python scripts/general_phase_profile.py
# build`), then scripts/gpu_profile_r04.sh (smoke, bench lines, rocprofv3 stats, PMC / SQ passes,
# configs, two-rank launcher rehearsal).
set -o pipefail
cd "$(dirname "$0")/.."
PROBE_LIBS=new SKIP_AB=1 bash scripts/gpu_r04.sh || exit 1
rm -f gpurun_out/r04/general_phases_final.txt
if [ -f ab/libsrbd_mpc_gprof5.so ]; then
  for n in 10 20; do
    GPROF_LIB=libsrbd_mpc_gprof5.so timeout -k 10 200 python scripts/general_phase_profile.py run $n 96 5 \
      >> gpurun_out/r04/general_phases_final.txt 2>&1 || exit 1
  done
fi
bash scripts/gpu_profile_r04.sh
