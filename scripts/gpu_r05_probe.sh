#!/bin/bash
# Round-5 diagnostics on one GPU box: SIMD placement of two-wave workgroups (scripts/simd_placement_probe.hip)
# and the N = 20 phase profile (ab/libsrbd_mpc_prof20.so: scripts/build_variant.py --no-regn
# --reg20=-include --reg20=scripts/phase_prof.hpp).  -> gpurun_out/r05/{simd_probe.txt,phases_N20.txt}
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
if [ -x scripts/simd_probe_bin ]; then
  timeout -k 10 60 scripts/simd_probe_bin 4096 2000 > $O/simd_probe.txt 2>&1 || { cat $O/simd_probe.txt; exit 1; }
  cat $O/simd_probe.txt
fi
for lib in ${PHASE_LIBS:-ab/libsrbd_mpc_prof20.so}; do
  [ -f "$lib" ] || continue
  echo "# $lib" >> $O/phases_N20.txt
  PHASE_LIB=$lib timeout -k 10 120 python scripts/phase_profile.py 20 4096 10 >> $O/phases_N20.txt 2>&1 || { tail -20 $O/phases_N20.txt; exit 1; }
done
cat $O/phases_N20.txt
