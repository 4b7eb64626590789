#!/bin/bash
# Round-5 closing evidence: the GPU suite and the default bench line at this build, then the fused and CCS
# N = 10 / N = 20 kernels A/B'd (alternating runs, scripts/ab_bench.sh) against earlier builds made on the
# CPU host by scripts/build_variant.py (ab/libsrbd_mpc_<rev>.so, AB_REVS, default 1184c6e); with
# WITH_PROFILE=1 also the round's profile set (scripts/gpu_profile_r05.sh).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
bash scripts/gpu_r05.sh || exit 1
for v in ${AB_REVS:-1184c6e}; do
  SKIP_TESTS=1 SKIP_BENCH=1 AB=1 AB_ROUNDS=2 AB_LIB=ab/libsrbd_mpc_$v.so bash scripts/gpu_r05.sh || exit 1
  mv $O/ab.txt $O/ab_$v.txt
done
[ -n "$WITH_PROFILE" ] && bash scripts/gpu_profile_r05.sh
exit 0
