#!/bin/bash
# With stable foot-block solves: is the W-triggered predictor refinement still needed? The variant without
# the trigger (ab/libsrbd_mpc_notrig.so: -DSRBD_AFFINE_REFINE_W=1e300, predictor refined only at a clamped s)
# on the same campaign cases as the product, and its fused-step time ("old" = the variant).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
SRBD_LIB=ab/libsrbd_mpc_notrig.so FUZZ_CASES=1200 timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_notrig.json > $O/fuzz_notrig.log 2>&1; echo "fuzz rc=$?"
tail -1 $O/fuzz_notrig.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('cases','n_failed','floor_explained_envs','max_u0_rel','build_id')})"
SRBD_LIB=ab/libsrbd_mpc_notrig.so FUZZ_CCS=1 FUZZ_CASES=3349 timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_notrig_big.json > $O/fuzz_notrig_big.log 2>&1; echo "fuzz big rc=$?"
tail -1 $O/fuzz_notrig_big.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('cases','n_failed','floor_explained_envs','max_u0_rel','build_id')})"
{ echo "# N=10 (old = no-trigger variant)"; AB_OLD=ab/libsrbd_mpc_notrig.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller &&
  echo "# N=20" && AB_OLD=ab/libsrbd_mpc_notrig.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller --horizon 20; } 2>&1 | grep -v amdgpu.ids > $O/ab_notrig.txt
cat $O/ab_notrig.txt
exit 0
