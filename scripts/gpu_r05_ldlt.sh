#!/bin/bash
# Stable foot-block solves (LDL^T of Phi_f in the register kernels' solves): the GPU suite, the fused step
# A/B'd against the build before (ab/libsrbd_mpc_132823.so, "old"), the 1200-case campaign in both
# refinement modes and the _ccs campaign (FUZZ_CCS=1, 240 s per mode).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu5.txt 2>&1 || { tail -40 $O/pytest_gpu5.txt; exit 1; }
tail -1 $O/pytest_gpu5.txt
{ echo "# N=10 (old = 132823b55c25a77d)"; AB_OLD=ab/libsrbd_mpc_132823.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller &&
  echo "# N=20" && AB_OLD=ab/libsrbd_mpc_132823.so bash scripts/ab_bench.sh 2 --sustain-seconds 0 --no-config3 --no-controller --horizon 20; } 2>&1 | grep -v amdgpu.ids > $O/ab_ldlt.txt
cat $O/ab_ldlt.txt
for m in adaptive every_iteration; do
  FUZZ_REFINE=$m FUZZ_CASES=1200 timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_ldlt_$m.json > $O/fuzz_ldlt_$m.log 2>&1; echo "fuzz $m rc=$?"
  tail -1 $O/fuzz_ldlt_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('cases','n_failed','floor_explained_envs','max_u0_rel','build_id','refinement')})"
  FUZZ_CCS=1 FUZZ_REFINE=$m timeout -k 10 330 python -u scripts/parity_fuzz.py 240 $O/fuzz_ldlt_big_$m.json > $O/fuzz_ldlt_big_$m.log 2>&1; echo "fuzz big $m rc=$?"
  tail -1 $O/fuzz_ldlt_big_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('cases','n_failed','floor_explained_envs','max_u0_rel','build_id','refinement')})"
done
exit 0
