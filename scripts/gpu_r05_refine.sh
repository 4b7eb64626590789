#!/bin/bash
# Round-5 refinement modes: the GPU suite, the default bench line, the fused step in both modes, and
# the randomised parity campaign (NC cases) in both modes.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
NC=${NC:-1200}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu4.txt 2>&1 || { tail -40 $O/pytest_gpu4.txt; exit 1; }
tail -1 $O/pytest_gpu4.txt
timeout -k 10 400 python3 bench.py > $O/bench_refine.json 2> $O/bench_refine.err || { tail -20 $O/bench_refine.err; exit 1; }
timeout -k 10 200 python3 scripts/refine_mode_timing.py > $O/refine_mode_timing.txt 2>&1 || { tail -20 $O/refine_mode_timing.txt; exit 1; }
grep -v amdgpu $O/refine_mode_timing.txt
for m in adaptive every_iteration; do
  FUZZ_REFINE=$m FUZZ_CASES=$NC timeout -k 10 400 python -u scripts/parity_fuzz.py 0 $O/fuzz_final_$m.json > $O/fuzz_final_$m.log 2>&1; echo "fuzz $m rc=$?"
  tail -1 $O/fuzz_final_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('cases','envs','n_failed','floor_explained_envs','max_u0_rel','build_id','refinement')})"
done
exit 0
