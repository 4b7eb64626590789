set -o pipefail
mkdir -p gpurun_out
for B in 2048 4096 6144 8192 16384 1024 512; do
  out=$(timeout -k 10 120 python bench.py --no-cpu-baseline --batch-per-gpu $B --steps 100 --warmup 20) || exit 1
  echo "$B $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["kernels_ms"]["mpc_step_fused"], d["ms_per_step"], d["value"])')"
done
