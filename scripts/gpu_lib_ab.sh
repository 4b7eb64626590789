# Interleaved A/B of library variants (SRBD_LIB) against the product library: fused-step kernel time
# at N = 10 and N = 20 (3 rounds), then SQ counters at N = 10 per variant.
#   bash scripts/gpu_lib_ab.sh NAME=LIB [NAME=LIB ...]   -> gpurun_out/libab_time.txt, libab_sq.txt
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
t() { SRBD_LIB=$1 timeout -k 10 120 python bench.py --horizon $2 --steps 50 --warmup 5 --no-cpu-baseline --no-controller 2>/dev/null | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["kernels_ms"]["mpc_step_fused"])'; }
{
for r in 1 2 3; do
  for H in 10 20; do
    echo "N=$H base $(t '' $H)"
    for v in "$@"; do echo "N=$H ${v%%=*} $(t ${v#*=} $H)"; done
  done
done
} > gpurun_out/libab_time.txt || exit 1
bash scripts/gpu_sq_ab.sh base= "$@" > gpurun_out/libab_sq.txt 2>&1
