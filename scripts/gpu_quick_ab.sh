# Parity suite + bench + SQ counters of the product library at HEAD (one gpurun call).
#   bash scripts/gpu_quick_ab.sh TAG   -> gpurun_out/{pytest_TAG.txt, bench_TAG.json, sq_TAG.txt}
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
T=${1:-head}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.txt 2>&1 && \
for r in 1 2 3; do timeout -k 10 120 python bench.py --no-cpu-baseline --no-controller --steps 100 --warmup 20 || exit 1; done > gpurun_out/bench_$T.json 2>/dev/null && \
for r in 1 2; do timeout -k 10 120 python bench.py --horizon 20 --no-cpu-baseline --no-controller --steps 50 --warmup 5 || exit 1; done >> gpurun_out/bench_$T.json 2>/dev/null && \
bash scripts/gpu_sq_ab.sh $T= > gpurun_out/sq_$T.log 2>&1
