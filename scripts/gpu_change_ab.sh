# One kernel change on the GPU: the parity suite on the product library, then an interleaved A/B of
# the fused-step time and SQ counters against the previous library (gpu_lib_ab.sh), then the driver's
# bench command (20 steps, 5 warm-up).
#   bash scripts/gpu_change_ab.sh NAME=LIB [NAME=LIB ...]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
bash scripts/gpu_lib_ab.sh "$@" && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
