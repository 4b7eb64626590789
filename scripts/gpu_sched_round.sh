set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k full_size > gpurun_out/pytest_full_size.log 2>&1 && \
timeout -k 10 600 python -u scripts/variant_bench.py --rounds 3 base= imin="-mllvm -amdgpu-sched-strategy=iterative-minreg" trk="-mllvm -amdgpu-use-amdgpu-trackers=1" > gpurun_out/sched_N10.txt 2>&1 && \
timeout -k 10 600 python -u scripts/variant_bench.py --rounds 3 --horizon 20 base= imin="-mllvm -amdgpu-sched-strategy=iterative-minreg" trk="-mllvm -amdgpu-use-amdgpu-trackers=1" > gpurun_out/sched_N20.txt 2>&1 && \
timeout -k 10 600 python -u scripts/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1
