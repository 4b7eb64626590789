# The round's GPU evidence in one call: parity suite, bench + rocprof stats + PMC traffic
# (gpu_round.sh), SQ utilisation counters (gpu_sq_counters.sh), per-config rates (bench_configs.py).
set -o pipefail
cd /root/repo
bash scripts/gpu_round.sh && bash scripts/gpu_sq_counters.sh && \
timeout -k 10 600 python -u scripts/bench_configs.py gpurun_out/configs.json > gpurun_out/configs.log 2>&1
