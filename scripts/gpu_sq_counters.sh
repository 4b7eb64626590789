set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-controller --no-dropin --kernel-reps 1 > gpurun_out/pmc_sq.json 2>gpurun_out/pmc_sq.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d gpurun_out/pmc_sq2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-controller --no-dropin --kernel-reps 1 > gpurun_out/pmc_sq2.json 2>gpurun_out/pmc_sq2.err && python3 scripts/sq_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq2 --json gpurun_out/sq_counters.json > gpurun_out/sq_counters.txt
