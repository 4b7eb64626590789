#!/bin/bash
# Round-5 evidence in one GPU call (after scripts/gpu_r05.sh passed): smoke, the default bench line,
# the driver-form run, rocprofv3 kernel stats of the bench command, PMC traffic (FETCH_SIZE, WRITE_SIZE)
# and SQ utilisation passes, the per-config rates, and a two-rank rehearsal of the rank launcher on one
# device over gloo. Output: gpurun_out/r05p/ (summarised into profiles/r05/ on the build host).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-controller --no-dropin --no-config3 --sustain-seconds 0 --kernel-reps 2"
B20="python3 bench.py --horizon 20 --steps 3 --warmup 1 --no-cpu-baseline --no-controller --no-dropin --no-config3 --sustain-seconds 0 --kernel-reps 2"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_form.json 2> $O/bench_driver_form.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-controller --no-dropin --no-config3 --sustain-seconds 0 > $O/bench_prof.json 2> $O/prof.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc1.json 2> $O/pmc1.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc2.json 2> $O/pmc2.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $O/pmc_sq -o run --output-format csv -- $B > $O/pmc_sq.json 2> $O/pmc_sq.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $O/pmc_sq2 -o run --output-format csv -- $B > $O/pmc_sq2.json 2> $O/pmc_sq2.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $O/pmc_sq20 -o run --output-format csv -- $B20 > $O/pmc_sq20.json 2> $O/pmc_sq20.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $O/pmc_sq20b -o run --output-format csv -- $B20 > $O/pmc_sq20b.json 2> $O/pmc_sq20b.err && \
timeout -k 10 900 python3 -u scripts/bench_configs.py $O/configs.json > $O/configs.log 2>&1 && \
SRBD_BENCH_ONE_DEVICE=1 SRBD_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > $O/bench_2rank_one_device_gloo.json 2> $O/bench_2rank.err
rc=$?
ls -R $O | head -50
exit $rc
