#!/bin/bash
# Round-6 GPU call, one script for every step (it replaces round 5's eleven single-use gpu_r05_*.sh):
#   gpurun -- 'STEPS="tests timing fuzz" bash scripts/gpu_r06.sh'     -> gpurun_out/r06/
# STEPS (run in this order, each under its own time limit; the call stops at the first failure):
#   tests    the GPU suite (pytest -m gpu)
#   timing   fused-step time per refinement policy (scripts/refine_mode_timing.py $TIMING_POLICIES)
#   fuzz     the default-sequence parity campaign, FUZZ_CASES (1200) cases, every policy in $FUZZ_POLICIES
#   ccs      the _ccs-sequence campaign, $CCS_SECONDS (420) s, the same policies
#   bench    the default bench line and the driver-form run
#   ab       alternating bench runs against $AB_LIB (default ab/libsrbd_mpc_r05.so), N = 10 and 20
#   fixture  the fuzz-regression fixture under each policy of $FIXTURE_POLICIES (scripts/fixture_policies.py)
#   seeds    chosen campaign cases ($SEEDS_DEFAULT, $SEEDS_CCS) under each library of $SEEDS_LIBS
#   profile  rocprofv3 kernel stats of the bench command, PMC traffic and SQ passes, the configs, smoke,
#            the two-rank launcher rehearsal on one device over gloo
# The campaigns' outputs are floor-checked afterwards on the CPU host (scripts/parity_floor.py).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
POL=${FUZZ_POLICIES:-adaptive,strict}
for step in ${STEPS:-tests}; do
  case $step in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.txt 2>&1 || { tail -60 $O/pytest_gpu.txt; exit 1; }
      tail -1 $O/pytest_gpu.txt ;;
    timing)
      REFINE_ROUNDS=${TIMING_ROUNDS:-3} timeout -k 10 600 python -u scripts/refine_mode_timing.py \
        ${TIMING_POLICIES:-adaptive strict} > $O/refine_timing.jsonl 2> $O/refine_timing.err || { tail -30 $O/refine_timing.err; exit 1; }
      tail -4 $O/refine_timing.jsonl ;;
    fuzz)
      FUZZ_POLICIES=$POL FUZZ_CASES=${FUZZ_CASES:-1200} timeout -k 10 900 python -u scripts/parity_fuzz.py 0 \
        $O/fuzz_default.json.gz > $O/fuzz_default.log 2>&1 || { tail -30 $O/fuzz_default.log; exit 1; }
      tail -1 $O/fuzz_default.log | cut -c1-600 ;;
    ccs)
      FUZZ_CCS=1 FUZZ_POLICIES=$POL timeout -k 10 $(( ${CCS_SECONDS:-420} + 300 )) python -u scripts/parity_fuzz.py \
        ${CCS_SECONDS:-420} $O/fuzz_ccs.json.gz > $O/fuzz_ccs.log 2>&1 || { tail -30 $O/fuzz_ccs.log; exit 1; }
      tail -1 $O/fuzz_ccs.log | cut -c1-600 ;;
    seeds)
      # chosen cases of both sequences (SEEDS_DEFAULT / SEEDS_CCS) under each library of SEEDS_LIBS ("product"
      # = the in-tree build), both modes: parity_fuzz.py's FUZZ_SEEDS replay
      for lib in ${SEEDS_LIBS:-product}; do
        tag=$(basename ${lib%.so})
        [ "$lib" = product ] && lib=
        for seq in default ccs; do
          seeds=$SEEDS_DEFAULT; cc=0
          [ $seq = ccs ] && seeds=$SEEDS_CCS && cc=1
          [ -z "$seeds" ] && continue
          SRBD_LIB=$lib FUZZ_CCS=$cc FUZZ_SEEDS=$seeds FUZZ_POLICIES=$POL timeout -k 10 300 python -u scripts/parity_fuzz.py 0 \
            $O/seeds_${seq}_$tag.json.gz > $O/seeds_${seq}_$tag.log 2>&1 || { tail -30 $O/seeds_${seq}_$tag.log; exit 1; }
        done
      done
      ls $O/seeds_* ;;
    fixture)
      timeout -k 10 300 python -u scripts/fixture_policies.py ${FIXTURE_POLICIES:-adaptive strict} > $O/fixture_policies.jsonl 2> $O/fixture.err || { tail -30 $O/fixture.err; exit 1; }
      cut -c1-400 $O/fixture_policies.jsonl ;;
    bench)
      timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
      timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_form.json 2> $O/bench_driver_form.err || exit 1
      tail -c 1500 $O/bench.json ;;
    ab)
      { echo "# N=10 (fused_ms pdipm_ms value max_rel_du)"; AB_OLD=${AB_LIB:-ab/libsrbd_mpc_r05.so} bash scripts/ab_bench.sh ${AB_ROUNDS:-3} --sustain-seconds 0 --no-config3 &&
        echo "# N=20" && AB_OLD=${AB_LIB:-ab/libsrbd_mpc_r05.so} bash scripts/ab_bench.sh ${AB_ROUNDS:-3} --sustain-seconds 0 --horizon 20 --no-controller; } 2>&1 | grep -v amdgpu.ids > $O/ab.txt || exit 1
      cat $O/ab.txt ;;
    profile)
      B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-controller --no-dropin --no-config3 --sustain-seconds 0 --kernel-reps 2"
      B20="python3 bench.py --horizon 20 --steps 3 --warmup 1 --no-cpu-baseline --no-controller --no-dropin --no-config3 --sustain-seconds 0 --kernel-reps 2"
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-controller --no-dropin --no-config3 --sustain-seconds 0 > $O/bench_prof.json 2> $O/prof.err && \
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc1.json 2> $O/pmc1.err && \
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc2.json 2> $O/pmc2.err && \
      timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $O/pmc_sq -o run --output-format csv -- $B > $O/pmc_sq.json 2> $O/pmc_sq.err && \
      timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $O/pmc_sq20 -o run --output-format csv -- $B20 > $O/pmc_sq20.json 2> $O/pmc_sq20.err && \
      timeout -k 10 900 python3 -u scripts/bench_configs.py $O/configs.json > $O/configs.log 2>&1 && \
      SRBD_BENCH_ONE_DEVICE=1 SRBD_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > $O/bench_2rank_one_device_gloo.json 2> $O/bench_2rank.err || exit 1
      ls $O ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
