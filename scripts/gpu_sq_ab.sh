# SQ counters of the fused step (horizon $H, default 10) for one or more library variants (SRBD_LIB)
# -> gpurun_out/sq_<name>.*   (per-wave figures; a QP is 2 waves at N = 11..21)
#   [H=20] bash scripts/gpu_sq_ab.sh NAME=LIB [NAME=LIB ...]     (LIB empty: the product library)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
H=${H:-10}
B="python3 bench.py --horizon $H --steps 2 --warmup 1 --no-cpu-baseline --no-controller --kernel-reps 1"
for v in "$@"; do
  n=${v%%=*}; l=${v#*=}
  if [ -n "$l" ]; then export SRBD_LIB=$l; else unset SRBD_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d gpurun_out/sq_$n/p1 -o run --output-format csv -- $B > /dev/null 2>gpurun_out/sq_$n.err1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d gpurun_out/sq_$n/p2 -o run --output-format csv -- $B > /dev/null 2>gpurun_out/sq_$n.err2 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA -d gpurun_out/sq_$n/p3 -o run --output-format csv -- $B > /dev/null 2>gpurun_out/sq_$n.err3 && \
  python3 scripts/sq_summary.py gpurun_out/sq_$n/p1 gpurun_out/sq_$n/p2 gpurun_out/sq_$n/p3 --kernel "mpc_step_reg_kernel<$H>" --horizon $H --json gpurun_out/sq_$n.json > gpurun_out/sq_$n.txt || exit 1
  echo "== $n"; cat gpurun_out/sq_$n.txt
done
