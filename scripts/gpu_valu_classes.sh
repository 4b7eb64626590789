# Dynamic VALU instruction classes of the fused N=10 step kernel (two rocprofv3 --pmc passes, 8 SQ
# counters each) -> gpurun_out/valu_classes.{txt,json}; per-wave (= per-QP) averages via sq_summary.py.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT -d gpurun_out/pmc_valu1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-controller --kernel-reps 1 > gpurun_out/pmc_valu1.json 2>gpurun_out/pmc_valu1.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_IOPS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F64 -d gpurun_out/pmc_valu2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-controller --kernel-reps 1 > gpurun_out/pmc_valu2.json 2>gpurun_out/pmc_valu2.err && \
python3 scripts/sq_summary.py gpurun_out/pmc_valu1 gpurun_out/pmc_valu2 --json gpurun_out/valu_classes.json > gpurun_out/valu_classes.txt
