set -o pipefail
cd /root/repo
t() { SRBD_LIB=$1 timeout -k 10 120 python bench.py --horizon 20 --steps 50 --warmup 5 --no-cpu-baseline --no-controller 2>/dev/null | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["kernels_ms"]["mpc_step_fused"])'; }
{ for r in 1 2; do echo "base $(t '')"; for v in pad20 fchain2 chain2; do echo "$v $(t ab/lib_$v.so)"; done; done; } > gpurun_out/n20_time.txt || exit 1
H=20 bash scripts/gpu_sq_ab.sh base20= pad20=ab/lib_pad20.so fchain2_20=ab/lib_fchain2.so > gpurun_out/n20_sq.txt 2>&1
