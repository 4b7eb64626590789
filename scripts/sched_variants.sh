# Compile the kernel library under LLVM scheduler variants (CPU, cross-compiled) and print the fused
# kernels' register use / spills per variant; the libraries land in /tmp/vs/<name>.so.
# Timing on the GPU box: scripts/variant_bench.py NAME="FLAGS" ... (builds its own copies there).
set -e
mkdir -p /tmp/vs
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS=(
  "base:"
  "milp:-mllvm -amdgpu-sched-strategy=max-ilp"
  "iilp:-mllvm -amdgpu-sched-strategy=iterative-ilp"
  "imin:-mllvm -amdgpu-sched-strategy=iterative-minreg"
  "mclause:-mllvm -amdgpu-sched-strategy=max-memory-clause"
  "bias0:-mllvm -amdgpu-schedule-metric-bias=0"
  "trk:-mllvm -amdgpu-use-amdgpu-trackers=1"
)
for v in "${VARIANTS[@]}"; do
  n=${v%%:*}; f=${v#*:}
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $f -I "$ROOT/include" \
      -Rpass-analysis=kernel-resource-usage -o /tmp/vs/$n.so "$ROOT/biped_pympc_amd/csrc/srbd_mpc.hip" \
      > /tmp/vs/$n.log 2>&1; echo "$n rc=$?" ) &
done
wait
for v in "${VARIANTS[@]}"; do
  n=${v%%:*}
  for k in '_ZN4srbd19mpc_step_reg_kernelILi10EEEvNS_9FusedArgsE' '_ZN4srbd19mpc_step_reg_kernelILi20EEEvNS_9FusedArgsE'; do
    echo "$n ${k:29:3}: $(grep -A10 "Function Name: $k" /tmp/vs/$n.log | grep -E 'VGPRs:|Spill|ScratchSize|Occupancy' | sed 's/.*remark: //' | tr '\n' ' ')"
  done
done
