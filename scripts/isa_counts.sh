#!/bin/bash
# Static instruction counts of one kernel (default: the fused N=10 step) from a csrc directory:
#   scripts/isa_counts.sh [CSRC_DIR] [KERNEL_SYMBOL] [extra hipcc flags...]
CSRC=${1:-$(dirname "$0")/../biped_pympc_amd/csrc}
SYM=${2:-_ZN4srbd19mpc_step_reg_kernelILi10EEEvNS_9FusedArgsE}
shift 2 2>/dev/null
INC=$(cd "$(dirname "$0")/.." && pwd)/include
OUT=$(mktemp /tmp/isa.XXXXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I"$INC" "$@" --cuda-device-only -S -o "$OUT" "$CSRC/srbd_mpc.hip" 2>/dev/null || exit 1
awk -v sym="$SYM:" '$1 == sym {on = 1} on {print} on && /s_endpgm/ {exit}' "$OUT" > "$OUT.k"
printf "valu %d  salu %d  ds %d  dpp %d  cndmask %d  vmem %d\n" \
  "$(grep -cE '^\s*v_' "$OUT.k")" "$(grep -cE '^\s*s_' "$OUT.k")" "$(grep -cE '^\s*ds_' "$OUT.k")" \
  "$(grep -c '_dpp' "$OUT.k")" "$(grep -c v_cndmask "$OUT.k")" "$(grep -cE '^\s*(global|buffer|flat)_' "$OUT.k")"
rm -f "$OUT" "$OUT.k"
