#!/bin/bash
# scripts/gpu_r04.sh then scripts/gpu_profile_r04.sh in one GPU call (boxes are scarce)
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_r04.sh && bash scripts/gpu_profile_r04.sh
