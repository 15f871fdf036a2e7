#!/bin/bash
# sparse-pass variant A/B (scripts/gpu_sparse_variants.sh) after the LDS-budget statistics; stops at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6var}
mkdir -p $O
if [ "${STATS:-1}" = "1" ]; then
  timeout -k 10 300 python -u scripts/window_stats.py > $O/window_stats.txt 2>&1 || { tail -20 $O/window_stats.txt; exit 1; }
  grep -v amdgpu.ids $O/window_stats.txt
fi
STAMPS=${STAMPS:-0} bash scripts/gpu_sparse_variants.sh ${1:-r6var}
