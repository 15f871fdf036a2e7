#!/bin/bash
# time each sm_distributed_amd/variants/*.so (diagnostic builds) with scripts/time_metrics.py, one process each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for so in sm_distributed_amd/variants/*.so; do
  SMG_LIB=$PWD/$so timeout -k 10 300 python scripts/time_metrics.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/variants.log || exit 1
done
