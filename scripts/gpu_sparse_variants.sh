#!/bin/bash
# A/B of the main pass at config 3 (scripts/time_metrics.py, one process each): ion_pipe_kernel<512> first (the
# reference table), the HEAD build's sparse pass, then every sm_distributed_amd/variants/*.so; then the stamps of the HEAD build.
# scripts/gpu_sparse_variants.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-spv}
mkdir -p gpurun_out/$TAG
rm -f gpurun_out/ab_ref.npz
SMG_MAIN_KERNEL=0 timeout -k 10 300 python scripts/time_metrics.py ${VARIANT_ARGS} > gpurun_out/variant.log 2>&1 || { tail -20 gpurun_out/variant.log; exit 1; }
grep -v amdgpu.ids gpurun_out/variant.log | tee gpurun_out/$TAG/variants.txt
SMG_MAIN_KERNEL=1 timeout -k 10 300 python scripts/time_metrics.py ${VARIANT_ARGS} > gpurun_out/variant.log 2>&1 || { tail -20 gpurun_out/variant.log; exit 1; }
grep -v amdgpu.ids gpurun_out/variant.log | tee -a gpurun_out/$TAG/variants.txt
for so in $(ls sm_distributed_amd/variants/*.so 2>/dev/null); do
  SMG_LIB=$PWD/$so timeout -k 10 300 python scripts/time_metrics.py ${VARIANT_ARGS} > gpurun_out/variant.log 2>&1 || { tail -20 gpurun_out/variant.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/variant.log | tee -a gpurun_out/$TAG/variants.txt
done
if [ "${STAMPS:-1}" = "1" ]; then
  timeout -k 10 300 python -u scripts/diag_sparse_stamps.py ${VARIANT_ARGS} > gpurun_out/$TAG/stamps.txt 2>&1 || { tail -20 gpurun_out/$TAG/stamps.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$TAG/stamps.txt
fi
