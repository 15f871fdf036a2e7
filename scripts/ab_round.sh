#!/bin/bash
# one A/B session: GPU parity tests, stamps of each variants/stamps/*.so, timing of each variants/*.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ "${AB_IGNORE_TESTS:-0}" = "1" ] || exit $rc
for so in sm_distributed_amd/variants/stamps/*.so; do
  [ -e "$so" ] || continue
  SMG_LIB=$PWD/$so timeout -k 10 300 python scripts/diag_stamps.py > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps.log | tee -a gpurun_out/stamps_all.log
done
bash scripts/variants.sh
