#!/bin/bash
# Dense-path session: parity file (forced dense modes 1 and 2), wide-pass phase stamps (libsmg_stamps.so),
# path timings on the 1000x1000 dense workload, then the config-5 per-rank bench under rocprofv3 stats.
# Each GPU step has its own limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-wide}
mkdir -p gpurun_out/$TAG
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/$TAG/pytest_parity.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest_parity.log; exit 1; }
  tail -3 gpurun_out/$TAG/pytest_parity.log
fi
if [ -f sm_distributed_amd/libsmg_stamps.so ]; then
  timeout -k 10 300 python3 -u scripts/diag_wide_stamps.py > gpurun_out/$TAG/stamps.txt 2>&1 \
    || { tail -20 gpurun_out/$TAG/stamps.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$TAG/stamps.txt
  for f in sm_distributed_amd/libsmg_stamps_x*.so; do
    [ -f "$f" ] || continue
    v=$(basename $f .so)
    SMG_LIB=$f timeout -k 10 300 python3 -u scripts/diag_wide_stamps.py > gpurun_out/$TAG/stamps_$v.txt 2>&1 \
      || { tail -20 gpurun_out/$TAG/stamps_$v.txt; exit 1; }
    echo "== $v"; grep -v amdgpu.ids gpurun_out/$TAG/stamps_$v.txt | tail -9
  done
fi
timeout -k 10 400 python -u scripts/time_paths.py 1000 1000 2100 1000 > gpurun_out/$TAG/time_paths_dense.txt 2>&1 \
  || { tail -20 gpurun_out/$TAG/time_paths_dense.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/time_paths_dense.txt
if [ "${C5:-1}" = "1" ]; then
  bash scripts/gpu_config5.sh $TAG/c5
fi
