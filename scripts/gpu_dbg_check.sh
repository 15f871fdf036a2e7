#!/bin/bash
# round-6 session: the release build on a parity subset, the -DSMG_CHECK build on one case (its printf unbuffered),
# then scripts/gpu_check.sh; then the LDS-budget statistics and the sparse-pass variants.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6dbg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "test_metrics_match_oracle and (basic or dups or kmix)" \
  --timeout 200 --timeout-method thread > $O/release.log 2>&1 || { tail -30 $O/release.log; exit 1; }
tail -2 $O/release.log
SMG_LIB=$PWD/sm_distributed_amd/libsmg_check.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -s -p no:cacheprovider \
  -k "test_metrics_match_oracle and basic" --timeout 200 --timeout-method thread > $O/check1.log 2>&1 || { grep -v "^  " $O/check1.log | tail -40; exit 1; }
grep -E "SMG_CHECK|passed|failed" $O/check1.log | tail -5
bash scripts/gpu_check.sh ${1:-r6dbg}/chk || exit 1
timeout -k 10 300 python -u scripts/window_stats.py > $O/window_stats.txt 2>&1 || { tail -20 $O/window_stats.txt; exit 1; }
grep -v amdgpu.ids $O/window_stats.txt
STAMPS=0 bash scripts/gpu_sparse_variants.sh ${1:-r6dbg}/var
