#!/bin/bash
# Round-end evidence in one call: the whole -m gpu suite, smoke(), a 20-step bench and the rocprofv3 kernel stats of a
# shorter run of the same command.  Each GPU step under its own time limit; stops at the first failure.
#   scripts/gpu_round_end.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r5end}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
STEPS=${STEPS:-20} WARMUP=3 bash scripts/gpu_bench.sh $TAG/bench
