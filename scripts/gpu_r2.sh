#!/bin/bash
# Round-2 GPU session: GPU tests (without the 160-GB huge case unless HUGE=1), smoke, bench + rocprofv3 stats.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r2x}
mkdir -p gpurun_out/$TAG
SEL=${SEL:-tests}
DESEL="--deselect tests/test_gpu_huge.py::test_more_than_2p32_points_sample_matches_oracle"
[ "${HUGE:-0}" = "1" ] && DESEL=""
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread $DESEL \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/$TAG/pytest_gpu.log
fi
if [ "${SMOKE:-1}" = "1" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
  cat gpurun_out/$TAG/smoke.log | tail -2
fi
if [ "${BENCH:-1}" = "1" ]; then
  STEPS=${STEPS:-10} WARMUP=${WARMUP:-3} PROFILE=${PROFILE:-1} bash scripts/gpu_bench.sh $TAG
fi
