#!/bin/bash
# round 3: GPU tests (optional subset) then the bench line; every GPU step under its own time limit, stop at the
# first failure.  TESTS="" skips the tests, BENCH=0 skips the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r3x}
mkdir -p gpurun_out/$TAG
if [ -n "${TESTS-tests}" ]; then
  timeout -k 10 ${TTEST:-900} python -u -m pytest ${TESTS-tests} -m gpu -v -p no:cacheprovider --timeout 600 \
    --timeout-method thread --durations=20 -rP ${PYTEST_ARGS} > gpurun_out/$TAG/pytest_gpu.log 2>&1
  rc=$?
  tail -40 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${TBENCH:-600} python -u bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS} \
    > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
  cat gpurun_out/$TAG/bench.json
  tail -3 gpurun_out/$TAG/bench.err
fi
