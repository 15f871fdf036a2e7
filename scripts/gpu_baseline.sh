#!/bin/bash
# One GPU call: the -m gpu suite, then the config-3 bench and rank 0's config-5 shard bench, each under
# rocprofv3 kernel-trace stats.  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r3base}
mkdir -p gpurun_out/$TAG
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 ${TTEST:-700} python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread --durations=15 ${PYTEST_ARGS} > gpurun_out/$TAG/pytest_gpu.log 2>&1
  rc=$?
  tail -25 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
prof() {  # prof <name> <bench args...>
  local name=$1; shift
  rm -rf /tmp/prof_$name
  timeout -k 10 ${TBENCH:-400} rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- \
    python3 -u bench.py "$@" > gpurun_out/$TAG/${name}_bench.json 2> gpurun_out/$TAG/${name}_bench.err \
    || { tail -30 gpurun_out/$TAG/${name}_bench.err; return 1; }
  cat gpurun_out/$TAG/${name}_bench.json
  tail -3 gpurun_out/$TAG/${name}_bench.err
  cp $(find /tmp/prof_$name -name "*kernel_stats.csv" | head -1) gpurun_out/$TAG/${name}_kernel_stats.csv
  python3 scripts/short_stats.py gpurun_out/$TAG/${name}_kernel_stats.csv > gpurun_out/$TAG/${name}_kernel_stats_short.txt
  head -8 gpurun_out/$TAG/${name}_kernel_stats_short.txt
}
if [ "${C3:-1}" = "1" ]; then
  prof c3 --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${C3_ARGS} || exit 1
fi
if [ "${C5:-1}" = "1" ]; then
  prof c5 --config 5 --shard-of 8 --shard-rank 0 --steps ${C5STEPS:-3} --warmup 1 --no-cpu-baseline ${C5_ARGS} || exit 1
fi
