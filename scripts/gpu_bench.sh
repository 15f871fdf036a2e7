#!/bin/bash
# one GPU session: bench (JSON line) + rocprofv3 kernel-trace stats of a shorter run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
tail -3 gpurun_out/$TAG/bench.err
if [ "${PROFILE:-1}" = "1" ]; then
  rm -rf /tmp/prof_$TAG
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/prof.log 2>&1 || { tail -30 gpurun_out/$TAG/prof.log; exit 1; }
  for f in $(find /tmp/prof_$TAG -name "*kernel_stats.csv"); do cp $f gpurun_out/$TAG/kernel_stats.csv; done
  python3 scripts/short_stats.py gpurun_out/$TAG/kernel_stats.csv | tee gpurun_out/$TAG/kernel_stats_short.txt
fi
