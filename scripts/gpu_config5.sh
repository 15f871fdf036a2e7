#!/bin/bash
# Config-5 per-rank workload on one GPU: 1000x1000 px, Poisson(5000) centroids (5e9 points, replicated on
# every rank), a 5,000-formula ion shard (40k formulas over 8 ranks).  Bench only, no profiler.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-c5}
mkdir -p gpurun_out/$TAG
timeout -k 10 ${T:-900} python -u bench.py --nrows 1000 --ncols 1000 --peaks 5000 --n-sf ${NSF:-5000} \
  --steps ${STEPS:-3} --warmup ${WARMUP:-1} --cpu-ions ${CPU_IONS:-64} ${EXTRA} \
  > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
cat gpurun_out/$TAG/bench.json
tail -20 gpurun_out/$TAG/bench.err
exit $rc
