#!/bin/bash
# Config-5 per-rank workload on one GPU: 1000x1000 px, Poisson(5000) centroids (5e9 points, replicated on
# every rank), a 5,000-formula ion shard (40k formulas over 8 ranks).  Bench under rocprofv3 kernel-trace stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-c5}
mkdir -p gpurun_out/$TAG
rm -rf /tmp/prof_c5
timeout -k 10 ${T:-900} rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c5 -o run -- \
  python3 -u bench.py --nrows 1000 --ncols 1000 --peaks 5000 --n-sf ${NSF:-5000} \
  --steps ${STEPS:-2} --warmup ${WARMUP:-1} --no-cpu-baseline ${EXTRA} \
  > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
for f in $(find /tmp/prof_c5 -name "*kernel_stats.csv"); do cp $f gpurun_out/$TAG/kernel_stats.csv; done
python3 scripts/short_stats.py gpurun_out/$TAG/kernel_stats.csv | tee gpurun_out/$TAG/kernel_stats_short.txt
