#!/bin/bash
# bench line + rocprofv3 kernel-trace stats of the same command: gpu_prof.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
rm -rf /tmp/prof_$TAG
timeout -k 10 ${TPROF:-500} rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
  python3 -u bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
tail -2 gpurun_out/$TAG/bench.err
for f in $(find /tmp/prof_$TAG -name "*kernel_stats.csv"); do cp $f gpurun_out/$TAG/kernel_stats.csv; done
python3 scripts/short_stats.py gpurun_out/$TAG/kernel_stats.csv 16 | tee gpurun_out/$TAG/kernel_stats_short.txt
