#!/bin/bash
# HBM traffic of the wide pass on one rank's shard of config 5 (FETCH_SIZE and WRITE_SIZE in separate rocprofv3
# runs of scripts/pmc_workload.py c5shard), calibrated -> gpurun_out/$TAG/traffic_wide.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-trw}
mkdir -p gpurun_out/$TAG
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/trw_$c
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/trw_$c -o p -- python3 scripts/pmc_workload.py c5shard > gpurun_out/$TAG/$c.log 2>&1 || { tail -20 gpurun_out/$TAG/$c.log; exit 1; }
  cp $(find /tmp/trw_$c -name "*counter_collection.csv" | head -1) gpurun_out/$TAG/$c.csv
done
n=$(grep "calibration bytes" gpurun_out/$TAG/FETCH_SIZE.log | awk '{print $3/8}')
alg=$(grep "sum window points" gpurun_out/$TAG/FETCH_SIZE.log | awk '{for(i=1;i<=NF;i++) if($i=="points" && $(i-1)=="window") print $(i+1)*12}')
python3 scripts/traffic_summary.py gpurun_out/$TAG/FETCH_SIZE.csv gpurun_out/$TAG/WRITE_SIZE.csv $n gpurun_out/$TAG/traffic_wide.json ${KERN:-ion_wide_join_kernel} config5 $alg
rc=$?
rm -f gpurun_out/$TAG/FETCH_SIZE.csv gpurun_out/$TAG/WRITE_SIZE.csv
exit $rc
