#!/bin/bash
# HBM-traffic counters of the ion kernel (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs), calibrated
# -> gpurun_out/$TAG/traffic.json (copy to profiles/ to have bench.py report it)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-traffic}
mkdir -p gpurun_out/$TAG
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/tr_$c
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/tr_$c -o p -- python3 scripts/pmc_ion.py > gpurun_out/$TAG/$c.log 2>&1 || { tail -20 gpurun_out/$TAG/$c.log; exit 1; }
  cp $(find /tmp/tr_$c -name "*counter_collection.csv" | head -1) gpurun_out/$TAG/$c.csv
done
n=$(grep "calibration bytes" gpurun_out/$TAG/FETCH_SIZE.log | awk '{print $3/8}')
# the main pass's kernel (KERNEL=ion_pipe_kernel[512] with SMG_MAIN_KERNEL=0); config 3's algorithmic bytes are
# 12 B x 6,439,292,385 window points
python3 scripts/traffic_summary.py gpurun_out/$TAG/FETCH_SIZE.csv gpurun_out/$TAG/WRITE_SIZE.csv $n gpurun_out/$TAG/traffic.json \
  "${KERNEL:-ion_sparse_kernel}" config3 77271508620
rc=$?
rm -f gpurun_out/$TAG/FETCH_SIZE.csv gpurun_out/$TAG/WRITE_SIZE.csv  # large; the summary keeps what is used
exit $rc
