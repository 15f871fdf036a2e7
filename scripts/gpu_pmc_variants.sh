#!/bin/bash
# SQ instruction counters of the sparse main pass for libsmg.so and every sm_distributed_amd/variants/*.so (one
# rocprofv3 --pmc pass each, --kernel-trace only), config-3 workload (scripts/pmc_workload.py c3).
#   scripts/gpu_pmc_variants.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-pmcv}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"}
for so in sm_distributed_amd/libsmg.so $(ls sm_distributed_amd/variants/*.so 2>/dev/null); do
  n=$(basename $so .so)
  rm -rf /tmp/pv_$n
  SMG_LIB=$PWD/$so SMG_MAIN_KERNEL=1 timeout -s KILL 200 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d /tmp/pv_$n -o p -- python3 scripts/pmc_workload.py c3 > $OUT/$n.log 2>&1 || { tail -20 $OUT/$n.log; exit 1; }
  f=$(find /tmp/pv_$n -name "*counter_collection.csv" | head -1)
  echo "## $n" >> $OUT/summary.txt
  python3 scripts/pmc_summarize.py $f | grep -E "ion_sparse" >> $OUT/summary.txt
done
cat $OUT/summary.txt
