#!/bin/bash
# Two SQ counter passes (instruction mix, waits, LDS) over scripts/pmc_workload.py $W (default c5shard), per kernel
# -> gpurun_out/$TAG/pmc_sq_$W.txt.  Counters with --kernel-trace only; each pass under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-pmcsq}
W=${2:-c5shard}
mkdir -p gpurun_out/$TAG
out=gpurun_out/$TAG/pmc_sq_$W.txt
: > $out
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/pmcsq_${W}_$i
  timeout -k 10 400 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d /tmp/pmcsq_${W}_$i -o p -- python3 scripts/pmc_workload.py $W > gpurun_out/$TAG/pmcsq_${W}_$i.log 2>&1 || { tail -20 gpurun_out/$TAG/pmcsq_${W}_$i.log; exit 1; }
  f=$(find /tmp/pmcsq_${W}_$i -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summarize.py $f >> $out
done
cat $out
