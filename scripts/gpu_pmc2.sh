#!/bin/bash
# rocprofv3 PMC passes over scripts/pmc_workload.py <c3|dense> (counters with --kernel-trace only; one counter
# set per run, each under its own time limit) -> gpurun_out/$TAG/pmc_<workload>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-pmc}
W=${2:-c3}
mkdir -p gpurun_out/$TAG
out=gpurun_out/$TAG/pmc_$W.txt
: > $out
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rm -rf /tmp/pmc_${W}_$i
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d /tmp/pmc_${W}_$i -o p -- python3 scripts/pmc_workload.py $W > gpurun_out/$TAG/pmc_${W}_$i.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc_${W}_$i.log; exit 1; }
  f=$(find /tmp/pmc_${W}_$i -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summarize.py $f >> $out
done
grep -h "points\|calibration" gpurun_out/$TAG/pmc_${W}_1.log >> $out
cat $out
