#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace; each pass its own run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rm -rf /tmp/pmc_$i
  timeout -k 10 400 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d /tmp/pmc_$i -o p -- python3 scripts/pmc_run.py > gpurun_out/$TAG/pmc_$i.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc_$i.log; exit 1; }
  f=$(find /tmp/pmc_$i -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summarize.py $f >> gpurun_out/$TAG/pmc_summary.txt
done
cat gpurun_out/$TAG/pmc_summary.txt
