#!/bin/bash
# SQ counters of the config-3 main pass, ion_pipe_kernel<512> (SMG_MAIN_KERNEL=0) against ion_sparse_kernel (1):
# two counter passes each (rocprofv3 --pmc with --kernel-trace only), scripts/pmc_workload.py c3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-pmcm}
mkdir -p gpurun_out/$TAG
for mk in ${KERNELS:-0 1}; do
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
              "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
              "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    rm -rf /tmp/pmcm_${mk}_$i
    SMG_MAIN_KERNEL=$mk timeout -s KILL 200 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d /tmp/pmcm_${mk}_$i -o p -- python3 scripts/pmc_workload.py c3 > gpurun_out/$TAG/pmc_${mk}_$i.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc_${mk}_$i.log; exit 1; }
    f=$(find /tmp/pmcm_${mk}_$i -name "*counter_collection.csv" | head -1)
    echo "## main kernel $mk pass $i" >> gpurun_out/$TAG/pmc_summary.txt
    python3 scripts/pmc_summarize.py $f | grep -E "ion_pipe|ion_sparse" >> gpurun_out/$TAG/pmc_summary.txt
  done
done
cat gpurun_out/$TAG/pmc_summary.txt
