#!/bin/bash
# PMC passes (SQ issue/wait mix, LDS, L2) of the ion kernel for each variants/*.so: one rocprofv3 run per
# (variant, counter set); summaries appended to gpurun_out/pmc_variants.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for so in sm_distributed_amd/variants/*.so; do
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
              "SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA" \
              "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    rm -rf /tmp/pmcv
    SMG_LIB=$PWD/$so timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d /tmp/pmcv -o p -- python3 scripts/pmc_ion.py > gpurun_out/pmcv.log 2>&1 || { tail -20 gpurun_out/pmcv.log; exit 1; }
    f=$(find /tmp/pmcv -name "*counter_collection.csv" | head -1)
    echo "== $(basename $so) pass $i" >> gpurun_out/pmc_variants.txt
    python3 scripts/pmc_summarize.py $f | grep "ion_pipe\|ion_lds" >> gpurun_out/pmc_variants.txt
  done
done
cat gpurun_out/pmc_variants.txt
