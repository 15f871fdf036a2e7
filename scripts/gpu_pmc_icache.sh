#!/bin/bash
# instruction-fetch and issue counters of the ion kernel (each pass its own run): is the 56-KB kernel
# waiting on its instruction cache?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-icache}
mkdir -p gpurun_out/$TAG
timeout -k 10 60 rocprofv3 -L > gpurun_out/$TAG/avail.txt 2>&1 || true
grep -oE "(SQC?_[A-Z_]*(ICACHE|IFETCH|INST)[A-Z_]*)" gpurun_out/$TAG/avail.txt | sort -u > gpurun_out/$TAG/avail_inst.txt
cat gpurun_out/$TAG/avail_inst.txt | tr '\n' ' '; echo
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"; do
  i=$((i+1))
  rm -rf /tmp/pmcI_$i
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d /tmp/pmcI_$i -o p -- python3 scripts/pmc_ion.py > gpurun_out/$TAG/pmc_$i.log 2>&1 || { tail -5 gpurun_out/$TAG/pmc_$i.log; continue; }
  f=$(find /tmp/pmcI_$i -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summarize.py $f | grep ion_pipe >> gpurun_out/$TAG/pmc_summary.txt
done
cat gpurun_out/$TAG/pmc_summary.txt
