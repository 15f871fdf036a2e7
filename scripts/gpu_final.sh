#!/bin/bash
# round-end session: full GPU suite (with the >2^32-point case), smoke, bench + rocprof stats, shard timing
# (scripts/gpu_full.sh), then the bench's step-time outlier A/B (collector frozen or not): scripts/gpu_final.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-final}
HUGE=1 bash scripts/gpu_full.sh $TAG > gpurun_out/$TAG.log 2>&1 || { tail -30 gpurun_out/$TAG.log; exit 1; }
tail -25 gpurun_out/$TAG.log
for i in 1 2; do
  for g in "" 1; do
    echo "## gc freeze=${g:-0}"
    SMG_BENCH_GC_FREEZE=$g SMG_BENCH_VERBOSE=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/$TAG/ab_${i}_${g:-0}.log 2>&1 || { tail -20 gpurun_out/$TAG/ab_${i}_${g:-0}.log; exit 1; }
    grep -E "step ms|steps:" gpurun_out/$TAG/ab_${i}_${g:-0}.log
  done
done
