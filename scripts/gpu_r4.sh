#!/bin/bash
# round-4 GPU session: GPU suite (without the >2^32-point case), a 100-step verbose bench (step-time outlier check),
# rocprof kernel stats of the bench, config-5 8-way shard timing.  Every GPU step under its own limit; stop at the
# first failure.   scripts/gpu_r4.sh TAG [steps...]  (steps: tests bench prof c5shards c3shards)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r4}
shift
STEPS=${@:-tests bench prof c5shards}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for s in $STEPS; do
  echo "## $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider \
        ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
      tail -3 gpurun_out/$TAG/pytest_gpu.log; grep -h "config 5\|rank [0-9]/8:\|config 3 API\|8-way\|steady-state" gpurun_out/$TAG/pytest_gpu.log | head -30 ;;
    bench)
      SMG_BENCH_VERBOSE=1 timeout -k 10 400 python -u bench.py --steps ${BENCH_STEPS:-100} --warmup 3 ${BENCH_ARGS} \
        > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
      grep -E "step ms|pinned host" gpurun_out/$TAG/bench.err | cut -c1-700; cut -c1-600 gpurun_out/$TAG/bench.json ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- \
        python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/prof_bench.json 2> gpurun_out/$TAG/prof_bench.err \
        || { tail -30 gpurun_out/$TAG/prof_bench.err; exit 1; }
      f=$(find gpurun_out/$TAG/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/$TAG/kernel_stats.csv
      python3 scripts/short_stats.py gpurun_out/$TAG/kernel_stats.csv 16 | tee gpurun_out/$TAG/kernel_stats_short.txt
      rm -rf gpurun_out/$TAG/prof ;;  # the traces exceed what gpurun copies back
    c5shards)
      CONFIG=5 timeout -k 10 900 python3 -u scripts/time_shards.py 8 > gpurun_out/$TAG/c5_time_shards_8.txt 2>&1 \
        || { tail -30 gpurun_out/$TAG/c5_time_shards_8.txt; exit 1; }
      grep -v amdgpu.ids gpurun_out/$TAG/c5_time_shards_8.txt ;;
    variants)
      timeout -k 10 900 bash scripts/variants.sh > gpurun_out/$TAG/variants.log 2>&1 || { tail -30 gpurun_out/$TAG/variants.log; exit 1; }
      cp gpurun_out/variants.log gpurun_out/$TAG/variants_summary.log 2>/dev/null; grep "ion_metrics" gpurun_out/$TAG/variants.log ;;
    stamps)
      timeout -k 10 300 python3 -u scripts/diag_stamps.py > gpurun_out/$TAG/stamps.txt 2>&1 || { tail -30 gpurun_out/$TAG/stamps.txt; exit 1; }
      grep -v amdgpu.ids gpurun_out/$TAG/stamps.txt ;;
    c3shards)
      timeout -k 10 400 python3 -u scripts/time_shards.py 8 > gpurun_out/$TAG/c3_time_shards_8.txt 2>&1 \
        || { tail -30 gpurun_out/$TAG/c3_time_shards_8.txt; exit 1; }
      grep -v amdgpu.ids gpurun_out/$TAG/c3_time_shards_8.txt ;;
  esac
done
echo "## done $(date +%T)"
