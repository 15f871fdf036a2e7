#!/bin/bash
# step-time outlier diagnosis: 40 verbose bench steps (per-step times, per-launch pass times, pinned host
# allocations), twice; every run under its own limit, stop at the first failure.  scripts/gpu_outlier.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-outlier}
mkdir -p gpurun_out/$TAG
for i in 1 2; do
  SMG_BENCH_VERBOSE=1 timeout -k 10 240 python -u bench.py --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/$TAG/run_$i.log 2>&1 || { tail -20 gpurun_out/$TAG/run_$i.log; exit 1; }
  grep -E "step ms|steps:|pinned|allocator" gpurun_out/$TAG/run_$i.log
done
# the same under a kernel trace: is ion_desc8_kernel itself slow in the slow steps, or is its timing window waiting?
export TMPDIR=/tmp
SMG_BENCH_VERBOSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- \
  python3 -u bench.py --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --chain-steps 0 \
  > gpurun_out/$TAG/run_prof.log 2>&1 || { tail -20 gpurun_out/$TAG/run_prof.log; exit 1; }
grep -E "step ms|steps:|pinned" gpurun_out/$TAG/run_prof.log
python3 scripts/trace_outlier.py gpurun_out/$TAG/prof > gpurun_out/$TAG/trace_outlier.txt 2>&1 || true
grep -c desc8 gpurun_out/$TAG/trace_outlier.txt || true
# copies by blit kernels instead of the SDMA engines
HSA_ENABLE_SDMA=0 SMG_BENCH_VERBOSE=1 timeout -k 10 240 python -u bench.py --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline \
  --chain-steps 0 > gpurun_out/$TAG/run_nosdma.log 2>&1 || { tail -20 gpurun_out/$TAG/run_nosdma.log; exit 1; }
grep -E "step ms|steps:|pinned" gpurun_out/$TAG/run_nosdma.log
