#!/bin/bash
# first-timed-step outlier: bench variants (warm-up length, pass timers off) with per-step times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-fs}
mkdir -p gpurun_out/$TAG
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py --no-cpu-baseline --chain-steps 0 --steps 12 $BA \
    > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || { tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  echo "$name: $(grep -E 'step ms|steps:' gpurun_out/$TAG/$name.err | cut -c1-140 | tr '\n' ' ')"
  echo "   $(grep 'pass launches' gpurun_out/$TAG/$name.err | cut -c1-120)"
}
BA="--warmup 3" run A1 SMG_BENCH_VERBOSE=1
BA="--warmup 10" run B SMG_BENCH_VERBOSE=1
BA="--warmup 3" run C SMG_BENCH_VERBOSE=1 SMG_BENCH_NO_TIMERS=1
BA="--warmup 3" run A2 SMG_BENCH_VERBOSE=1
BA="--warmup 3" run D SMG_BENCH_NO_TIMERS=1
