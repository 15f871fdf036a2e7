#!/bin/bash
# slow-mode A/B: 60-step verbose benches with the side and copy streams (default) and with one stream
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sab}
mkdir -p gpurun_out/$TAG
for v in one1 def1 one2 def2; do
  case $v in one*) E="SMG_ONE_STREAM=1";; *) E="SMG_ONE_STREAM=0";; esac
  timeout -k 10 300 env $E SMG_BENCH_VERBOSE=1 python3 -u bench.py --no-cpu-baseline --chain-steps 0 --steps 60 --warmup 3 \
    > gpurun_out/$TAG/$v.json 2> gpurun_out/$TAG/$v.err || { tail -20 gpurun_out/$TAG/$v.err; exit 1; }
  echo "$v: $(grep -E 'step ms' gpurun_out/$TAG/$v.err)"
  echo "   $(grep -E 'steps:' gpurun_out/$TAG/$v.err | cut -c1-330)"
done
