#!/bin/bash
# A/B of an environment switch on the API bench: scripts/gpu_ab_env.sh VAR (runs VAR=0,1,0,1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abenv
for v in 0 1 0 1; do
  env $1=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --chain-steps 0 \
    > gpurun_out/abenv/bench_$v.json 2> gpurun_out/abenv/bench_$v.err || { tail -20 gpurun_out/abenv/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abenv/bench_$v.json')); print('$1=$v', round(d['ms_per_step'],2), 'ms', round(d['value']/1e6,3), 'M ions/s')"
done
