#!/bin/bash
# step-time outlier census: four verbose 25-step benches (per-step and per-pass times), GPU clocks before/after
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-ol}
mkdir -p gpurun_out/$TAG
(rocm-smi --showclocks 2>/dev/null | grep -E "sclk|mclk|fclk" | head -6) > gpurun_out/$TAG/clocks_before.txt
for i in 1 2 3 4; do
  timeout -k 10 300 env SMG_BENCH_VERBOSE=1 python3 -u bench.py --no-cpu-baseline --chain-steps 0 --steps 25 --warmup 3 \
    > gpurun_out/$TAG/b$i.json 2> gpurun_out/$TAG/b$i.err || { tail -20 gpurun_out/$TAG/b$i.err; exit 1; }
  echo "b$i: $(grep -E 'steps:' gpurun_out/$TAG/b$i.err | cut -c1-200)"
  python3 - gpurun_out/$TAG/b$i.err <<'PY'
import sys, re
t = open(sys.argv[1]).read()
m = re.search(r"pass launches \(pass:ms\): (.*)", t)
if m:
    v = [tuple(x.split(":")) for x in m.group(1).split()]
    slow = [(i // 6, p, float(ms)) for i, (p, ms) in enumerate(v) if (p == "1" and float(ms) > 36.5) or (p == "0" and float(ms) > 1.5)]
    print("   slow passes (step, pass, ms):", slow)
PY
done
(rocm-smi --showclocks 2>/dev/null | grep -E "sclk|mclk|fclk" | head -6) > gpurun_out/$TAG/clocks_after.txt
cat gpurun_out/$TAG/clocks_before.txt gpurun_out/$TAG/clocks_after.txt
