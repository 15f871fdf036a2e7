#!/bin/bash
# A/B of the descriptor pass: per-launch HIP-event times of pass 0 (and the main pass) from verbose benches,
# alternating the current library and a variant (SMG_LIB), with the shader clock of each run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-dab}; VAR=${2:-sm_distributed_amd/variants/d8old.so}
mkdir -p gpurun_out/$TAG
for r in new1 old1 new2 old2; do
  case $r in old*) L=$VAR;; *) L=sm_distributed_amd/libsmg.so;; esac
  timeout -k 10 300 env SMG_LIB=$L SMG_BENCH_VERBOSE=1 python3 -u bench.py --no-cpu-baseline --chain-steps 0 --steps 15 --warmup 3 \
    > gpurun_out/$TAG/$r.json 2> gpurun_out/$TAG/$r.err || { tail -20 gpurun_out/$TAG/$r.err; exit 1; }
  python3 - gpurun_out/$TAG/$r.err $r <<'PY'
import re, sys, numpy as np
t = open(sys.argv[1]).read()
v = [x.split(":") for x in re.search(r"pass launches \(pass:ms\): (.*)", t).group(1).split()]
d = [float(ms) for p, ms in v if p == "0"]; m = [float(ms) for p, ms in v if p == "1"]
clk = re.search(r"shader clock MHz (.*)", t).group(1)
print(f"{sys.argv[2]}: desc median {np.median(d):.3f} ms, main median {np.median(m):.2f} ms, clock {clk}")
PY
done
