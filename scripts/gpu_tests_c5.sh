#!/bin/bash
# GPU parity suite, then the 1000x1000 bench leg; each step under its own limit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-c5}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --nrows 1000 --ncols 1000 --peaks ${C5_PEAKS:-1000} --n-sf ${C5_NSF:-2000} > gpurun_out/$TAG/c5.json 2> gpurun_out/$TAG/c5.err || { tail -20 gpurun_out/$TAG/c5.err; exit 1; }
cat gpurun_out/$TAG/c5.json
