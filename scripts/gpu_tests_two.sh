#!/bin/bash
# GPU parity suite, then the 1000x1000 bench leg (two-level LDS passes); each step under its own limit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/two
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/two/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/two/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/two/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --nrows 1000 --ncols 1000 --peaks 1000 --n-sf 2000 > gpurun_out/two/c5.json 2> gpurun_out/two/c5.err || { tail -20 gpurun_out/two/c5.err; exit 1; }
cat gpurun_out/two/c5.json
