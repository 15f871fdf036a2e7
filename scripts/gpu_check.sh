#!/bin/bash
# The -DSMG_CHECK diagnostic library (make -C sm_distributed_amd/csrc check -> libsmg_check.so) over the GPU parity
# suite, the API tests and a config-3 bench: every position claimed once per pass, every descriptor equal to its
# lo / hi / ion_off / ion_order, every hit index inside its window and [0, n_points), no reject-list overflow
# (DESIGN.md §6).  Each GPU step under its own time limit; stops at the first failure.
#   scripts/gpu_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r6chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export SMG_LIB=$PWD/sm_distributed_amd/libsmg_check.so
export SMG_CHECK_OUT=$OUT/check_counters.txt
timeout -k 10 900 python -u -m pytest ${CHECK_TESTS:-tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_distributed.py} \
  -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_check.log 2>&1 \
  || { tail -40 $OUT/pytest_check.log; exit 1; }
tail -3 $OUT/pytest_check.log
cat $OUT/check_counters.txt
timeout -k 10 600 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --chain-steps 2 \
  > $OUT/bench_check.json 2> $OUT/bench_check.err || { tail -30 $OUT/bench_check.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench_check.json')); print('check bench:', d['ms_per_step'], d.get('check'))"
