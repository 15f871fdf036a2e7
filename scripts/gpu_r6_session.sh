#!/bin/bash
# round-6 session: the parity suite, a config-3 bench, the 8-way shard timing.  Each GPU step under its own time limit;
# stops at the first failure.   scripts/gpu_r6_session.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6s}
mkdir -p $O
if [ "${PARITY:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
  tail -2 $O/parity.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err \
    || { tail -30 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), 'ions/s', round(d['ms_per_step'],2), 'ms/step; roofline', round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms_avg'],3), 'ms; stages', d['device_chain']['stages_ms'])"
fi
if [ "${SHARDS:-1}" = "1" ]; then
  timeout -k 10 900 python -u scripts/time_shards.py 8 > $O/time_shards_8.txt 2>&1 || { tail -30 $O/time_shards_8.txt; exit 1; }
  grep -v amdgpu.ids $O/time_shards_8.txt | grep -v "passes:\|^FIT" | tail -24
fi
