#!/bin/bash
# One call, round 5: the clip_ties parity case on every path, (PROBE=1) the step-time outlier probe (3 runs), (CLIP=1)
# the clip cost at config 3 and 1000x1000, and the 8-way shard timing of config 3.  Every step under its own time limit; stops at the
# first failure.   scripts/gpu_r5_batch.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r5b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "clip_ties" \
  > $OUT/parity_clip_ties.log 2>&1 || { tail -30 $OUT/parity_clip_ties.log; exit 1; }
grep -E "passed|failed" $OUT/parity_clip_ties.log | tail -2
if [ "${PROBE:-0}" = "1" ]; then
  QPROBE=0 RUNS="a1 a2 a3" bash scripts/gpu_outlier_probe.sh $TAG/ol > $OUT/outlier.log 2>&1 || { tail -30 $OUT/outlier.log; exit 1; }
  grep -v "^  +" $OUT/outlier.log | grep -E "step ms|run |vmstat|evicted_ms" | cut -c1-600
fi
if [ "${CLIP:-0}" = "1" ]; then
  rm -f gpurun_out/clip_ref.npz
  timeout -k 10 300 python scripts/time_clip.py 500 500 2000 20000 99 > $OUT/clip_c3.txt 2>&1 || { tail -20 $OUT/clip_c3.txt; exit 1; }
  rm -f gpurun_out/clip_ref.npz
  timeout -k 10 300 python scripts/time_clip.py > $OUT/clip_1000.txt 2>&1 || { tail -20 $OUT/clip_1000.txt; exit 1; }
  grep -h "clip" $OUT/clip_c3.txt $OUT/clip_1000.txt
fi
timeout -k 10 500 python -u scripts/time_shards.py 8 > $OUT/c3_time_shards_8.txt 2>&1 || { tail -20 $OUT/c3_time_shards_8.txt; exit 1; }
grep -E "one search|estimated|gather payload|1 GPU" $OUT/c3_time_shards_8.txt
