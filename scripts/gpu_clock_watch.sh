#!/bin/bash
# step-time outlier vs clocks/power: rocm-smi sampled every ~0.2 s in the background during 60-step verbose benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-cw}
mkdir -p gpurun_out/$TAG
watch_smi() {
  local end=$((SECONDS + 200))
  while [ $SECONDS -lt $end ]; do
    echo "T $(date +%s.%N)"
    rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|Power|Temperature" | grep -v "^$"
    sleep 0.2
  done
}
watch_smi > gpurun_out/$TAG/smi.txt 2>&1 &
WPID=$!
for i in 1 2 3; do
  echo "B$i start $(date +%s.%N)" >> gpurun_out/$TAG/marks.txt
  timeout -k 10 300 env SMG_BENCH_VERBOSE=1 python3 -u bench.py --no-cpu-baseline --chain-steps 0 --steps 60 --warmup 3 \
    > gpurun_out/$TAG/b$i.json 2> gpurun_out/$TAG/b$i.err || { kill $WPID; tail -20 gpurun_out/$TAG/b$i.err; exit 1; }
  echo "B$i end $(date +%s.%N)" >> gpurun_out/$TAG/marks.txt
  echo "b$i: $(grep -E 'step ms' gpurun_out/$TAG/b$i.err)"
done
kill $WPID
wc -l gpurun_out/$TAG/smi.txt
grep -E "sclk" gpurun_out/$TAG/smi.txt | sort | uniq -c | sort -rn | head -12
grep -E "Power" gpurun_out/$TAG/smi.txt | sort | uniq -c | sort -rn | head -5
grep -E "Temperature" gpurun_out/$TAG/smi.txt | sort | uniq -c | sort -rn | head -8
