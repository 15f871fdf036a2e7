#!/bin/bash
# Step-time outlier probe (verdict round 4, item 3), one call:
#   1. scripts/queue_slice_probe: does a second queue with pending work stall a kernel that holds every CU?
#   2. the KFD queues on our GPU (/sys/class/kfd/kfd/proc, gpu_id matched by PCI bus), sampled every 0.25 s during
#   3. 60-step verbose benches (RUNS="1 2 ...": per-step clock and device pass times in each line)
# scripts/gpu_outlier_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-olp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${QPROBE:-1}" = "1" ]; then
  timeout -k 10 120 scripts/queue_slice_probe > $OUT/queue_probe.txt 2>&1 || { cat $OUT/queue_probe.txt; exit 1; }
  cat $OUT/queue_probe.txt
fi
# our GPU's KFD gpu_id: the topology node whose PCI location matches the device torch sees
OURS=$(timeout -k 10 120 python3 - <<'EOF3'
import glob, os, torch
bus = torch.cuda.get_device_properties(0).pci_bus_id
for d in glob.glob("/sys/class/kfd/kfd/topology/nodes/*"):
    try:
        props = dict(l.split() for l in open(os.path.join(d, "properties")) if len(l.split()) == 2)
        gid = open(os.path.join(d, "gpu_id")).read().strip()
    except OSError:
        continue
    if gid != "0" and (int(props.get("location_id", "-1")) >> 8) & 0xFF == bus:
        print(gid)
EOF3
)
echo "our gpu_id: $OURS"
echo "numa_balancing $(cat /proc/sys/kernel/numa_balancing 2>&1); THP $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>&1); khugepaged defrag $(cat /sys/kernel/mm/transparent_hugepage/khugepaged/defrag 2>&1)"
for run in ${RUNS:-1}; do
# runs named a* / c*: the default memory policy (SMG_NUMA_OPTOUT=0); b*: the process opted out of NUMA balancing
case $run in a*|c*) export SMG_NUMA_OPTOUT=0 ;; *) export SMG_NUMA_OPTOUT=1 ;; esac
# runs named c*: no shader-clock polling (pp_dpm_sclk) by the bench
case $run in c*) export SMG_BENCH_NO_CLOCK=1 ;; *) unset SMG_BENCH_NO_CLOCK ;; esac
SMG_BENCH_VERBOSE=1 timeout -k 10 400 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --chain-steps 0 \
  > $OUT/bench_$run.json 2> $OUT/bench_err_$run.txt &
TPID=$!
# every KFD process's queues on this node with the GPU each queue is on; the bench's own queues name our GPU
( while kill -0 $TPID 2>/dev/null; do
    echo "t $(date +%s.%N)"
    for d in /sys/class/kfd/kfd/proc/*; do
      [ -d "$d" ] || continue
      p=$(basename $d)
      for q in $d/queues/*; do
        [ -d "$q" ] || continue
        echo "q $p $(cat $q/gpuid 2>/dev/null)"
      done
      # KFD's per-process eviction time on our GPU (queues evicted, e.g. for a userptr invalidation)
      [ -r "$d/stats_$OURS/evicted_ms" ] && echo "e $p $(cat $d/stats_$OURS/evicted_ms 2>/dev/null)"
    done
    # node-wide page migration / compaction / THP / KSM counters (what can invalidate a userptr range)
    echo "v $(grep -E '^(pgmigrate_success|compact_migrate_scanned|compact_isolated|compact_daemon_wake|thp_collapse_alloc|thp_split_pmd|numa_pages_migrated|ksm_[a-z_]*|pswpout|pgsteal_kswapd|pgscan_kswapd|drop_pagecache) ' /proc/vmstat | tr ' \n' '= ')"
    sleep 0.25
  done ) > $OUT/kfd_queues_$run.txt 2>&1 &
# (once) what KFD exposes per process
if [ "$run" = "${RUNS%% *}" ]; then
  sleep 3
  for d in /sys/class/kfd/kfd/proc/*; do
    [ -d "$d/stats_$OURS" ] || continue
    echo "== $d"; ls -R "$d" | head -40; for f in $d/stats_$OURS/*; do echo "$f: $(cat $f 2>/dev/null)"; done
  done > $OUT/kfd_proc_files.txt 2>&1
fi
SAMPLER=$!
wait $TPID
rc=$?
wait $SAMPLER
echo "bench rc $rc"
grep -E "step ms" $OUT/bench_err_$run.txt
python3 -c "
import json, sys
d = json.loads(open('$OUT/bench_$run.json').read().strip().splitlines()[-1])
e = d.get('steps_evicted_ms')
print('run $run: numa', d.get('numa_balancing'), 'evicted ms over the timed steps', None if e is None else sum(e),
      'steps with evictions', None if e is None else sum(1 for x in e if x))"
[ $rc = 0 ] || exit $rc
python3 - "$OUT/kfd_queues_$run.txt" "$OURS" <<'EOF2'
import sys, collections
ours = set(sys.argv[2].split())
samples, cur = [], None
ev = collections.defaultdict(list)
vm = []
for ln in open(sys.argv[1]):
    p = ln.split()
    if p[0] == "t":
        cur = collections.Counter()
        samples.append((float(p[1]), cur))
    elif p[0] == "q" and cur is not None and len(p) == 3:
        cur[(p[1], p[2])] += 1
    elif p[0] == "e" and cur is not None and len(p) == 3:
        ev[p[1]].append((samples[-1][0], p[2]))
    elif p[0] == "v" and samples:
        vm.append((samples[-1][0], dict(x.split("=") for x in p[1:] if "=" in x)))
t0 = samples[0][0] if samples else 0.0
pids = collections.Counter()
for t, c in samples:
    on = {pid: n for (pid, g), n in c.items() if g in ours}
    pids.update(on.keys())
print(f"{len(samples)} samples over {samples[-1][0] - t0 if samples else 0:.1f} s; processes with queues on our GPU "
      f"(host pid -> samples): {dict(pids)}")
for t, c in samples:
    on = {pid: n for (pid, g), n in c.items() if g in ours}
    print(f"  +{t - t0:6.2f} s  queues on our GPU by pid: {on}")
for pid, v in ev.items():
    if pid in pids:
        print(f"evicted_ms of {pid} on our GPU: " + " ".join(f"+{t - t0:.2f}s:{x}" for t, x in v))
# vmstat counters that moved during the run, sample by sample
if vm:
    keys = sorted(vm[0][1])
    prev = vm[0][1]
    for t, d in vm[1:]:
        moved = {k: int(d[k]) - int(prev[k]) for k in keys if k in d and d[k] != prev.get(k)}
        if moved:
            print(f"  vmstat +{t - t0:6.2f} s: {moved}")
        prev = d
EOF2
done
