#!/bin/bash
# HBM traffic of the sort kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs of scripts/pmc_sort.py
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsort
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/ps_$c
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/ps_$c -o p -- python3 scripts/pmc_sort.py > gpurun_out/pmcsort/$c.log 2>&1 || { tail -20 gpurun_out/pmcsort/$c.log; exit 1; }
  python3 - "$c" $(find /tmp/ps_$c -name "*counter_collection.csv" | head -1) > gpurun_out/pmcsort/$c.txt <<'PY'
import csv, sys, re
from collections import defaultdict
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[2])):
    if r["Counter_Name"] != sys.argv[1]:
        continue
    k = r.get("Kernel_Name") or ""
    m = re.search(r"smg::(\w+)(<[^>]*>)?", k)
    key = (m.group(1) + (m.group(2) or "")) if m else k[:40]
    acc[key].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:60s} n={len(v):3d} avg={sum(v)/len(v):.4e}")
PY
done
cat gpurun_out/pmcsort/FETCH_SIZE.txt gpurun_out/pmcsort/WRITE_SIZE.txt
