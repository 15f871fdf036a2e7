"""Average rocprofv3 counter_collection.csv per (kernel, counter) for our kernels + the calibration copy."""
import csv, re, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
acc = defaultdict(list)
for r in rows:
    name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
    short = re.sub(r"\(anonymous namespace\)::", "", name)
    short = re.sub(r"\(.*", "", short)
    short = re.sub(r"<.*>", "<..>", short)
    m = re.search(r"ion_pipe_kernel<[^,]*, (\d+)", name)
    if m:
        short = "smg::ion_pipe_kernel[" + m.group(1) + "]"
    if not any(k in name for k in ("smg::", "rocprim")):
        continue
    acc[(short[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:62s} {c:24s} n={len(v):3d} avg={sum(v)/len(v):.4g}")
