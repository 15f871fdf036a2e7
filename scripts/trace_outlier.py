"""Step-outlier diagnosis from a rocprofv3 CSV trace (scripts/gpu_outlier.sh): for every ion_desc8_kernel launch,
its duration, the idle gap before it and the events just before it (kernels and memory copies), so a slow step
shows whether the descriptor kernel itself, a copy queued before it, or an idle GPU fills its timing window.

  python scripts/trace_outlier.py gpurun_out/<tag>/prof
"""
import csv
import glob
import os
import sys


def load(root):
    ev = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
    for f in glob.glob(os.path.join(root, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            b = r.get("Bytes", r.get("Size", "?"))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"C {r.get('Direction', '?')} {b} B"))
    ev.sort()
    return ev


def main():
    ev = load(sys.argv[1])
    last_end = 0
    n = 0
    for i, (s, e, name) in enumerate(ev):
        if "ion_desc8_kernel" in name:
            n += 1
            before = ev[max(0, i - 4):i]
            gap = (s - last_end) / 1e6
            line = f"desc8 #{n}: {(e - s) / 1e6:.3f} ms, idle before {gap:.3f} ms | " + "; ".join(
                f"{nm} {(ee - ss) / 1e6:.3f} ms (ends {(s - ee) / 1e6:.3f} ms before)" for ss, ee, nm in before)
            print(line)
        last_end = max(last_end, e)


if __name__ == "__main__":
    main()
