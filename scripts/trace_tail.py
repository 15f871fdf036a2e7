"""Summarise the last N dispatches of a rocprofv3 kernel_trace.csv (name, duration, gap to the previous end):
the timeline of the final timed repetition of a short script.  usage: trace_tail.py trace.csv N"""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2])
prev = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(.*", "", r["Kernel_Name"])
    name = re.sub(r"<.*>", "<..>", name)[:70]
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(e - s) / 1e3:9.1f} us  gap {gap:8.1f} us  {name}")
    prev = e
