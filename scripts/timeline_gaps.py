"""Timeline of one step from rocprofv3 CSV traces (scripts/gpu_timeline.sh): kernels in start order with their
duration and the GPU idle gap before each, and the HIP runtime calls longer than a threshold in that window.
A step starts at a launch of `--start` (default flag_duplicates_kernel / slice_count_kernel) and ends before the
next one; the last complete step is printed.

usage: timeline_gaps.py kernel_trace.csv hip_api_trace.csv [--start NAME] [--min-us 30]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("ktrace")
ap.add_argument("htrace")
ap.add_argument("--start", default="flag_duplicates_kernel")
ap.add_argument("--min-us", type=float, default=30.0)
ap.add_argument("--which", type=int, default=-2, help="step index among the detected starts (-2: second to last)")
a = ap.parse_args()


def rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


ks = []
for r in rows(a.ktrace):
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "?")))
ks.sort()
starts = [i for i, k in enumerate(ks) if a.start in k[2]]
if len(starts) < 2:
    raise SystemExit(f"fewer than two launches of {a.start}")
# every step: its window and its longest kernels
for j, st_i in enumerate(starts):
    en_i = starts[j + 1] if j + 1 < len(starts) else len(ks)
    top = sorted(ks[st_i:en_i], key=lambda k: k[0] - k[1])[:4]
    print(f"step {j}: window {(ks[en_i - 1][1] - ks[st_i][0]) / 1e6:.3f} ms; longest: " +
          ", ".join(f"{k[2].split('(')[0][-40:]} {(k[1] - k[0]) / 1e3:.0f} us" for k in top))
s = starts[a.which]
e = starts[a.which + 1] if a.which + 1 < len(starts) and a.which != -1 else len(ks)
t0, t1 = ks[s][0], ks[e - 1][1]
print(f"step window {(t1 - t0) / 1e6:.3f} ms, {e - s} kernels")
busy = 0
prev_end = t0
agg = {}
for st, en, nm, sid in ks[s:e]:
    gap = max(0, st - prev_end)
    short = nm.split("(")[0][:70]
    if (en - st) / 1e3 >= a.min_us or gap / 1e3 >= a.min_us:
        print(f"  +{(st - t0) / 1e6:8.3f} ms  dur {(en - st) / 1e3:9.1f} us  gap {gap / 1e3:8.1f} us  s{sid}  {short}")
    agg.setdefault(short, [0, 0.0])
    agg[short][0] += 1
    agg[short][1] += (en - st) / 1e3
    busy += en - st
    prev_end = max(prev_end, en)
print(f"kernel time {busy / 1e6:.3f} ms (sum, overlap counted twice); idle gaps vs window {(t1 - t0 - busy) / 1e6:.3f} ms")
print("per kernel name (count, total us):")
for nm, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"  {c:5d} {t:10.1f}  {nm}")
print(f"HIP calls >= {a.min_us} us in the window:")
hc = {}
for r in rows(a.htrace):
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if st >= t0 and st <= t1:
        fn = r.get("Function", r.get("Operation", "?"))
        hc.setdefault(fn, [0, 0.0])
        hc[fn][0] += 1
        hc[fn][1] += (en - st) / 1e3
        if (en - st) / 1e3 >= a.min_us:
            print(f"  +{(st - t0) / 1e6:8.3f} ms  {(en - st) / 1e3:9.1f} us  {fn}")
print("HIP calls in the window (count, total us):")
for fn, (c, t) in sorted(hc.items(), key=lambda x: -x[1][1])[:15]:
    print(f"  {c:6d} {t:10.1f}  {fn}")
