"""Shorten rocprofv3 kernel_stats.csv names (template noise) for reading; prints the top kernels."""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*>", "<..>", n)
    return n[:90]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f'{short(r["Name"]):92s} calls={r["Calls"]:>7s} avg_ms={float(r["AverageNs"])/1e6:10.4f} total%={float(r["Percentage"]):6.2f}')
