"""HBM traffic per launch of the ion kernel from two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE) of
scripts/pmc_ion.py, calibrated on its smg_debug_stream_read dispatch (n_points x 8 B read once with the same
8-byte-per-lane access width: MI355X_MICROARCH.md says FETCH_SIZE is exact only for 16-B-per-lane reads and
must be calibrated otherwise).  FETCH_SIZE counts L2 -> fabric requests (Infinity-Cache hits included).

usage: traffic_summary.py FETCH.csv WRITE.csv n_points out.json [kernel-key config alg_bytes]
  kernel-key: ion_pipe_kernel[512] (default) | ion_sparse_kernel | ion_pipe_kernel[1024] | ion_wave_kernel |
              ion_wide_kernel | ion_wide_join_kernel | ion_dense_kernel
"""
import csv, json, re, sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r.get("Kernel_Name") or ""
        m = re.search(r"ion_pipe_kernel<[^,]*, (\d+)", name)
        key = f"ion_pipe_kernel[{m.group(1)}]" if m else ("stream_read" if "stream_read_kernel" in name else None)
        for k in ("ion_sparse_kernel", "ion_wave_kernel", "ion_wide_join_kernel", "ion_wide_kernel", "ion_dense_kernel"):
            if key is None and k in name:
                key = k
        if key:
            acc[key].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
n_points = int(sys.argv[3])
calib_bytes = n_points * 8
scale = calib_bytes / fetch["stream_read"]  # bytes per FETCH_SIZE unit for 8-B-per-lane loads
kern = sys.argv[5] if len(sys.argv) > 5 else "ion_pipe_kernel[512]"
res = {"kernel": kern, "calibration": {"bytes": calib_bytes, "fetch_size": fetch["stream_read"],
                                                          "bytes_per_unit": scale},
       "fetch_size_raw": fetch, "write_size_raw": write,
       "read_bytes": {k: v * scale for k, v in fetch.items()},
       "write_bytes_kb_units": write}
res["traffic_bytes_per_launch"] = res["read_bytes"][kern] + 1024.0 * write.get(kern, 0.0)
if len(sys.argv) > 6:
    res["config"] = sys.argv[6]
if len(sys.argv) > 7:
    res["algorithmic_bytes_12B_per_point"] = float(sys.argv[7])
    res["traffic_over_algorithmic"] = res["traffic_bytes_per_launch"] / float(sys.argv[7])
    res["read_over_algorithmic"] = res["read_bytes"][kern] / float(sys.argv[7])
json.dump(res, open(sys.argv[4], "w"), indent=1)
print(json.dumps(res, indent=1))
