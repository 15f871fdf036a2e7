"""Workload for rocprofv3 --pmc passes over the ion kernel alone: config-3 dataset, one warm hot-path pass,
then two ion_metrics launches (the library is whatever SMG_LIB names, else libsmg.so)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import engine as E, synthetic as syn

ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
for _ in range(2):
    m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
torch.cuda.synchronize()
print("ok")
# calibration dispatch for the HBM-traffic counters: one read of the sorted hits (known byte count) with the
# ion kernel's access width; scripts/traffic_summary.py converts FETCH_SIZE with it
import ctypes
from sm_distributed_amd import _lib
out = torch.zeros(4096, dtype=torch.int64, device="cuda")
rc = _lib.lib().smg_debug_stream_read(ctypes.c_void_p(peaks.hits_sorted.data_ptr()), peaks.n_points,
                                      ctypes.c_void_p(out.data_ptr()), 4096, None)
assert rc == 0
torch.cuda.synchronize()
print("calibration bytes", peaks.n_points * 8)
