"""Workload for rocprofv3 --pmc passes: config-3 dataset, one full warm pass, then 2 timed hot-path passes,
plus a 1 GiB device copy as a FETCH_SIZE/WRITE_SIZE calibration dispatch (known bytes, wide loads)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import engine as E, synthetic as syn

ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
for _ in range(3):
    m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
a = torch.ones(1 << 27, dtype=torch.int64, device="cuda")  # 1 GiB
b = torch.empty_like(a)
b.copy_(a)
torch.cuda.synchronize()
print("sum window points", int((hi - lo).sum().item()), "points", peaks.n_points)
