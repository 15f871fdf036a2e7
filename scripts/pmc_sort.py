"""PMC workload: the config-3 dataset's fused flag + sort twice, after the 8-byte-per-lane calibration stream
(smg_debug_stream_read over the hits) that scripts/gpu_pmc_sort.sh scales FETCH_SIZE by."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from sm_distributed_amd import engine as E
from sm_distributed_amd import synthetic as syn
from sm_distributed_amd._lib import lib

ions = syn.make_ion_table(200, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
peaks.key_bits(), peaks.spectra_sorted()
out = torch.zeros(4096, dtype=torch.int64, device="cuda")
n = peaks.n_points
lib().smg_debug_stream_read(ctypes.c_void_p(hits.data_ptr()), n, ctypes.c_void_p(out.data_ptr()), 4096, None)
torch.cuda.synchronize()
print(f"calibration bytes {n * 8}", flush=True)
for _ in range(2):
    peaks.flag_and_sort(2.0)
torch.cuda.synchronize()
print("done", flush=True)
