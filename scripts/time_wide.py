"""A/B timing of the wide pass (whatever SMG_LIB names): a 1000x1000 / Poisson(5000) workload whose principal windows
exceed the LDS passes; prints the median ion_metrics time over 3 launches.  usage: time_wide.py [n_sf]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from sm_distributed_amd import _lib, engine as E, synthetic as syn

n_sf = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 5000, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
ts.sort()
f = m.flags.cpu().numpy()
print(f"{os.path.basename(_lib.LIB_PATH)}: ion_metrics median {ts[1]*1e3:.1f} ms (min {ts[0]*1e3:.1f}), "
      f"{int(((f & 0x20) != 0).sum())} wide ions of {dions.n_ions}, chaos sum {float(m.chaos.sum()):.6f}")
