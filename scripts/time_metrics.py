"""Diagnostic: time the fused ion-metrics launch of whatever libsmg the SMG_LIB env var names (config 3)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import engine as E, synthetic as syn, _lib

ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
ref = m.to_numpy()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
got = m.to_numpy()
import numpy as np
err = max(float(np.nanmax(np.abs(got[c] - ref[c]))) for c in ("chaos", "spatial", "spectral", "msm"))
print(f"{os.path.basename(_lib.LIB_PATH)}: ion_metrics min {min(ts)*1e3:.2f} ms median {sorted(ts)[2]*1e3:.2f} ms "
      f"(self-consistency {err:.1e}, dense {int(((got['flags'] & 2) != 0).sum())})", flush=True)
