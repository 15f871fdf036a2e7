"""Diagnostic: ion-stage time of the normal passes, the forced dense path and the hot-spot clip
(do_preprocessing) on one synthetic workload; max |difference| normal vs forced dense.

usage: time_paths.py [nrows ncols peaks n_sf]   (default config 3: 500 500 2000 20000)
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sm_distributed_amd import engine as E, synthetic as syn, _lib

a = sys.argv[1:]
nrows, ncols, peaks_per, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else (500, 500, 2000.0, 20000)
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, peaks_per, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
L = _lib.lib()
cols = ("chaos", "spatial", "spectral", "msm")


def timed(reps=3, **kw):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = E.ion_metrics(peaks, dions, lo, hi, nlevels=30, **kw)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, r.to_numpy()


t_n, g_n = timed()
print(f"{nrows}x{ncols} P={peaks_per:g} n_sf={n_sf}: {dions.n_ions} ions; normal {t_n:.2f} ms "
      f"(big {int(((g_n['flags'] & 8) != 0).sum())}, dense {int(((g_n['flags'] & 2) != 0).sum())})", flush=True)
L.smg_debug_force_dense(1)
try:
    t_d, g_d = timed()
finally:
    L.smg_debug_force_dense(0)
err = max(float(np.abs(g_n[c] - g_d[c]).max()) for c in cols)
print(f"forced dense {t_d:.2f} ms, max|d| vs normal {err:.1e}, scored set same "
      f"{bool(np.array_equal(g_n['flags'] & 1, g_d['flags'] & 1))}", flush=True)
L.smg_debug_force_dense(2)
try:
    t_p, g_p = timed()
finally:
    L.smg_debug_force_dense(0)
err = max(float(np.abs(g_n[c] - g_p[c]).max()) for c in cols)
print(f"forced pixel-indexed dense {t_p:.2f} ms, max|d| vs normal {err:.1e}, wide ions normal "
      f"{int(((g_n['flags'] & 0x20) != 0).sum())}", flush=True)
t_c, g_c = timed(reps=3, do_preprocessing=True, q=99.0)
fc = g_c["flags"]
print(f"do_preprocessing (q99 clip) {t_c:.2f} ms = {t_c / t_n:.2f}x normal (LDS passes "
      f"{int((((fc & 2) == 0) & ((fc & 1) != 0)).sum())}, wide pass {int(((fc & 0x20) != 0).sum())}, "
      f"pixel-indexed {int((((fc & 2) != 0) & ((fc & 0x20) == 0) & ((fc & 1) != 0)).sum())} ions)", flush=True)
