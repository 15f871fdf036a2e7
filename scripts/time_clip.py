"""Diagnostic: ion-stage time without and with the hot-spot clip (do_preprocessing) for the library SMG_LIB names;
max |difference| of the clipped table from the first variant's (gpurun_out/clip_ref.npz).
usage: time_clip.py [nrows ncols peaks n_sf q]   (default 1000 1000 1000 2000 99)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sm_distributed_amd import engine as E, synthetic as syn, _lib

a = sys.argv[1:]
nrows, ncols, pk, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else (1000, 1000, 1000.0, 2000)
q = float(a[4]) if len(a) >= 5 else 99.0
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()


def timed(reps=3, **kw):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = E.ion_metrics(peaks, dions, lo, hi, nlevels=30, **kw)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, r.to_numpy()


t_n, _ = timed()
CFD = int(os.environ.get("CLIP_FORCE_DENSE", "0"))  # the clipped run on the dense path (1: wide pass, 2: pixel kernel)
if CFD:
    _lib.lib().smg_debug_force_dense(CFD)
t_c, g = timed(do_preprocessing=True, q=q)
_lib.lib().smg_debug_force_dense(0)
cols = ("chaos", "spatial", "spectral", "msm")
ref = os.path.join("gpurun_out", "clip_ref.npz")
if os.path.exists(ref):
    r = np.load(ref)
    note = f"max|d| vs first {max(float(np.nanmax(np.abs(g[c] - r[c]))) for c in cols):.1e}"
else:
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(ref, **{c: g[c] for c in cols})
    note = "reference"
print(f"{os.path.basename(_lib.LIB_PATH)} {nrows}x{ncols}: normal {t_n:.2f} ms, clip q{q:g} {t_c:.2f} ms = "
      f"{t_c / t_n:.2f}x ({note}; clipped run forced dense {CFD})", flush=True)
