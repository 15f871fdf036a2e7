"""Diagnostic: time the fused ion-metrics launch of whatever libsmg the SMG_LIB env var names (config 3).

The first variant run in a GPU session saves its outputs (gpurun_out/ab_ref.npz); later variants report their
max |difference| from it, so an A/B session checks that a faster variant still computes the same table.
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sm_distributed_amd import engine as E, synthetic as syn, _lib

a = sys.argv[1:]  # optional workload: nrows ncols peaks n_sf (default config 3)
nrows, ncols, pk, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else (500, 500, 2000.0, 20000)
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
if os.environ.get("SMG_FORCE_TWO"):  # diagnostic: the two-level LDS passes for every image size
    _lib.lib().smg_debug_force_two_level(1)
if os.environ.get("SMG_MAIN_KERNEL"):  # A/B: 0 = ion_pipe_kernel<512>, 1 = ion_sparse_kernel
    _lib.lib().smg_debug_main_kernel(int(os.environ["SMG_MAIN_KERNEL"]))
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
got = m.to_numpy()
cols = ("chaos", "spatial", "spectral", "msm")
ref_path = os.path.join("gpurun_out", "ab_ref.npz")
if os.path.exists(ref_path):
    ref = np.load(ref_path)
    err = max(float(np.nanmax(np.abs(got[c] - ref[c]))) for c in cols)
    hits_same = bool(np.array_equal(got["flags"] & 1, ref["flags"] & 1))
    note = f"max|d| vs first variant {err:.1e}, scored set same {hits_same}"
else:
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(ref_path, **{c: got[c] for c in cols + ("flags",)})
    note = "reference variant"
fl = got["flags"]
tag = os.path.basename(_lib.LIB_PATH) + (f" main_kernel={os.environ['SMG_MAIN_KERNEL']}" if os.environ.get("SMG_MAIN_KERNEL") else "")
print(f"{tag}: ion_metrics min {min(ts)*1e3:.2f} ms median {sorted(ts)[2]*1e3:.2f} ms "
      f"({note}; big {int(((fl & 8) != 0).sum())} dense {int(((fl & 2) != 0).sum())})", flush=True)
