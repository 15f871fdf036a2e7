"""Diagnostic: one parity case on the device with a forced path, checked against the oracle.
usage: diag_clip_case.py CASE [force_dense 0|1|2] [force_two_level 0|1]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.parity_cases import make_case, oracle_run
from sm_distributed_amd import engine as E, _lib

name = sys.argv[1]
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
two = int(sys.argv[3]) if len(sys.argv) > 3 else 0
ds, ions, ppm, kw = make_case(name)
imgs, df = oracle_run(ds, ions, ppm, **kw)
L = _lib.lib()
L.smg_debug_force_dense(mode)
L.smg_debug_force_two_level(two)
pm, dims = ds.pixel_map_dims()
peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
print(f"{name} dense={mode} two={two}: {dions.n_ions} ions, dims {dims}", flush=True)
m, lo, hi = E.run_hot_path(peaks, dions, ppm, 30, **kw)
torch.cuda.synchronize()
m = m.to_numpy()
has = (m["flags"] & 1) != 0
idx = {k: i for i, k in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))}
rows = np.array([idx[k] for k in df.index.tolist()], dtype=np.int64)
err = max(float(np.abs(df[c].to_numpy() - m[c][rows]).max(initial=0.0)) for c in ("chaos", "spatial", "spectral", "msm"))
f = m["flags"][has]
cols = ("chaos", "spatial", "spectral", "msm")
e = np.max([np.abs(df[c].to_numpy() - m[c][rows]) for c in cols], axis=0)
K = np.diff(ions.win_off)
for j in np.argsort(-e)[:6]:
    if e[j] > 1e-5:
        i = rows[j]
        print(f"  ion {i}: err {e[j]:.2e} flags {m['flags'][i]:#x} K {K[i]} | " +
              " ".join(f"{c} {df[c].to_numpy()[j]:.6f}/{m[c][i]:.6f}" for c in cols), flush=True)
print(f"  ok: max err {err:.1e}; LDS {int(((f & 2) == 0).sum())} (big {int(((f & 8) != 0).sum())}), wide "
      f"{int(((f & 0x20) != 0).sum())}, pixel {int((((f & 2) != 0) & ((f & 0x20) == 0)).sum())}", flush=True)
