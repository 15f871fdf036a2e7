"""Diagnostic: which of two library variants is right where they disagree (config 3, no planting).

  SMG_LIB=variants/a.so python3 scripts/ab_oracle.py save a     -> /tmp/abo_a.npz (the ion table's metrics)
  python3 scripts/ab_oracle.py check a b                         -> the ions where a and b differ by > 1e-6, up to
                                                                   48 of them scored by the oracle
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sm_distributed_amd import engine as E
from sm_distributed_amd import synthetic as syn

COLS = ("chaos", "spatial", "spectral", "msm")
ppm, nlevels = 2.0, 30


def main():
    ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions)
    peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    out = os.path.join("/tmp", "abo_%s.npz")  # large: kept off gpurun_out/
    if sys.argv[1] == "save":
        dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
        m, lo, hi = E.run_hot_path(peaks, dions, ppm, nlevels)
        torch.cuda.synchronize()
        got = m.to_numpy()
        np.savez(out % sys.argv[2], **{c: got[c] for c in COLS + ("flags",)})
        print("saved", sys.argv[2], flush=True)
        return

    from oracle import cpu_baseline as CB
    from oracle import msm_oracle as O

    a, b = (np.load(out % n) for n in sys.argv[2:4])
    d = np.zeros(ions.n_ions)
    for c in COLS:
        d = np.maximum(d, np.nan_to_num(np.abs(a[c] - b[c]), nan=9.0))
    diff = np.nonzero(d > 1e-6)[0]
    print(f"{diff.size} ions differ (max {d.max():.3g}); flags differ on {(a['flags'] != b['flags']).sum()}", flush=True)
    pick = diff[:48]
    if pick.size == 0:
        return
    wins = np.concatenate([np.arange(ions.win_off[i], ions.win_off[i + 1]) for i in pick])
    lower, upper = O.window_bounds(ions.peak_mz[wins], ppm)
    print("selecting window points", flush=True)
    b_pix, b_mz, b_int = CB.select_window_points(peaks.mz, peaks.hits, lower, upper)
    print(f"{b_mz.size:,} window points; oracle on {len(pick)} ions", flush=True)
    tasks = [(int(i), ions.peak_mz[ions.win_off[i]:ions.win_off[i + 1]].copy(),
              ions.peak_int[ions.win_off[i]:ions.win_off[i + 1]].copy()) for i in pick]
    rows, wall, _ = CB.run_pool(b_pix, b_mz, b_int, dims, ppm, nlevels, tasks, CB.default_workers(cap=16))
    wa = wb = 0
    for ion_id, c, s, p in rows:
        ref = {"chaos": c, "spatial": s, "spectral": p, "msm": c * s * p}
        ea = max(abs(a[k][ion_id] - ref[k]) for k in COLS)
        eb = max(abs(b[k][ion_id] - ref[k]) for k in COLS)
        wa += ea > 1e-5
        wb += eb > 1e-5
        print(f"ion {ion_id}: oracle chaos {c:.6f} | {sys.argv[2]} {a['chaos'][ion_id]:.6f} (err {ea:.1e}) | "
              f"{sys.argv[3]} {b['chaos'][ion_id]:.6f} (err {eb:.1e}) flags {a['flags'][ion_id]} {b['flags'][ion_id]}")
    print(f"wrong vs oracle: {sys.argv[2]} {wa}, {sys.argv[3]} {wb} of {len(rows)}")


if __name__ == "__main__":  # the oracle pool spawns workers that import this file
    main()
