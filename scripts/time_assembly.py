"""Diagnostic: the pieces of the rank-0 table assembly (distributed.rows_to_frame) at config-3 size, each timed
with a device synchronisation: row scatter + compaction, gathers, pinned D2H, MultiIndex, DataFrame."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pandas as pd
import torch
from sm_distributed_amd import distributed as D, synthetic as syn
from sm_distributed_amd.formulas import FormulasSegm
from sm_distributed_amd.formula_imager_segm import IonKeys, METRIC_COLUMNS

ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
f = FormulasSegm.from_ion_table(ions, 2.0)
keys = f.ion_sf.astype(np.int64) * max(len(f.adducts), 1) + f.ion_adduct_code
gk = IonKeys(keys, f.adducts)
n = len(gk)
W = 8
rng = np.random.default_rng(0)
perm = rng.permutation(n)
n_max = (n + W - 1) // W
tab = np.full((W * n_max, 5), -1.0)
for r in range(W):
    part = np.sort(perm[r::W])
    keep = rng.random(len(part)) < 0.96
    tab[r * n_max:r * n_max + len(part), 0] = np.where(keep, part, -1)
    tab[r * n_max:r * n_max + len(part), 1:] = rng.random((len(part), 4))
t = torch.from_numpy(tab).cuda()
sync = torch.cuda.synchronize
for rep in range(4):
    T = {}
    sync(); t0 = time.perf_counter()
    gi = t[:, 0].long()
    gi = torch.where(gi >= 0, gi, torch.full_like(gi, n))
    row = torch.full((n + 1,), -1, dtype=torch.int64, device=t.device)
    row[gi] = torch.arange(t.shape[0], device=t.device)
    idx = torch.nonzero(row[:n] >= 0).flatten()
    sync(); T["scatter+nonzero"] = time.perf_counter() - t0; t0 = time.perf_counter()
    cols = t[row[idx], 1:5].T
    sfc, adc = gk.codes_dev(t.device)
    parts = (cols, sfc[idx], adc[idx])
    sync(); T["gathers"] = time.perf_counter() - t0; t0 = time.perf_counter()
    host = [torch.empty(x.shape, dtype=x.dtype, pin_memory=True) for x in parts]
    T["pinned alloc"] = time.perf_counter() - t0; t0 = time.perf_counter()
    for h, x in zip(host, parts):
        h.copy_(x, non_blocking=True)
    sync(); T["D2H"] = time.perf_counter() - t0; t0 = time.perf_counter()
    c, c_sf, c_ad = (h.numpy() for h in host)
    mi = gk.multi_index_from_codes(c_sf, c_ad)
    T["MultiIndex"] = time.perf_counter() - t0; t0 = time.perf_counter()
    df = pd.DataFrame(c.T, index=mi, columns=METRIC_COLUMNS, copy=False)
    T["DataFrame"] = time.perf_counter() - t0; t0 = time.perf_counter()
    sync(); t1 = time.perf_counter()
    df2 = D.rows_to_frame(t, gk)
    sync(); T["rows_to_frame total"] = time.perf_counter() - t1
print("  ".join(f"{k} {v*1e3:.3f} ms" for k, v in T.items()), len(df))
