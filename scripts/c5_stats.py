"""Diagnostic: what the wide pass holds per ion on one rank's shard of config 5 (the c5shard workload of
scripts/pmc_workload.py: rank 0 of the 8-way plan), for a seeded sample of ions:
  * principal points / principal pixels (np: the per-pixel arrays the wide pass writes to its slot),
  * tail points and tail hits on principal pixels (the x gathers),
  * the chaos screen's candidates E = erode_box(dilate_cross(principal presence)) (border 0) and the distinct pixels
    of their 5x5 neighbourhoods (what an exact eL reads),
from the sorted hits with torch ops on the device."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import torch.nn.functional as Fn
from sm_distributed_amd import distributed as D, engine as E, synthetic as syn
from sm_distributed_amd.formulas import FormulasSegm

ions = syn.make_ion_table_both_polarities(40000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 5000, seed=42, device="cuda", ions=ions)
full = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
formulas = FormulasSegm.from_ion_table(ions, 2.0)
plan = D.plan_shards(formulas, full, 2.0, 8, 0)
peaks = D.slice_peaks(full, plan)
f = plan.formulas
dions = E.DeviceIons.from_arrays(f.ion_off, f.peak_mz, f.peak_int)
peaks.flag_and_sort(2.0)
lo, hi = E.window_bounds(peaks, dions, 2.0)
torch.cuda.synchronize()
nr, nc = dims
pix = (peaks.hits_sorted & 0x7FFFFFFF).to(torch.int64)
off = dions.win_off.cpu().numpy()
lo_h, hi_h = lo.cpu().numpy(), hi.cpu().numpy()
rng = np.random.default_rng(5)
pick = rng.choice(dions.n_ions, size=min(300, dions.n_ions), replace=False)
cross = torch.tensor([[0, 1, 0], [1, 1, 1], [0, 1, 0]], dtype=torch.float32, device="cuda").view(1, 1, 3, 3)
rows = []
for i in pick:
    w0, w1 = off[i], off[i + 1]
    a, b = lo_h[w0], hi_h[w0]
    if b <= a:
        continue
    P = torch.zeros(nr * nc, dtype=torch.float32, device="cuda")
    P[pix[a:b]] = 1.0
    npx_ = int(P.sum().item())
    img = P.view(1, 1, nr, nc)
    dil = (Fn.conv2d(img, cross, padding=1) > 0).float()
    ero = -Fn.max_pool2d(-dil, 3, stride=1, padding=1)          # min over the 3x3 box, border 0 outside:
    ero = ero * (Fn.conv2d(torch.ones_like(dil), torch.ones(1, 1, 3, 3, device="cuda"), padding=1) == 9).float()
    ncand = int(ero.sum().item())
    nb = int((Fn.max_pool2d(ero, 5, stride=1, padding=2) * img).sum().item())  # principal pixels within 2 of a candidate
    tp = torch.cat([pix[lo_h[w]:hi_h[w]] for w in range(w0 + 1, w1)]) if w1 > w0 + 1 else pix[:0]
    th = int(P[tp].sum().item()) if tp.numel() else 0
    rows.append((b - a, npx_, int(tp.numel()), th, ncand, nb))
r = np.array(rows, dtype=np.float64)
names = ["principal points", "principal pixels", "tail points", "tail hits on principal pixels", "chaos candidates",
         "principal pixels within 2 of a candidate"]
print(f"{len(r)} sampled ions of {dions.n_ions} (rank 0 of the 8-way plan of config 5), {peaks.n_points:,} slice points")
for j, nm in enumerate(names):
    q = np.quantile(r[:, j], [0.5, 0.9, 0.99, 1.0])
    print(f"{nm}: mean {r[:, j].mean():.0f} median {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f}", flush=True)
print(f"ions with a chaos candidate: {(r[:, 4] > 0).mean() * 100:.1f}%")
