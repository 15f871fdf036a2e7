"""Diagnostic: the sizes the sparse main pass's LDS budget has to hold at config 3 (or the workload given).

Per ion of the search (run_hot_path at ppm 2): the principal window's points (ion_sparse_kernel's CAPC), its
duplicate-candidate points (the side table holds one f64 sum per pixel with >= 2 points), and the flagged points of
the tail windows (the deferred lists: SP_DSEG per wave).  Prints quantiles and the share of ions above each cap.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sm_distributed_amd import engine as E, synthetic as syn

a = sys.argv[1:]
nrows, ncols, pk, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else (500, 500, 2000.0, 20000)
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
flag = ((peaks.hits_sorted >> 31) & 1).to(torch.int64)
cf = torch.zeros(flag.numel() + 1, dtype=torch.int64, device=flag.device)
torch.cumsum(flag, 0, out=cf[1:])
off = dions.win_off
n = (hi - lo)
fl = cf[hi] - cf[lo]
n0 = n[off[:-1]].cpu().numpy()
f0 = fl[off[:-1]].cpu().numpy()
cs = torch.zeros(n.numel() + 1, dtype=torch.int64, device=n.device)
torch.cumsum(fl, 0, out=cs[1:])
ftail = (cs[off[1:]] - cs[off[:-1]] - fl[off[:-1]]).cpu().numpy()
ct = torch.zeros(n.numel() + 1, dtype=torch.int64, device=n.device)
torch.cumsum(n, 0, out=ct[1:])
ntail = (ct[off[1:]] - ct[off[:-1]] - n[off[:-1]]).cpu().numpy()
sparse = (m.flags.cpu().numpy() & 0x40) != 0
q = [0.5, 0.9, 0.99, 0.999, 1.0]
def show(name, x, caps):
    print(f"{name}: mean {x.mean():.1f} quantiles {dict(zip(q, np.quantile(x, q).round(1).tolist()))}; "
          + ", ".join(f"> {c}: {(x > c).mean() * 100:.3f}%" for c in caps), flush=True)
print(f"{len(n0)} ions, {sparse.sum()} on the sparse pass; window points {int(n.sum())}")
show("principal points", n0, [1536, 2048, 2304, 2560])
show("principal flagged points", f0, [64, 128, 168, 336])
show("tail points", ntail, [2048, 4096, 8192])
show("tail flagged points (4 waves' deferred lists)", ftail, [64, 128, 192, 256])
ch = m.chaos.cpu().numpy()
fl = m.flags.cpu().numpy()
print(f"ions with chaos != 0 (some chaos candidate): {(ch[sparse] != 0).mean() * 100:.2f}% of the sparse-pass ions; "
      f"chaos NaN flag: {((fl[sparse] & 4) != 0).mean() * 100:.2f}%")
