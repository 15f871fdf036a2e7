"""Window search timing and output at config 3 (or argv nrows ncols peaks n_sf) for the library SMG_LIB points to:
best-of-20 HIP-event time of smg_window_bounds over the sorted resident peaks, and (argv OUT) lo/hi saved for an
A/B comparison between builds (also: every window in the ion order and in m/z order, and with NaN / negative
m/z windows mixed in)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sm_distributed_amd import engine as E, synthetic as syn

out = sys.argv[1] if len(sys.argv) > 1 else None
ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions,
                                              plant_fraction=0.02, plant_seed=45)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
peaks.flag_and_sort(2.0)
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int, device=peaks.device)
for _ in range(3):
    lo, hi = E.window_bounds(peaks, dions, 2.0)
ts = []
for _ in range(20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    lo, hi = E.window_bounds(peaks, dions, 2.0)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(f"{os.path.basename(os.environ.get('SMG_LIB', 'libsmg.so'))}: window search best {min(ts):.3f} ms "
      f"median {np.median(ts):.3f} ms over {dions.n_windows:,} windows, {peaks.n_points:,} points")
# the odd cases: ion order (no m/z order), NaN and negative m/z mixed in
pm = dions.peak_mz.clone()
pm[::97] = float("nan")
pm[5::101] = -1.0
odd = E.DeviceIons(win_off=dions.win_off, peak_mz=pm, theor=None, win_order=None, ion_order=dions.ion_order,
                   n_ions=dions.n_ions, n_windows=dions.n_windows, max_k=dions.max_k)
lo2, hi2 = E.window_bounds(peaks, odd, 2.0)
if out:
    np.savez(out, lo=lo.cpu().numpy(), hi=hi.cpu().numpy(), lo2=lo2.cpu().numpy(), hi2=hi2.cpu().numpy())
