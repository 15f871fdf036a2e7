"""Diagnostic: per-phase wall cycles of the wave main pass on the config-3 workload (library built with
-DSMG_WAVE_STAMPS: SMG_LIB=.../wvst.so python3 scripts/diag_wave_stamps.py).  Prints the cycles per scored ion
(one wave per ion) of each phase."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from sm_distributed_amd import _lib, engine as E, synthetic as syn

raw = ctypes.CDLL(_lib.LIB_PATH)
ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
st = (ctypes.c_ulonglong * 8)()
raw.smg_debug_wave_stamps(st)  # reset
t0 = time.perf_counter()
m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
assert raw.smg_debug_wave_stamps(st) == 0
fl = m.flags.cpu().numpy()
wave = int((((fl & 1) != 0) & ((fl & (2 | 8 | 0x10)) == 0)).sum())
names = ["principal+directory", "chaos screen", "eL+Kruskal", "next desc/ticket", "tail stream",
         "parked+flagged", "issue+finalize", "skipped ions"]
tot = sum(st)
print(f"ion_metrics {dt*1e3:.1f} ms; wave-scored ions {wave}; total stamped cycles {tot:.3e}")
for i, n in enumerate(names):
    print(f"  {n:22s} {st[i] / max(wave, 1):10.0f} cycles/ion  {100.0 * st[i] / max(tot, 1):5.1f}%")
