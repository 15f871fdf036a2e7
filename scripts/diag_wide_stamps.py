"""Diagnostic: per-phase wall cycles of the wide dense pass (libsmg_stamps.so, -DSMG_STAMPS) on a workload whose
windows exceed the LDS passes.  usage: diag_wide_stamps.py [nrows ncols peaks n_sf]  (default 1000 1000 5000 2000)
CLIP=q: with the hot-spot clip at q (do_preprocessing; its passes fall in "pass2+stats" and "tail windows")."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sm_distributed_amd import _lib
_lib.LIB_PATH = os.environ.get("SMG_LIB") or _lib.LIB_PATH.replace("libsmg.so", "libsmg_stamps.so")
import torch
from sm_distributed_amd import engine as E, synthetic as syn

a = sys.argv[1:]
nrows, ncols, pk, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else (1000, 1000, 5000.0, 2000)
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
L = _lib.lib()
print(L.smg_version().decode() if hasattr(L.smg_version(), "decode") else L.smg_version())
L.smg_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
L.smg_debug_stamps(buf, 16)
t0 = time.perf_counter()
CLIP = os.environ.get("CLIP")
kw = dict(q=float(CLIP), do_preprocessing=True) if CLIP else {}
m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30, **kw)
torch.cuda.synchronize()
L.smg_debug_stamps(buf, 16)
t0 = time.perf_counter()
m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30, **kw)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
L.smg_debug_stamps(buf, 16)
f = m.flags.cpu().numpy()
nw = int(((f & 0x20) != 0).sum())
w = (hi - lo).cpu().numpy()
print(f"{nrows}x{ncols} P={pk:g} clip {CLIP}: {dions.n_ions} ions, launch {dt*1e3:.1f} ms, {nw} wide ions, "
      f"mean window points {w.mean():.0f}")
names = {10: "pass1+rank", 11: "pass2+stats", 12: "tail windows", 13: "levels", 8: "screen: dilate",
         9: "screen: erode+list", 14: "candidates exact eL", 15: "kruskal+finalize+fetch"}
tot = sum(buf[i] for i in names)
for i, nm in names.items():
    print(f"  {nm:20s} {buf[i]/max(nw,1):10.0f} cycles/ion  {100*buf[i]/max(tot,1):5.1f}%")
