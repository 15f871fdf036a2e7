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
if os.environ.get("C5SHARD"):  # rank 0's shard of the 8-way plan of BASELINE config 5 (scripts/pmc_workload.py c5shard)
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table_both_polarities(40000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 5000, seed=42, device="cuda", ions=ions)
    full = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    plan = D.plan_shards(FormulasSegm.from_ion_table(ions, 2.0), full, 2.0, 8, 0)
    peaks = D.slice_peaks(full, plan)
    del full, mz, hits
    f = plan.formulas
    dions = E.DeviceIons.from_arrays(f.ion_off, f.peak_mz, f.peak_int)
else:
    ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
    peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
L = _lib.lib()
print(L.smg_version().decode() if hasattr(L.smg_version(), "decode") else L.smg_version())
L.smg_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
L.smg_debug_wide_impl(int(os.environ.get("WIDE_IMPL", "1")))
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
if os.environ.get("WIDE_IMPL", "1") == "1" and not CLIP:  # ion_wide_join_kernel's phases
    names = {10: "principal stream+stats", 12: "tail windows", 8: "screen (bitmap walk)", 11: "JH + join stream",
             13: "hits", 14: "candidates exact eL", 9: "kruskal",
             15: "finalize+cleanup+next ion"}
tot = sum(buf[i] for i in names)
for i, nm in names.items():
    print(f"  {nm:20s} {buf[i]/max(nw,1):10.0f} cycles/ion  {100*buf[i]/max(tot,1):5.1f}%")
if buf[0]:
    print(f"  screen calls per ion {buf[0]/max(nw,1):.1f} (per wave), active lanes per call {buf[1]/buf[0]:.1f}, "
          f"screened pixels per ion {buf[1]/max(nw,1):.0f}")
