"""Diagnostic: per-phase wall cycles of the dense ion kernel (libsmg_stamps.so, -DSMG_STAMPS) with every ion
forced onto the dense path (smg_debug_force_dense).  usage: diag_dense_stamps.py [nrows ncols peaks n_sf]"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sm_distributed_amd import _lib
_lib.LIB_PATH = os.environ.get("SMG_LIB") or _lib.LIB_PATH.replace("libsmg.so", "libsmg_stamps.so")
import torch
from sm_distributed_amd import engine as E, synthetic as syn

a = sys.argv[1:]
nrows, ncols, pk, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else (500, 500, 2000.0, 20000)
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
L = _lib.lib()
L.smg_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
for force in (0, 1):
    L.smg_debug_force_dense(force)
    L.smg_debug_stamps(buf, 16)
    t0 = time.perf_counter()
    m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    L.smg_debug_stamps(buf, 16)
    f = m.flags.cpu().numpy()
    nd = int(((f & 2) != 0).sum())
    names = ["fetch+fresh+flags", "principal+stats", "tail windows", "levels+candidates", "kruskal",
             "finalize+clean+next"]
    tot = sum(buf[10 + i] for i in range(6))
    print(f"{nrows}x{ncols} force_dense={force}: launch {dt*1e3:.1f} ms, {nd} dense ions; "
          f"dense cycles/ion {tot/max(nd,1):.0f}")
    for i, nm in enumerate(names):
        print(f"  {nm:22s} {buf[10+i]/max(nd,1):10.0f} cycles/ion  {100*buf[10+i]/max(tot,1):5.1f}%")
L.smg_debug_force_dense(0)
