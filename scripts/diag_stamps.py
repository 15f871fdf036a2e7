"""Diagnostic: per-phase wall cycles of the LDS ion kernel (libsmg_stamps.so, built with -DSMG_STAMPS)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sm_distributed_amd import _lib
if not os.environ.get("SMG_LIB"):
    _lib.LIB_PATH = _lib.LIB_PATH.replace("libsmg.so", "libsmg_stamps.so")
import torch
from sm_distributed_amd import engine as E, synthetic as syn

a = sys.argv[1:]  # n_sf, or nrows ncols peaks n_sf
nrows, ncols, pk, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else \
    (500, 500, 2000.0, int(a[0]) if a else 20000)
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
L = _lib.lib()
L.smg_debug_main_kernel(0)  # ion_pipe_kernel (the sparse pass has its own stamps: diag_sparse_stamps.py)
L.smg_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
print("flagged fraction", float(((peaks.hits >> 31) & 1).float().mean()))
torch.cuda.synchronize()
L.smg_debug_stamps(buf, 16)
t0 = time.perf_counter()
m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
L.smg_debug_stamps(buf, 16)
names = ["p0 load+zero", "p1 ticket wait+barrier", "p2-3 stats+levels", "d duplicate table", "p4a screen",
         "p4a exact eL", "p4b kruskal", "record+loop", "p5 tail windows", "tail barrier+stats", "issue next+clear",
         "p1 bitmap/prefix/vals"]
n = dions.n_ions
tot = sum(buf[i] for i in range(len(names)))
print(os.path.basename(_lib.LIB_PATH))
print(f"metrics launch {dt*1e3:.1f} ms for {n} ions; sum cycles/ion {tot/n:.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:24s} {buf[i]/n:10.0f} cycles/ion  {100*buf[i]/max(tot,1):5.1f}%")
f = m.flags.cpu().numpy()
print("dense ions", int(((f & 2) != 0).sum()), "chaos-NaN ions", int(((f & 4) != 0).sum()))
