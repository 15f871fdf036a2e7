"""Diagnostic: per-phase wall cycles of the sparse main pass (ion_sparse_kernel) at config 3 (libsmg_stamps.so, built
with `make -C sm_distributed_amd/csrc stamps`: -DSMG_STAMPS).  Cycles are summed over workgroups and divided by the
ions the pass scored, i.e. wall cycles per ion per workgroup (four workgroups share a CU)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sm_distributed_amd import _lib
if not os.environ.get("SMG_LIB"):
    _lib.LIB_PATH = _lib.LIB_PATH.replace("libsmg.so", "libsmg_stamps.so")
import torch
from sm_distributed_amd import engine as E, synthetic as syn

a = sys.argv[1:]
nrows, ncols, pk, n_sf = (int(a[0]), int(a[1]), float(a[2]), int(a[3])) if len(a) >= 4 else (500, 500, 2000.0, 20000)
ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
L = _lib.lib()
buf = (ctypes.c_ulonglong * 16)()
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
torch.cuda.synchronize()
L.smg_debug_sparse_stamps(buf, 16)
t0 = time.perf_counter()
m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
L.smg_debug_sparse_stamps(buf, 16)
names = ["top: ticket, descriptor checks", "build: filter, bucket counts, directory", "entries, values, side sums",
         "ticket barrier, stats, levels", "tail stream", "issue next ion, tail barrier", "duplicate table",
         "(unused)", "chaos screen (bands)", "exact eL", "kruskal", "record, clear, loop barrier"]
extra = {12: "(tail stream: in counted waits)", 13: "(tail stream: parked events resolved)",
         14: "(tail stream: events handled in place)", 15: "(tail stream: refills issued)"}
f = m.flags.cpu().numpy()
n = int(((f & 0x41) == 0x41).sum())
tot = sum(buf[i] for i in range(len(names)))
print(os.path.basename(_lib.LIB_PATH), f"{nrows}x{ncols} px, Poisson({pk:g}), {n_sf} formulas")
print(f"ion_metrics {dt*1e3:.1f} ms; sparse-pass ions {n} of {dions.n_ions}; sum cycles/ion/workgroup {tot/max(n,1):.0f}")
for i, nm in enumerate(names):
    print(f"  {nm:40s} {buf[i]/max(n,1):10.0f} cycles/ion  {100*buf[i]/max(tot,1):5.1f}%")
for i, nm in extra.items():
    print(f"  {nm:40s} {buf[i]/max(n,1):10.0f} cycles/ion")
print("big-pass ions", int(((f & 8) != 0).sum()), "dense ions", int(((f & 2) != 0).sum()),
      "chaos-NaN ions", int(((f & 4) != 0).sum()))
