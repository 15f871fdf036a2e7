"""Workload for rocprofv3 --pmc passes (one counter set per run, scripts/gpu_pmc2.sh).
  c3    : config 3 (500x500, Poisson(2000), 20,000 formulas): the main LDS pass ion_pipe_kernel<512>
  dense : 1000x1000, Poisson(2100), 1,000 formulas: most principal windows exceed the LDS passes -> dense path
  c5    : 1000x1000, Poisson(5000), 2,000 formulas (config-5-like windows): the wide dense pass ion_wide_kernel
One warm hot-path pass, then two ion_metrics launches, then a calibration read of the sorted hits (known bytes,
the kernels' 8-byte-per-lane access width) for FETCH_SIZE."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import _lib, engine as E, synthetic as syn

which = sys.argv[1] if len(sys.argv) > 1 else "c3"
if which == "c5shard":
    # bench.py --config 5 --shard-of 8 --shard-rank 0: one rank's shard of BASELINE config 5, two metric launches
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table_both_polarities(40000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 5000, seed=42, device="cuda", ions=ions)
    full = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    formulas = FormulasSegm.from_ion_table(ions, 2.0)
    plan = D.plan_shards(formulas, full, 2.0, 8, 0)
    peaks = D.slice_peaks(full, plan)
    f = plan.formulas
    dions = E.DeviceIons.from_arrays(f.ion_off, f.peak_mz, f.peak_int)
    if os.environ.get("SMG_WIDE_IMPL"):  # 1 = ion_wide_join_kernel (default), 0 = ion_wide_kernel
        _lib.lib().smg_debug_wide_impl(int(os.environ["SMG_WIDE_IMPL"]))
    m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
    for _ in range(2):
        m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
    torch.cuda.synchronize()
    fl = m.flags.cpu()
    print(which, "points", peaks.n_points, "ions", dions.n_ions, "sum window points", int((hi - lo).sum().item()),
          "wide ions", int(((fl & 0x20) != 0).sum()))
    out = torch.zeros(4096, dtype=torch.int64, device="cuda")
    assert _lib.lib().smg_debug_stream_read(ctypes.c_void_p(peaks.hits_sorted.data_ptr()), peaks.n_points,
                                            ctypes.c_void_p(out.data_ptr()), 4096, None) == 0
    torch.cuda.synchronize()
    print("calibration bytes", peaks.n_points * 8)
    sys.exit(0)
if which == "c3":
    ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000, seed=42, device="cuda", ions=ions)
elif which == "c5":
    ions = syn.make_ion_table(2000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 5000, seed=42, device="cuda", ions=ions)
else:
    ions = syn.make_ion_table(1000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 2100, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
if os.environ.get("SMG_MAIN_KERNEL"):  # 0 = ion_pipe_kernel<512>, 1 = ion_sparse_kernel (default)
    _lib.lib().smg_debug_main_kernel(int(os.environ["SMG_MAIN_KERNEL"]))
m, lo, hi = E.run_hot_path(peaks, dions, 2.0, 30)
for _ in range(2):
    m = E.ion_metrics(peaks, dions, lo, hi, nlevels=30)
torch.cuda.synchronize()
f = m.flags.cpu()
print(which, "points", peaks.n_points, "ions", dions.n_ions, "sum window points", int((hi - lo).sum().item()),
      "dense ions", int(((f & 2) != 0).sum()), "big ions", int(((f & 8) != 0).sum()))
out = torch.zeros(4096, dtype=torch.int64, device="cuda")
assert _lib.lib().smg_debug_stream_read(ctypes.c_void_p(peaks.hits_sorted.data_ptr()), peaks.n_points,
                                        ctypes.c_void_p(out.data_ptr()), 4096, None) == 0
torch.cuda.synchronize()
print("calibration bytes", peaks.n_points * 8)
