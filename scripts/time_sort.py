"""Diagnostic: time the config-3 dataset's flag + sort stage three ways -- the flag pass then rocPRIM's onesweep
sort, the flag pass then the hand-written sort, and the fused flag_and_sort -- and check that all three give the
same sorted arrays.  Usage: python3 scripts/time_sort.py [nrows ncols lambda]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from sm_distributed_amd import engine as E
from sm_distributed_amd import synthetic as syn
from sm_distributed_amd._lib import lib

nr, nc, lam = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (500, 500, 2000.0)
ions = syn.make_ion_table(200, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nr, nc, lam, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
print(f"{peaks.n_points:,} points, key_bits {peaks.key_bits()}, spectra sorted {peaks.spectra_sorted()}", flush=True)


def timed(fn, reps=8):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[1:])
    return ts[0] * 1e3, ts[len(ts) // 2] * 1e3


def two_calls():
    peaks.flag_duplicates(2.0)
    peaks.sort()


out = {}
for name, impl, fn in [("flag pass + rocPRIM sort", 0, two_calls), ("flag pass + hand-written sort", 1, two_calls),
                       ("rocPRIM sort alone", 0, peaks.sort), ("hand-written sort alone", 1, peaks.sort),
                       ("fused flag_and_sort", 1, lambda: peaks.flag_and_sort(2.0)),
                       ("hand-written look-back sort alone", 2, peaks.sort),
                       ("fused flag_and_sort, look-back", 2, lambda: peaks.flag_and_sort(2.0))]:
    lib().smg_debug_sort_impl(impl)
    lo, med = timed(fn)
    if "alone" not in name:
        out[name] = (peaks.mz_sorted.clone(), peaks.hits_sorted.clone())
    print(f"{name:32s} min {lo:7.2f} ms  median {med:7.2f} ms", flush=True)
lib().smg_debug_sort_impl(1)
ref = out["flag pass + rocPRIM sort"]
for k, (a, b) in out.items():
    print(f"{k:32s} identical to rocPRIM path: keys {torch.equal(a, ref[0])} hits {torch.equal(b, ref[1])}",
          flush=True)
