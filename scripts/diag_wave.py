"""Diagnostic: one parity case through the main pass twice -- the legacy 512-thread LDS kernel and the wave
kernel -- and the per-ion differences of their outputs, with the wave kernel's trace of each differing ion
(library built with -DSMG_WAVE_TRACE: SMG_LIB=.../wtrace.so python3 scripts/diag_wave.py [case])."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from sm_distributed_amd import _lib
from sm_distributed_amd import engine as E
from tests.parity_cases import make_case

name = sys.argv[1] if len(sys.argv) > 1 else "basic"
ds, ions, ppm, kw = make_case(name)
pm, dims = ds.pixel_map_dims()
L = _lib.lib()
raw = ctypes.CDLL(_lib.LIB_PATH)
res = {}
for which in (1, 0):
    assert L.smg_debug_main_kernel(which) == 0
    peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
    m, lo, hi = E.run_hot_path(peaks, dions, ppm, **kw)
    torch.cuda.synchronize()
    res[which] = m.to_numpy()
    print(f"main kernel {which}: done", flush=True)
L.smg_debug_main_kernel(0)
if hasattr(raw, "smg_debug_wave_check"):
    ck = (ctypes.c_ulonglong * 8)()
    assert raw.smg_debug_wave_check(ck) == 0
    print(f"wave checks: first failed code {ck[0]} value {ck[1]} (as signed {ctypes.c_longlong(ck[1]).value}) "
          f"at position {ck[3]}; failures {ck[2]}; ions scored {ck[4]}", flush=True)
tr = (ctypes.c_longlong * (8192 * 8))()
assert raw.smg_debug_wave_trace(tr, 8192) == 0
tr = np.frombuffer(tr, dtype=np.int64).reshape(8192, 8)
by_ion = {int(r[1]): r for r in tr if r[2] > 0}
old, new = res[1], res[0]
n = ions.n_ions
print(f"case {name}: {n} ions, dims {dims}, traced {len(by_ion)}")
bad = [i for i in range(n) if old["flags"][i] != new["flags"][i] or
       any(abs(old[c][i] - new[c][i]) > 1e-9 for c in ("chaos", "spatial", "spectral", "msm"))]
print(f"{len(bad)} ions differ")
for i in bad[:25]:
    t = by_ion.get(i)
    print(i, "K", ions.win_off[i + 1] - ions.win_off[i], "flags", hex(old["flags"][i]), hex(new["flags"][i]),
          "chaos %.6f %.6f spatial %.6f %.6f spectral %.6f %.6f" % (old["chaos"][i], new["chaos"][i], old["spatial"][i],
                                                                   new["spatial"][i], old["spectral"][i], new["spectral"][i]),
          "trace", None if t is None else t.tolist())
