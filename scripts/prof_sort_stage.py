"""Diagnostic: the config-3 flag + sort + scan stage alone (DevicePeaks.flag_and_sort + prefix_sums, as the
search runs it), 10 times after a warm-up, for rocprofv3 --kernel-trace --stats: per-kernel times of the stage.
Also prints the stage's wall time per repetition (events around it)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import engine as E, synthetic as syn

ions = syn.make_ion_table(int(os.environ.get("N_SF", "200")), seed=43, decoy_seed=44)  # (bench.py: 20000)
PLANT = float(os.environ.get("PLANT", "0"))  # bench.py's dataset plants 2 % of the formulas' peaks (PLANT=0.02)
kw = dict(plant_fraction=PLANT, plant_seed=45) if PLANT > 0 else {}
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions, **kw)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
for _ in range(2):
    peaks.flag_and_sort(2.0)
    peaks.prefix_sums()
torch.cuda.synchronize()
ts = []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    peaks.flag_and_sort(2.0)
    peaks.prefix_sums()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
print(f"plant {PLANT}: {peaks.n_points:,} points: flag+sort+scan min {ts[0]:.3f} median {ts[len(ts)//2]:.3f} ms", flush=True)
