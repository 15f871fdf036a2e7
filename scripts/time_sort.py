"""Diagnostic: time flag_duplicates + sort of the config-3 dataset for whatever libsmg SMG_LIB names, and check
the result against a full 31-bit sort of the same library (sorted keys identical, hits a permutation)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import engine as E, synthetic as syn, _lib

ions = syn.make_ion_table(200, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
peaks.flag_duplicates(2.0)
kb = peaks.key_bits()
tf = []
for _ in range(6):  # repeated passes (the flag-state path a step takes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    peaks.flag_duplicates(2.0)
    torch.cuda.synchronize()
    tf.append(time.perf_counter() - t0)
print(f"{os.path.basename(_lib.LIB_PATH)}: flag_duplicates min {min(tf[1:])*1e3:.2f} ms median "
      f"{sorted(tf[1:])[2]*1e3:.2f} ms", flush=True)
ts = []
for _ in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    peaks.sort()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
ks, hs = peaks.mz_sorted.clone(), peaks.hits_sorted.clone()
peaks.sort_key_bits = 31
peaks.sort()
same_keys = bool(torch.equal(ks, peaks.mz_sorted))
perm = bool(torch.equal(torch.sort(hs)[0], torch.sort(peaks.hits_sorted)[0]))
print(f"{os.path.basename(_lib.LIB_PATH)}: sort key_bits={kb} min {min(ts[1:])*1e3:.2f} ms median "
      f"{sorted(ts[1:])[2]*1e3:.2f} ms; keys identical to 31-bit sort {same_keys}, hits permutation {perm}",
      flush=True)
