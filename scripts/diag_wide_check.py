"""Diagnostic: rank 0's config-5 shard (tests/test_gpu_config5.py's path) through the wide pass built with
-DSMG_WIDE_CHECK (scripts/build_variant.sh wchk -DSMG_WIDE_CHECK): prints the first failed index check of the
wide pass (code, value), the failure count and the ions it scored.  Usage: SMG_LIB=.../wchk.so python3 this."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
assert os.environ.get("SMG_LIB", "").endswith("wchk.so"), "run with SMG_LIB pointing at the check build"
import torch

from sm_distributed_amd import _lib
from sm_distributed_amd import distributed as D
from sm_distributed_amd import engine as E
from sm_distributed_amd import synthetic as syn
from sm_distributed_amd.formulas import FormulasSegm

chk = ctypes.CDLL(_lib.LIB_PATH).smg_debug_wide_check
out = (ctypes.c_ulonglong * 4)()
ions = syn.make_ion_table_both_polarities(40000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 5000.0, seed=42, device="cuda", ions=ions,
                                              plant_fraction=0.02, plant_seed=45)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
formulas = FormulasSegm.from_ion_table(ions, 2.0)
conf = {"image_generation": {"ppm": 2.0, "nlevels": 30, "q": 99, "do_preprocessing": False}}
for rank in [int(r) for r in (sys.argv[1:] or ["0"])]:
    plan = D.plan_shards(formulas, peaks, 2.0, 8, rank)
    rows, _ = D._device_rows(plan, peaks, conf)
    torch.cuda.synchronize()
    assert chk(out) == 0
    print(f"rank {rank}: first failed check code {out[0]} value {out[1]} failures {out[2]} ions seen {out[3]}; "
          f"rows {rows.shape[0]}", flush=True)
