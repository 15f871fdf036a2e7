"""A/B of library builds at config 3 (SMG_LIB): main-pass HIP-event times over 12 API steps and the full
metrics table, saved to argv[1] (.npz) so that builds can be compared bit for bit (scripts/gpu_ab_libs.sh)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sm_distributed_amd import _lib, engine as E, synthetic as syn
from sm_distributed_amd.dataset import ResidentDataset
from sm_distributed_amd.formula_imager_segm import compute_sf_images
from sm_distributed_amd.formula_img_validator import sf_image_metrics
from sm_distributed_amd.formulas import FormulasSegm

ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions,
                                              plant_fraction=0.02, plant_seed=45)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
formulas = FormulasSegm.from_ion_table(ions, 2.0)
conf = {"image_generation": {"ppm": 2.0, "nlevels": 30, "q": 99, "do_preprocessing": False}}
dds = ResidentDataset(peaks)
sdf = formulas.get_sf_peak_df()
step = lambda: sf_image_metrics(compute_sf_images(None, dds, sdf, 2.0), None, formulas, dds, conf)
L = _lib.lib()
for _ in range(3):
    df = step()
L.smg_debug_time_main_pass(1)
L.smg_debug_main_pass_times(None, 0, ctypes.byref(ctypes.c_int32(0)))
for _ in range(12):
    df = step()
torch.cuda.synchronize()
buf = (ctypes.c_double * 64)()
n = ctypes.c_int32(0)
L.smg_debug_main_pass_times(buf, 64, ctypes.byref(n))
L.smg_debug_time_main_pass(0)
t = np.array(buf[:n.value])
np.savez(sys.argv[1], vals=df.to_numpy())
print(f"{os.path.basename(os.environ.get('SMG_LIB', 'libsmg.so'))}: main pass median {np.median(t):.2f} ms "
      f"min {t.min():.2f} ({n.value} launches), {len(df)} rows", flush=True)
