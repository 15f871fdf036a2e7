"""Breakdown of one drop-in API step at config 3 (diagnostic): wall time of each phase with a device
synchronisation after it, so host and device costs show separately.  Usage: python scripts/time_api.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sm_distributed_amd import engine as E, synthetic as syn
from sm_distributed_amd.dataset import ResidentDataset
from sm_distributed_amd import formula_imager_segm as FIS
from sm_distributed_amd import formula_img_validator as FIV
from sm_distributed_amd.formulas import FormulasSegm

ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions)
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
formulas = FormulasSegm.from_ion_table(ions)
df = formulas.get_sf_peak_df()
dds = ResidentDataset(peaks)
conf = {"image_generation": {"ppm": 2.0, "nlevels": 30, "q": 99, "do_preprocessing": False}}
sync = torch.cuda.synchronize
T = {}
def tick(name, t0):
    sync(); t = time.perf_counter(); T.setdefault(name, []).append((t - t0) * 1e3); return t
for it in range(6):
    sync(); t = time.perf_counter(); t_all = t
    peaks.flag_duplicates(2.0); t = tick("flag", t)
    peaks.sort(); t = tick("sort", t)
    peaks.prefix_sums(); t = tick("scan", t)
    codes, cats = FIS._adduct_codes(df["adduct"]); t = tick("host: adduct codes", t)
    keys, dions, K = FIS.device_layout(df, peaks.device); t = tick("device_layout (host+device)", t)
    lo, hi = E.window_bounds(peaks, dions, 2.0); t = tick("window_bounds", t)
    ims = FIS.IonImageSet(peaks, keys, dions, K, lo, hi, dims, 2.0); t = tick("IonImageSet", t)
    keep, m = FIV._metrics_device_rows(ims, formulas.get_sf_peak_ints(), conf["image_generation"]); t = tick("metrics rows (align + kernel)", t)
    idx = torch.nonzero(keep).flatten()
    vals = torch.stack([m.chaos[idx], m.spatial[idx], m.spectral[idx], m.msm[idx]], 1).cpu().numpy(); t = tick("D2H rows", t)
    import pandas as pd
    out = pd.DataFrame(vals, index=ims.ion_keys.multi_index(idx.cpu().numpy()), columns=["chaos", "spatial", "spectral", "msm"]); t = tick("DataFrame", t)
    tick("TOTAL (serialised)", t_all)
    sync(); t = time.perf_counter()
    ims = FIS.compute_sf_images(None, dds, df, 2.0); t = tick("API compute_sf_images", t)
    r = FIV.sf_image_metrics(ims, None, formulas, dds, conf); t = tick("API sf_image_metrics", t)
for k, v in T.items():
    print(f"{k:40s} {np.median(v[1:]):9.2f} ms")
