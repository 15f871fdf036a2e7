"""Where the cold-cache search's extra host time goes (config 3): one warm search, then the PeakInts device cache
dropped (as bench.py's cold_cache_step_ms does) and the next search run under cProfile; prints the top
cumulative-time entries and the warm/cold wall times."""
import cProfile, os, pstats, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import engine as E, synthetic as syn
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
for _ in range(3):
    step()
torch.cuda.synchronize()
t = time.perf_counter(); step(); torch.cuda.synchronize(); warm = (time.perf_counter() - t) * 1e3
formulas.get_sf_peak_ints().__dict__.pop("_dev_cache", None)
torch.cuda.synchronize()
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable(); step(); torch.cuda.synchronize(); pr.disable()
cold = (time.perf_counter() - t) * 1e3
print(f"warm {warm:.1f} ms, cold (profiled) {cold:.1f} ms")
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
