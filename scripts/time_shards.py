"""Per-rank critical path of the sharded (multi-GPU) step, measured on ONE GPU: every rank's shard of a
W-way plan (config 3 by default) is scored in turn with the product code (distributed._device_rows), broken into
slice copy, compute_sf_images and sf_image_metrics rows, plus the rank-0 assembly (rows_to_frame) of all ranks'
rows.  One search alone takes ~ max over ranks + gather + assembly; back to back (bench.py) the other ranks start
the next search while rank 0 assembles, so the re-cut gives rank 0 that much less (rebalance's head_seconds) and
a step takes ~ max(rank 0 + assembly, the other ranks) + gather.

usage: time_shards.py [W=8] [nrows ncols peaks n_sf]
CONFIG=5: BASELINE config 5 (1000x1000 px, Poisson(5000), 40k formulas x 6 adducts in both polarities); every rank
also gets a roofline per pass (12 B per window point of the ions the pass scored over its HIP-event time)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import ctypes
from sm_distributed_amd import _lib, distributed as D, engine as E, synthetic as syn
from sm_distributed_amd.dataset import ResidentDataset
from sm_distributed_amd.formula_imager_segm import compute_sf_images
from sm_distributed_amd.formula_img_validator import _metrics_device_rows, sf_image_metrics
from sm_distributed_amd.formulas import FormulasSegm

a = sys.argv[1:]
W = int(a[0]) if a else 8
nrows, ncols, pk, n_sf = (int(a[1]), int(a[2]), float(a[3]), int(a[4])) if len(a) >= 5 else (500, 500, 2000.0, 20000)
ppm = 2.0
if os.environ.get("WIDE_IMPL"):  # 1 = ion_wide_join_kernel (default), 0 = ion_wide_kernel (A/B)
    _lib.lib().smg_debug_wide_impl(int(os.environ["WIDE_IMPL"]))
CONFIG5 = os.environ.get("CONFIG") == "5"
if CONFIG5:
    nrows, ncols, pk, n_sf = 1000, 1000, 5000.0, 40000
    ions = syn.make_ion_table_both_polarities(n_sf, seed=43, decoy_seed=44)
else:
    ions = syn.make_ion_table(n_sf, seed=43, decoy_seed=44)
mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, pk, seed=42, device="cuda", ions=ions,
                                              plant_fraction=0.02, plant_seed=45)  # bench.py defaults
peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
formulas = FormulasSegm.from_ion_table(ions, ppm)
conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
sync = torch.cuda.synchronize


def timed(f, reps=3):
    best, out = 1e9, None
    for _ in range(reps):
        sync()
        t0 = time.perf_counter()
        out = f()
        sync()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3, out


# single-GPU API step for reference (SKIP_T1=1: skip it; the efficiency is then not printed)
dds = ResidentDataset(peaks)
sdf = formulas.get_sf_peak_df()
SKIP_T1 = bool(os.environ.get("SKIP_T1"))
if SKIP_T1:
    t1, df1 = float("nan"), None
else:
    t1, df1 = timed(lambda: sf_image_metrics(compute_sf_images(None, dds, sdf, ppm), None, formulas, dds, conf),
                    reps=2 if CONFIG5 else 3)
    print(f"1 GPU API step {t1:.2f} ms, {len(df1)} rows, {peaks.n_points:,} points, {formulas.n_ions:,} ions",
          flush=True)
    peaks.mz_sorted = peaks.hits_sorted = peaks.cum = None  # the slices need the HBM at config 5
    E._ws_cache.clear()
    torch.cuda.empty_cache()

ONLY = int(os.environ.get("ONLY_RANK", "-1"))


def run_ranks(plans, tag):
  rows_all, worst, times = [], 0.0, []
  for r, plan in enumerate(plans):
      if ONLY >= 0 and r != ONLY:
          continue
      t_sl, sl = timed(lambda: D.slice_peaks(peaks, plan, cache=False))
      sds = ResidentDataset(sl)
      t_img, ims = timed(lambda: compute_sf_images(None, sds, plan.sf_peak_df, ppm))
      L = _lib.lib()
      L.smg_debug_main_pass_times(None, 0, ctypes.byref(ctypes.c_int32(0)))
      L.smg_debug_time_main_pass(1)
      t_met, (_, mets) = timed(lambda: _metrics_device_rows(ims, plan.formulas.get_sf_peak_ints(),
                                                             conf["image_generation"]))
      L.smg_debug_time_main_pass(0)
      buf = (ctypes.c_double * 64)()
      pbuf = (ctypes.c_int32 * 64)()
      nt = ctypes.c_int32(0)
      L.smg_debug_pass_times(pbuf, buf, 64, ctypes.byref(nt))
      by = {}
      for i in range(min(nt.value, 64)):
          by.setdefault(int(pbuf[i]), []).append(float(buf[i]))
      t_main = min(by.get(_lib.SMG_PASS_MAIN, [float("nan")]))
      # per pass: best launch time and 12 B per window point of the ions it scored
      fl = mets.flags.cpu().numpy().astype(np.int64)
      cs = torch.zeros(ims.lo.numel() + 1, dtype=torch.int64, device=ims.lo.device)
      torch.cumsum(ims.hi - ims.lo, 0, out=cs[1:])
      wo = ims.ions_dev.win_off
      ipts = (cs[wo[1:]] - cs[wo[:-1]]).cpu().numpy()
      pas = np.full(len(fl), _lib.SMG_PASS_MAIN)
      pas[(fl & _lib.SMG_ION_BIG) != 0] = _lib.SMG_PASS_BIG
      pas[(fl & _lib.SMG_ION_DENSE) != 0] = _lib.SMG_PASS_DENSE
      pas[(fl & _lib.SMG_ION_WIDE) != 0] = _lib.SMG_PASS_WIDE
      has = (fl & _lib.SMG_ION_HAS_HITS) != 0
      roof = []
      for p_, ts in sorted(by.items()):
          if p_ == _lib.SMG_PASS_DESC:
              roof.append(f"{_lib.PASS_NAMES.get(p_, p_)} {min(ts):.2f} ms")
              continue
          n_p = int((has & (pas == p_)).sum())
          pts = int(ipts[has & (pas == p_)].sum())
          t = min(ts)
          frac = 12.0 * pts / (t * 1e-3) / 8e12 if t > 0 and pts else 0.0
          roof.append(f"{_lib.PASS_NAMES.get(p_, p_)} {t:.2f} ms {n_p:,} ions {pts:,} window pts -> {frac:.3f} of 8 TB/s")
      print(f"  rank {r} passes: " + "; ".join(roof), flush=True)
      t_all, (rows, _) = timed(lambda: D._device_rows(plan, peaks, conf))
      rows_all.append(rows)
      hist, edges = D.mz_histogram(peaks.mz)
      wpts = float(((D.ion_costs(plan.formulas.ion_off, plan.formulas.peak_mz, ppm, hist, edges) - D.C_ION)
                    / D.C_WINDOW_POINT).sum())
      print(f"FIT rank={r} n_ions={plan.formulas.n_ions} wpts={wpts:.0f} slice={sl.n_points} t_rows={t_all:.3f} "
            f"t_slice={t_sl:.3f} t_img={t_img:.3f} t_met={t_met:.3f} t_main={t_main:.3f}", flush=True)
      worst = max(worst, t_all)
      print(f"[{tag}] rank {r}/{W}: {plan.formulas.n_ions:,} ions, slice {sl.n_points:,} pts [{plan.mz_lo:.2f}, {plan.mz_hi:.2f}] "
            f"est {plan.est_cost[r]*1e3:.2f} ms | slice {t_sl:.2f} + images {t_img:.2f} + metrics {t_met:.2f} "
            f"(main kernel {t_main:.2f}); "
            f"_device_rows {t_all:.2f} ms (the rank's slice cached, as on the rank between searches)", flush=True)
      times.append(t_all * 1e-3)
  return rows_all, worst, times


def table_of(rows_all):
    n_max = max(x.shape[0] for x in rows_all)
    table = torch.full((W * n_max, 5), -1.0, dtype=torch.float64, device="cuda")
    for r, x in enumerate(rows_all):
        table[r * n_max:r * n_max + x.shape[0]] = x
    return table, n_max


plans = [D.plan_shards(formulas, peaks, ppm, W, r) for r in range(W)]
rows_all, worst, times = run_ranks(plans, "cost model")
if ONLY >= 0:
    sys.exit(0)
worst0 = worst
# rank 0's assembly (the steady-state form, placement cached), then the plan re-cut from the measured per-rank
# times with it as rank 0's head (what bench.py does after its warm-up: one all_gather of W + 1 floats)
table, _ = table_of(rows_all)
D.rows_to_frame(table, plans[0].global_keys)
t_head, _ = timed(lambda: D.rows_to_frame(table, plans[0].global_keys))
NO_HEAD = bool(os.environ.get("NO_HEAD"))
print(f"rank-0 assembly of the cost-model table {t_head:.2f} ms (head cut {'off' if NO_HEAD else 'on'})", flush=True)
# re-cut until the ranks (rank 0 with its assembly) agree within 3 %, at most ROUNDS times (bench.py does the same)
for it in range(int(os.environ.get("ROUNDS", "3"))):
    loads = [times[0] + (0.0 if NO_HEAD else t_head * 1e-3)] + times[1:]
    spread = max(loads) / min(loads) - 1.0
    print(f"re-cut round {it}: spread {spread * 100:.1f} %", flush=True)
    if spread <= 0.03:
        break
    plans = [D.rebalance(p, formulas, peaks, times, head_seconds=0.0 if NO_HEAD else t_head * 1e-3) for p in plans]
    print("rebalanced counts", plans[0].counts, flush=True)
    rows_all, worst, times = run_ranks(plans, f"rebalanced {it + 1}")
print(f"max rank: cost model {worst0:.2f} ms, rebalanced {worst:.2f} ms", flush=True)
table, n_max = table_of(rows_all)
plan0 = plans[0]
t_asm, df = timed(lambda: D.rows_to_frame(table, plan0.global_keys))
# assembly breakdown
def asm_parts():
    out = {}
    t0 = time.perf_counter()
    t = table
    n = len(plan0.global_keys)
    valid = t[:, 0] >= 0
    sel = t[valid]
    gi = sel[:, 0].long()
    full = torch.zeros(4, n, dtype=t.dtype, device=t.device)
    full[:, gi] = sel[:, 1:5].T
    has = torch.zeros(n, dtype=torch.bool, device=t.device)
    has[gi] = True
    idx = torch.nonzero(has).flatten()
    sync(); out["device scatter+nonzero"] = time.perf_counter() - t0; t0 = time.perf_counter()
    g = full[:, idx]
    sync(); out["gather cols"] = time.perf_counter() - t0; t0 = time.perf_counter()
    cols = g.cpu().numpy()
    out["D2H cols"] = time.perf_counter() - t0; t0 = time.perf_counter()
    ih = idx.cpu().numpy()
    out["D2H idx"] = time.perf_counter() - t0; t0 = time.perf_counter()
    mi = plan0.global_keys.multi_index(ih)
    out["multi_index"] = time.perf_counter() - t0; t0 = time.perf_counter()
    import pandas as pd
    pd.DataFrame(cols.T, index=mi, columns=["chaos", "spatial", "spectral", "msm"], copy=False)
    out["DataFrame"] = time.perf_counter() - t0
    return out
for _ in range(2):
    parts = asm_parts()
print("assembly parts (ms): " + ", ".join(f"{k} {v*1e3:.2f}" for k, v in parts.items()))
same = df1 is not None and df.index.equals(df1.index) and np.allclose(df.to_numpy(), df1.to_numpy(), rtol=0,
                                                                       atol=1e-12)
print(f"assembly (rank 0) {t_asm:.2f} ms; table identical to 1 GPU: {same}")
# the gather's payload: W blocks of n_max rows x 5 f64 into rank 0 (RCCL gather).  One GPU cannot run the
# collective; what it can time is the payload's own device copy (HBM to HBM, a floor) -- the xGMI leg is estimated
# from it: W-1 blocks over W-1 point-to-point links into rank 0 at once, ~50 GB/s achieved per link, plus RCCL's
# launch latency (~50 us).  bench.py --gpus N prints every rank's measured gather median on the driver's node.
payload = W * n_max * 5 * 8
src = torch.empty(W * n_max * 5, dtype=torch.float64, device="cuda")
dst = torch.empty_like(src)
t_copy, _ = timed(lambda: dst.copy_(src), reps=5)
gather_est = (n_max * 40) / 50e9 * 1e3 + 0.05
print(f"gather payload {payload / 1e6:.2f} MB ({W} x {n_max:,} rows x 40 B): device copy of it {t_copy:.3f} ms; "
      f"xGMI estimate {gather_est:.3f} ms")
est1 = worst + gather_est + t_asm
others = max(times[1:]) * 1e3
est = max(times[0] * 1e3 + t_asm, others) + gather_est
print(f"one search alone {est1:.2f} ms = max rank {worst:.2f} + gather ~{gather_est:.2f} + assembly {t_asm:.2f}; "
      f"strong-scaling efficiency {t1 / (W * est1):.2f}")
print(f"estimated {W}-GPU step (back to back) {est:.2f} ms = max(rank 0 {times[0] * 1e3:.2f} + assembly "
      f"{t_asm:.2f}, other ranks {others:.2f}) + gather ~{gather_est:.2f}; strong-scaling efficiency "
      f"{t1 / (W * est):.2f}")
print("(both efficiencies assume every rank runs at the clock it had alone on this GPU; eight busy GPUs of one "
      "node may run slower)")
