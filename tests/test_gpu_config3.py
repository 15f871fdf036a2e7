"""Config 3 (the headline workload) at full size on the device, checked against the oracle (GPU only).

500x500 px, Poisson(2000) centroids per spectrum (~5e8 points), 20,000 synthetic formulas x (+H, +Na, +K +
distinct decoys) ~ 0.98M ions, ppm 2, nlevels 30 -- the dataset bench.py times, generated in HBM with the same
seeds.  The oracle cannot image 5e8 points for 1M ions, so the check is a seeded sample of 576 ions drawn
across the WHOLE m/z range (512 uniformly from every ion + 64 ions with planted signal): every data point of
the sample's windows is selected from the resident dataset (by m/z, with a margin), and the oracle
(oracle/cpu_baseline.py = formula_imager_segm.py:66-92 + formula_img_validator.py:72-84) images and scores
the sample from those points.  Bars: window sizes identical (searchsorted f64 semantics on the same points),
scored / unscored status identical, chaos / spatial / spectral / msm within 1e-5 absolute.  Size-independent
properties cover the rest: the sort is a permutation of the resident points and every scored ion has a
window with points.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

METRIC_ATOL = 1e-5


@pytest.mark.timeout(600)
def test_config3_full_size_sample_matches_oracle():
    import torch
    from oracle import cpu_baseline as CB
    from oracle import msm_oracle as O
    from sm_distributed_amd import engine as E
    from sm_distributed_amd import synthetic as syn

    ppm, nlevels = 2.0, 30
    ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions,
                                                  plant_fraction=0.02, plant_seed=45)
    assert dims == (500, 500) and info["n_points"] > 4.9e8 and ions.n_ions > 9.5e5
    peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
    m, lo, hi = E.run_hot_path(peaks, dions, ppm, nlevels)
    torch.cuda.synchronize()
    got = m.to_numpy()
    lo_h, hi_h = lo.cpu().numpy(), hi.cpu().numpy()

    # size-independent properties over every ion
    n = info["n_points"]
    assert (lo_h <= hi_h).all() and (hi_h <= n).all()
    assert bool((peaks.mz_sorted[1:] >= peaks.mz_sorted[:-1]).all())
    cnt = hi_h - lo_h
    has = np.add.reduceat(cnt, ions.win_off[:-1]) > 0
    np.testing.assert_array_equal((got["flags"] & 1) != 0, has)
    assert np.isfinite(got["msm"]).all()

    # the sample: uniform over every ion (so over the whole m/z range) + planted-signal target ions
    rng = np.random.default_rng(2024)
    pick = rng.choice(ions.n_ions, size=512, replace=False)
    prng = np.random.default_rng(45)  # make_dataset_torch's planting draw
    tgt = np.nonzero(np.isin(ions.adducts, list(ions.target_adducts)))[0]
    planted = prng.choice(tgt, size=max(1, int(round(0.02 * len(tgt)))), replace=False)
    pick = np.unique(np.concatenate([pick, planted[:64]]))
    first = ions.peak_mz[ions.win_off[:-1]][pick]
    assert first.min() < 250 and first.max() > 850, "sample must span the m/z range"
    wins = np.concatenate([np.arange(ions.win_off[i], ions.win_off[i + 1]) for i in pick])
    lower, upper = O.window_bounds(ions.peak_mz[wins], ppm)
    b_pix, b_mz, b_int = CB.select_window_points(peaks.mz, peaks.hits, lower, upper)
    del peaks, mz, hits, lo, hi, m
    for k in list(E._ws_cache):
        E._ws_cache.pop(k)
    torch.cuda.empty_cache()

    # window sizes: searchsorted over the selected points == the device's windows over all points
    seg = np.sort(b_mz).astype(np.float64)
    olo = np.searchsorted(seg, lower, "left")
    ohi = np.searchsorted(seg, upper, "right")
    np.testing.assert_array_equal(ohi - olo, cnt[wins])

    tasks = [(int(i), ions.peak_mz[ions.win_off[i]:ions.win_off[i + 1]].copy(),
              ions.peak_int[ions.win_off[i]:ions.win_off[i + 1]].copy()) for i in pick]
    workers = CB.default_workers(cap=16)
    rows, wall, _ = CB.run_pool(b_pix, b_mz, b_int, dims, ppm, nlevels, tasks, workers)
    scored = {r[0] for r in rows}
    assert scored == {int(i) for i in pick if has[i]}
    planted_scored = 0
    for ion_id, c, s, p in rows:
        for col, v in (("chaos", c), ("spatial", s), ("spectral", p), ("msm", c * s * p)):
            assert abs(got[col][ion_id] - v) <= METRIC_ATOL, (ion_id, col, got[col][ion_id], v)
        planted_scored += int(c * s * p > 0)
    assert planted_scored >= 10, "the sample must contain ions with real signal"
    print(f"config 3: {len(rows)} sampled ions checked ({planted_scored} with msm > 0), oracle wall {wall:.1f}s "
          f"on {workers} workers, {b_mz.size:,} window points")
