"""Shared seeded parity cases: the same inputs feed the oracle (CPU) and the device path (GPU)."""
from __future__ import annotations

import numpy as np
import pandas as pd

from sm_distributed_amd import synthetic as syn


def subset_ions(ions: syn.IonTable, idx) -> syn.IonTable:
    idx = np.asarray(idx)
    K = np.diff(ions.win_off)[idx]
    off = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(K, out=off[1:])
    sel = np.concatenate([np.arange(ions.win_off[i], ions.win_off[i + 1]) for i in idx]) if len(idx) else np.zeros(0, np.int64)
    return syn.IonTable(sf_ids=ions.sf_ids[idx], adducts=ions.adducts[idx], win_off=off,
                        peak_mz=ions.peak_mz[sel], peak_int=ions.peak_int[sel],
                        target_adducts=ions.target_adducts, decoy_sample_size=ions.decoy_sample_size, td=ions.td)


def sf_peak_df(ions: syn.IonTable) -> pd.DataFrame:
    """FormulasSegm.get_sf_peak_df (formulas_segm.py:56-63): one row per theoretical peak, sorted by mz."""
    K = np.diff(ions.win_off)
    owner = np.repeat(np.arange(ions.n_ions), K)
    peak_i = np.arange(ions.n_windows) - np.repeat(ions.win_off[:-1], K)
    df = pd.DataFrame({"sf_id": ions.sf_ids[owner], "adduct": ions.adducts[owner], "peak_i": peak_i,
                       "mz": ions.peak_mz})
    return df.sort_values(by="mz", kind="stable")


def sf_peak_ints(ions: syn.IonTable) -> dict:
    return {(s, a): ions.peak_int[ions.win_off[i]:ions.win_off[i + 1]].tolist()
            for i, (s, a) in enumerate(zip(ions.sf_ids, ions.adducts))}


def add_duplicates(ds: syn.SpectraSet, frac: float, seed: int) -> syn.SpectraSet:
    """Duplicate a fraction of points inside their own spectrum at m/z*(1+1e-7): same-window duplicate pixels."""
    rng = np.random.default_rng(seed)
    sp_of = np.repeat(np.arange(ds.n_spectra), np.diff(ds.sp_off))
    pick = rng.random(ds.n_points) < frac
    mz = np.concatenate([ds.mz, (ds.mz[pick].astype(np.float64) * (1 + 1e-7)).astype(np.float32)])
    ints = np.concatenate([ds.ints, (ds.ints[pick] * rng.uniform(0.5, 2.0, pick.sum())).astype(np.float32)])
    sp = np.concatenate([sp_of, sp_of[pick]])
    order = np.lexsort((mz, sp))
    sp, mz, ints = sp[order], mz[order], ints[order]
    off = np.zeros(ds.n_spectra + 1, np.int64)
    np.cumsum(np.bincount(sp, minlength=ds.n_spectra), out=off[1:])
    return syn.SpectraSet(sp_off=off, mz=mz, ints=ints, coords=ds.coords)


def boundary_ions(ds: syn.SpectraSet, ppm: float, n: int, seed: int) -> syn.IonTable:
    """Ions whose windows have a data point exactly on the f64 lower or upper bound (inclusive window)."""
    rng = np.random.default_rng(seed)
    xs = ds.mz[rng.choice(ds.n_points, size=2 * n, replace=False)].astype(np.float64)
    mzs = []
    for j, x in enumerate(xs):
        want_lower = j % 2 == 0
        M = x / (1 - ppm * 1e-6) if want_lower else x / (1 + ppm * 1e-6)
        found = None
        for _ in range(2000):
            d = M * ppm * 1e-6
            b = (M - d) if want_lower else (M + d)
            if b == x:
                found = M
                break
            M = np.nextafter(M, np.inf if b < x else -np.inf)
        if found is not None:
            mzs.append(found)
        if len(mzs) >= n:
            break
    mzs = np.array(mzs)
    k = 4
    win_off = np.arange(len(mzs) + 1, dtype=np.int64) * k
    peak_mz = (mzs[:, None] + np.arange(k)[None, :] * syn.ISOTOPE_SPACING).ravel()
    peak_int = np.tile(np.array([100.0, 40.0, 12.0, 3.0]), len(mzs))
    return syn.IonTable(sf_ids=np.arange(len(mzs), dtype=np.int64) + 900000,
                        adducts=np.array(['+H'] * len(mzs), dtype=object), win_off=win_off, peak_mz=peak_mz,
                        peak_int=peak_int, td=(np.zeros(0), np.zeros(0), np.zeros(0)))


def make_case(name: str):
    """Returns (spectra, ions, ppm, kwargs) for a named parity case."""
    if name == "basic":
        ions = syn.make_ion_table(30, seed=1, decoy_seed=2)
        ds = syn.make_dataset_np(32, 32, 500, seed=3, ions=ions, plant_fraction=0.3, plant_seed=4)
        return ds, ions, 20.0, {}
    if name == "zeros_rect":
        ions = syn.make_ion_table(20, seed=11, decoy_seed=12)
        ds = syn.make_dataset_np(24, 40, 400, seed=13, ions=ions, plant_fraction=0.4, plant_seed=14,
                                 blob_sigma=(1.0, 4.0), zero_fraction=0.2)
        return ds, ions, 30.0, {}
    if name == "dups":
        ions = syn.make_ion_table(20, seed=21, decoy_seed=22)
        ds = syn.make_dataset_np(30, 30, 600, seed=23, ions=ions, plant_fraction=0.4, plant_seed=24)
        return add_duplicates(ds, 0.2, 25), ions, 25.0, {}
    if name == "row":
        ions = syn.make_ion_table(15, seed=31, decoy_seed=32)
        ds = syn.make_dataset_np(1, 300, 800, seed=33, ions=ions, plant_fraction=0.5, plant_seed=34)
        return ds, ions, 40.0, {}
    if name == "column":
        ions = syn.make_ion_table(15, seed=41, decoy_seed=42)
        ds = syn.make_dataset_np(200, 1, 800, seed=43, ions=ions, plant_fraction=0.5, plant_seed=44)
        return ds, ions, 40.0, {}
    if name == "row_border1":
        ds, ions, ppm, _ = make_case("row")
        return ds, ions, ppm, {"erosion_border": 1}
    if name == "conn8_border1":
        ds, ions, ppm, _ = make_case("basic")
        return ds, ions, ppm, {"connectivity": 8, "erosion_border": 1}
    if name == "nlevels":
        ds, ions, ppm, _ = make_case("zeros_rect")
        return ds, ions, ppm, {"nlevels": 7}
    if name == "nlevels1":
        ds, ions, ppm, _ = make_case("basic")
        return ds, ions, ppm, {"nlevels": 1}
    if name == "big_window":   # principal window > LDS capacity -> dense path
        ions = syn.make_ion_table(6, seed=51, decoy_seed=52)
        ds = syn.make_dataset_np(80, 80, 60, seed=53, ions=ions, plant_fraction=1.0, plant_seed=54,
                                 blob_sigma=(150.0, 200.0))
        return ds, ions, 10.0, {}
    if name == "huge_window":  # principal window > big-ion LDS capacity (8192 points) -> dense path
        ions = syn.make_ion_table(4, seed=81, decoy_seed=82)
        ds = syn.make_dataset_np(105, 105, 20, seed=83, ions=ions, plant_fraction=1.0, plant_seed=84,
                                 blob_sigma=(300.0, 400.0))
        return add_duplicates(ds, 0.02, 85), ions, 10.0, {}
    if name == "large_image":  # > 2^18 pixels -> dense path for every ion
        full = syn.make_ion_table(2, seed=61, decoy_seed=62)
        tgt = np.nonzero(np.isin(full.adducts, list(full.target_adducts)))[0][:4]
        ions = subset_ions(full, np.concatenate([tgt, [0, 1]]))
        ds = syn.make_dataset_np(520, 520, 3, seed=63, ions=ions, plant_fraction=1.0, plant_seed=64,
                                 blob_sigma=(3.0, 8.0))
        return ds, ions, 50.0, {}
    if name == "xl_image":     # 1.32M pixels: the dense path's presence bitmap no longer fits the LDS (global)
        full = syn.make_ion_table(2, seed=121, decoy_seed=122)
        tgt = np.nonzero(np.isin(full.adducts, list(full.target_adducts)))[0][:3]
        ions = subset_ions(full, np.concatenate([tgt, [0]]))
        ds = syn.make_dataset_np(1200, 1100, 1, seed=123, ions=ions, plant_fraction=1.0, plant_seed=124,
                                 blob_sigma=(4.0, 9.0))
        return ds, ions, 50.0, {}
    if name == "large_blobs":  # > 2^18 pixels with big blobs: two-level main / big-ion passes, chaos with many
        full = syn.make_ion_table(4, seed=111, decoy_seed=112)  # candidates, olist from the set (nnz > OL_MAX)
        tgt = np.nonzero(np.isin(full.adducts, list(full.target_adducts)))[0][:8]
        dec = np.nonzero(~np.isin(full.adducts, list(full.target_adducts)))[0][:4]
        ions = subset_ions(full, np.concatenate([tgt, dec]))
        ds = syn.make_dataset_np(600, 600, 10, seed=113, ions=ions, plant_fraction=1.0, plant_seed=114,
                                 blob_sigma=(14.0, 30.0))
        return add_duplicates(ds, 0.01, 115), ions, 20.0, {}
    if name == "long_tail":    # tails of several register chunks (chunk refills, window changes inside chunks)
        full = syn.make_ion_table(12, seed=91, decoy_seed=92)
        ions = subset_ions(full, np.arange(0, full.n_ions, 6))
        ds = syn.make_dataset_np(128, 256, 250, seed=93, ions=ions, plant_fraction=0.5, plant_seed=94)
        return ds, ions, 100.0, {}
    if name == "dups_heavy":   # duplicate lists overflow the main pass (-> big-ion pass -> dense path)
        ds, ions, ppm, _ = make_case("long_tail")
        return add_duplicates(ds, 0.3, 95), ions, ppm, {}
    if name == "kmix":         # 1..10 isotope peaks per ion: K = 1 (no tail) and K > 8 (dense path)
        ions = syn.make_ion_table(25, seed=101, decoy_seed=102, k_range=(1, 10))
        ds = syn.make_dataset_np(40, 40, 500, seed=103, ions=ions, plant_fraction=0.4, plant_seed=104)
        return ds, ions, 30.0, {}
    if name == "clip99":       # gated q-percentile hot-spot clip (do_preprocessing): dense path, radix select
        ds, ions, ppm, _ = make_case("dups")
        return ds, ions, ppm, {"do_preprocessing": True, "q": 99.0}
    if name == "clip_q50_conn8":
        ds, ions, ppm, _ = make_case("zeros_rect")
        return ds, ions, ppm, {"do_preprocessing": True, "q": 50.0, "connectivity": 8}
    if name == "clip_dups_heavy":  # the clip with many flagged tail pixels (LDS table overflow -> global table)
        ds, ions, ppm, _ = make_case("dups_heavy")
        return ds, ions, ppm, {"do_preprocessing": True, "q": 90.0}
    if name == "clip_large":   # the clip on a > 2^18-pixel image with planted blobs (wide pass, q 99.5)
        ds, ions, ppm, _ = make_case("large_image")
        return ds, ions, ppm, {"do_preprocessing": True, "q": 99.5}
    if name == "wide_range":   # intensities over ~1e-3..1e9 with the bright mass BEFORE the scored windows: the
        # window sums must not depend on the total intensity (or squared intensity) preceding them in m/z order
        ions = syn.make_ion_table(30, seed=151, decoy_seed=152, mass_range=(480.0, 880.0))
        ds = syn.make_dataset_np(48, 48, 400, seed=153, ions=ions, plant_fraction=0.5, plant_seed=154)
        rng = np.random.default_rng(155)
        ints = ds.ints.copy()
        bright = ds.mz < 420.0
        ints[bright] = rng.lognormal(17.0, 1.0, int(bright.sum())).astype(np.float32)
        ints[~bright] = (ints[~bright] * 1e-3).astype(np.float32)  # background ~0.4, planted blobs ~3
        return syn.SpectraSet(sp_off=ds.sp_off, mz=ds.mz, ints=ints, coords=ds.coords), ions, 100.0, {}
    if name == "wide_overflow":  # windows beyond the LDS passes whose flagged tail pixels overflow the wide pass's
        # duplicate table (8192 entries): the pixel-indexed dense kernel takes them over
        full = syn.make_ion_table(2, seed=161, decoy_seed=162)
        tgt = np.nonzero(np.isin(full.adducts, list(full.target_adducts)))[0][:3]
        ions = subset_ions(full, tgt)
        ds = syn.make_dataset_np(150, 150, 4, seed=163, ions=ions, plant_fraction=1.0, plant_seed=164,
                                 blob_sigma=(400.0, 500.0))
        return add_duplicates(ds, 0.7, 165), ions, 20.0, {}
    if name == "nlevels100":   # level indices above 63 (the exact eL packs them 8 bits per column)
        ds, ions, ppm, _ = make_case("basic")
        return ds, ions, ppm, {"nlevels": 100}
    if name == "bands":        # 250 x 1000 px: the sparse main pass screens chaos in two row bands; planted blobs give
        # ions with > 64 chaos candidates (the hash-indexed Kruskal) and blobs across the band boundary
        full = syn.make_ion_table(16, seed=171, decoy_seed=172)
        tgt = np.nonzero(np.isin(full.adducts, list(full.target_adducts)))[0][:24]
        dec = np.nonzero(~np.isin(full.adducts, list(full.target_adducts)))[0][:8]
        ions = subset_ions(full, np.concatenate([tgt, dec]))
        ds = syn.make_dataset_np(250, 1000, 3, seed=173, ions=ions, plant_fraction=1.0, plant_seed=174,
                                 blob_sigma=(4.0, 10.0))
        return add_duplicates(ds, 0.02, 175), ions, 20.0, {}
    if name == "clip_ties":    # the clip's radix selects down every path: intensities from five values, three of
        # them one f32 ulp apart (the select runs to its last byte, many ties: the pair pass), windows whose positive
        # values are all equal (no pass), a value alone in its top byte (fetch + next order statistic in one pass)
        ds, ions, ppm, _ = make_case("long_tail")
        rng = np.random.default_rng(181)
        one = np.float32(1.0)
        vals = np.array([one, np.nextafter(one, np.float32(2)), np.nextafter(np.nextafter(one, np.float32(2)),
                                                                              np.float32(2)), 2.5, 1e6, 0.0],
                        dtype=np.float32)
        pick = rng.choice(len(vals), size=ds.ints.size, p=[0.45, 0.2, 0.1, 0.12, 0.03, 0.1])
        ints = vals[pick]
        # every point of the first ion's windows the same value: all-equal sets (lo == hi)
        lo_mz, hi_mz = float(ions.peak_mz[ions.win_off[0]]) * (1 - 2e-4), float(ions.peak_mz[ions.win_off[1] - 1]) * (1 + 2e-4)
        ints[(ds.mz >= lo_mz) & (ds.mz <= hi_mz)] = np.float32(3.0)
        return (syn.SpectraSet(sp_off=ds.sp_off, mz=ds.mz, ints=ints, coords=ds.coords), ions, ppm,
                {"do_preprocessing": True, "q": 75.0})
    if name == "boundary":
        ds = syn.make_dataset_np(16, 16, 300, seed=71)
        return ds, boundary_ions(ds, 5.0, 40, 72), 5.0, {}
    raise KeyError(name)


CASES = ["basic", "zeros_rect", "dups", "row", "column", "row_border1", "conn8_border1", "nlevels", "nlevels1", "big_window", "huge_window",
         "large_image", "xl_image", "large_blobs", "boundary", "long_tail", "dups_heavy", "kmix", "clip99", "clip_q50_conn8",
         "clip_dups_heavy", "clip_large", "wide_range", "wide_overflow", "nlevels100", "bands", "clip_ties"]


def oracle_run(ds, ions, ppm, nlevels=30, connectivity=4, erosion_border=0, q=99.0, do_preprocessing=False):
    from oracle import msm_oracle as O
    pm, dims = ds.pixel_map_dims()
    imgs = O.compute_sf_images(ds.spectra(), pm, dims, sf_peak_df(ions), ppm)
    df = O.sf_image_metrics(imgs, sf_peak_ints(ions), dims[0], dims[1], nlevels, connectivity=connectivity,
                            erosion_border=erosion_border, q=q, do_preprocessing=do_preprocessing)
    return imgs, df
