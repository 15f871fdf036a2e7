#!/usr/bin/env python
"""Generate the committed golden fixtures under tests/golden/.

1. kats.json -- the hot path's known-answer tests transcribed from the reference unit tests (small
   hand-written inputs and expected outputs): sm/engine/tests/msm_basic/test_formula_imager.py:11-51,
   test_formula_imager_segm.py:7-26, test_formula_img_validator.py:17-92, sm/engine/tests/test_fdr.py:29-75,
   sm/engine/tests/test_formulas.py:24-27, tests/test_search_results.py:59-77.
2. synth_<case>_expected.csv -- oracle metric tables of seeded synthetic parity cases (tests/parity_cases.py),
   pinning the oracle against regressions.
3. synthetic_example.imzML/.ibd -- a 3x3 continuous-mode imzML written by our own writer
   (tests/imzml_writer.py) with the shape of the reference's bundled example (config 1), plus its oracle
   metric table.  No reference data is copied or derived.

Usage: python scripts/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")

# C12H24O (the formula tests/test_search_job_imzml_example.py:28-33 searches) and a hand-made pattern
C12H24O = 12 * 12.0 + 24 * 1.00782503207 + 15.99491461956
PATTERN = [100.0, 13.33, 0.967, 0.052]
EXAMPLE_ADDUCTS = ["+H", "+Na", "+K", "+He", "+Li", "+C", "+O", "+Mg", "+Cl"]


def kats():
    return {
        "sample_spectra_2by3": {
            "spectra": [[0, [100.0], [0, 100.0]], [1, [100.0], [0, 100.0]], [2, [50.0], [0, 100.0]],
                        [3, [200.0], [0, 100.0]], [4, [200.0], [0, 100.0]]],
            "lower": [100 - 0.01, 200 - 0.01], "upper": [100 + 0.01, 200 + 0.01],
            "sf_peak_map": [[0, 0], [0, 1]],
            "expected": [[[0, 0], [0, 100.0]], [[0, 0], [1, 100.0]], [[0, 1], [3, 100.0]], [[0, 1], [4, 100.0]]],
        },
        "compute_sf_peak_images_2by3": {
            "dims": [2, 3], "pixel_inds": [1, 2, 3, 4, 5],
            "sf_sp_intens": [[[0, 0], [0, 100.0]], [[0, 0], [1, 100.0]], [[0, 1], [3, 100.0]], [[0, 1], [4, 100.0]]],
            "expected": {"0": [[0, 100, 100], [0, 0, 0]], "1": [[0, 0, 0], [0, 100, 100]]},
        },
        "gen_iso_sf_images": {
            "shape": [1, 3],
            "pairs": [[0, [[1.0, 0.0, 0.0]]], [3, [[2.0, 1.0, 0.0]]], [3, [[0.0, 0.0, 10.0]]]],
            "expected": [[[1.0, 0.0, 0.0]], None, None, [[2.0, 1.0, 0.0]]],
        },
        "compute_img_measures_plumbing": {
            "mocked": {"chaos": 0.99, "spatial": 0.8, "spectral": 0.95}, "expected": [0.99, 0.8, 0.95],
            "images": [[[0.0, 100.0, 100.0], [10.0, 0.0, 3.0]], [[0.0, 50.0, 50.0], [0.0, 20.0, 0.0]]],
            "sf_ints": [100.0, 10.0, 1.0],
        },
        "replace_invalid": {"inputs": [None, "nan", "inf"], "expected": 0.0},
        "estimate_fdr_1": {
            "decoy_sample_size": 2, "target_adducts": ["+H"], "fdr_levels": [0.2, 0.8],
            "td": [[1, "+H", "+Cu"], [1, "+H", "+Co"], [2, "+H", "+Ag"], [2, "+H", "+Ar"]],
            "msm": [[1, "+H", 0.85], [2, "+H", 0.5], [1, "+Cu", 0.5], [1, "+Co", 0.5], [2, "+Ag", 0.75],
                    [2, "+Ar", 0.0]],
            "expected": [[1, "+H", 0.2], [2, "+H", 0.8]],
        },
        "estimate_fdr_digitize": {
            "decoy_sample_size": 1, "target_adducts": ["+H"], "fdr_levels": [0.4, 0.8],
            "td": [[1, "+H", "+Cu"], [2, "+H", "+Ag"], [3, "+H", "+Cl"], [4, "+H", "+Co"]],
            "msm": [[1, "+H", 1.0], [2, "+H", 0.75], [3, "+H", 0.5], [4, "+H", 0.25], [1, "+Cu", 0.75],
                    [2, "+Ag", 0.3], [3, "+Cl", 0.25], [4, "+Co", 0.1]],
            "expected": [[1, "+H", 0.4], [2, "+H", 0.4], [3, "+H", 0.4], [4, "+H", 0.8]],
        },
        "decoy_selection": {"decoy_adducts": ["+He", "+Li"], "target_adducts": ["+H", "+K"], "sf_ids": [1],
                            "decoy_sample_size": 2,
                            "expected": [[1, "+H", "+He"], [1, "+H", "+Li"], [1, "+K", "+He"], [1, "+K", "+Li"]]},
        "legacy_ppm_bounds": {"mz": 100.0, "ppm": 1.0, "expected_lower": 100 - 100e-6, "expected_upper": 100 + 100e-6},
        "iso_image_rows": {
            "dims": [2, 3], "images": [[[100, 0, 0], [0, 0, 0]], [[0, 0, 0], [0, 0, 10]]],
            "expected": [[0, 0, 1, "+H", 0, [0], [100.0], 0.0, 100.0], [0, 0, 1, "+H", 1, [5], [10.0], 0.0, 10.0]],
        },
        "sf_image_metrics_table": {
            "dims": [2, 3], "mocked": [0.9, 0.9, 0.9],
            "expected": [[0, "+H", 0.9, 0.9, 0.9, 0.729], [1, "+H", 0.9, 0.9, 0.9, 0.729]],
        },
    }


def example_ions():
    from sm_distributed_amd import synthetic as syn
    mzs, ints, sfs, adds = [], [], [], []
    for a in EXAMPLE_ADDUCTS:
        base = C12H24O + syn.adduct_shift(a)
        mzs.append([round(base + k * syn.ISOTOPE_SPACING, 6) for k in range(len(PATTERN))])
        ints.append(PATTERN)
        sfs.append(10007)
        adds.append(a)
    K = [len(m) for m in mzs]
    off = np.concatenate([[0], np.cumsum(K)]).astype(np.int64)
    return syn.IonTable(sf_ids=np.array(sfs, np.int64), adducts=np.array(adds, dtype=object), win_off=off,
                        peak_mz=np.concatenate(mzs), peak_int=np.concatenate(ints).astype(np.float64),
                        td=(np.zeros(0), np.zeros(0), np.zeros(0)))


def synthetic_example_spectra(seed=5):
    """3x3 continuous-mode spectra: shared m/z axis 100..800 step 1/12, sparse positive intensities with
    explicit zeros (the shape of the reference's bundled example), the example ions' peaks planted."""
    from sm_distributed_amd import synthetic as syn
    rng = np.random.default_rng(seed)
    axis = (100.0 + np.arange(8399) / 12.0).astype(np.float32)
    ions = example_ions()
    mzs, its, coords = [], [], []
    for y in range(1, 4):
        for x in range(1, 4):
            it = np.where(rng.random(axis.size) < 0.3, rng.lognormal(4.0, 1.0, axis.size), 0.0)
            for k, m in enumerate(ions.peak_mz):
                j = int(np.argmin(np.abs(axis - m)))
                it[j] += 1000.0 * PATTERN[k % len(PATTERN)] / 100.0 * rng.uniform(0.5, 1.5)
            mzs.append(axis.copy())
            its.append(it.astype(np.float32))
            coords.append((x, y))
    off = np.concatenate([[0], np.cumsum([len(m) for m in mzs])]).astype(np.int64)
    return syn.SpectraSet(sp_off=off, mz=np.concatenate(mzs), ints=np.concatenate(its), coords=np.array(coords))


def synthetic_example():
    from oracle import msm_oracle as O
    from tests.imzml_writer import write_imzml
    from tests.parity_cases import sf_peak_df, sf_peak_ints
    ds = synthetic_example_spectra()
    write_imzml(os.path.join(GOLDEN, "synthetic_example.imzML"), ds, continuous=True)
    ions = example_ions()
    pm, dims = ds.pixel_map_dims()
    ppm, nlevels = 100.0, 30
    imgs = O.compute_sf_images(ds.spectra(), pm, dims, sf_peak_df(ions), ppm)
    df = O.sf_image_metrics(imgs, sf_peak_ints(ions), dims[0], dims[1], nlevels)
    df.reset_index().to_csv(os.path.join(GOLDEN, "synthetic_example_expected.csv"), index=False,
                            float_format="%.17g")
    print("synthetic example:", ds.n_points, "points,", len(df), "scored ions")


def synth_fixtures():
    from tests.parity_cases import make_case, oracle_run
    for name in ("basic", "dups", "conn8_border1"):
        ds, ions, ppm, kw = make_case(name)
        _, df = oracle_run(ds, ions, ppm, **kw)
        df.reset_index().to_csv(os.path.join(GOLDEN, f"synth_{name}_expected.csv"), index=False,
                                float_format="%.17g")
        print(name, len(df), "rows")


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    with open(os.path.join(GOLDEN, "kats.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    synthetic_example()
    synth_fixtures()


if __name__ == "__main__":
    main()
