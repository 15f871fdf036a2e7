"""Oracle check of a seeded ion sample of a full-size device run (shared by the config-3 / config-5 GPU tests).

The oracle cannot image a 5e8-5e9-point dataset for ~1M ions, so the full-size tests score a sample: every data
point of the sample's windows is selected from the resident dataset by m/z (oracle/cpu_baseline.select_window_points,
with a margin), and the oracle (formula_imager_segm.py:66-92 + formula_img_validator.py:72-84) images and scores
the sample from those points on the host cores.
"""
from __future__ import annotations

import numpy as np

METRIC_ATOL = 1e-5


def planted_ions(ions, fraction=0.02, seed=45):
    """The target ions make_dataset_torch planted signal for (its seeded draw)."""
    prng = np.random.default_rng(seed)
    tgt = np.nonzero(ions.target_mask())[0]
    return prng.choice(tgt, size=max(1, int(round(fraction * len(tgt)))), replace=False)


def oracle_rows(ions, pick, peaks, dims, ppm, nlevels, workers_cap=16):
    """Oracle (chaos, spatial, spectral) of the ions ``pick`` (positions in ``ions``) from every point of their
    windows in the resident dataset; returns (rows [(ion, chaos, spatial, spectral)], window sizes of the
    selected points, number of points, wall seconds)."""
    from oracle import cpu_baseline as CB
    from oracle import msm_oracle as O
    wins = np.concatenate([np.arange(ions.win_off[i], ions.win_off[i + 1]) for i in pick])
    lower, upper = O.window_bounds(ions.peak_mz[wins], ppm)
    b_pix, b_mz, b_int = CB.select_window_points(peaks.mz, peaks.hits, lower, upper)
    seg = np.sort(b_mz).astype(np.float64)
    sizes = np.searchsorted(seg, upper, "right") - np.searchsorted(seg, lower, "left")
    tasks = [(int(i), ions.peak_mz[ions.win_off[i]:ions.win_off[i + 1]].copy(),
              ions.peak_int[ions.win_off[i]:ions.win_off[i + 1]].copy()) for i in pick]
    rows, wall, _ = CB.run_pool(b_pix, b_mz, b_int, dims, ppm, nlevels, tasks, CB.default_workers(cap=workers_cap))
    return rows, wins, sizes, b_mz.size, wall


def assert_rows_match(rows, lookup, atol=METRIC_ATOL):
    """Every oracle row within ``atol`` of the device's values; ``lookup(ion) -> (chaos, spatial, spectral,
    msm)``.  Returns the number of rows with msm > 0."""
    n_pos = 0
    for ion_id, c, s, p in rows:
        got = lookup(ion_id)
        for col, g, v in zip(("chaos", "spatial", "spectral", "msm"), got, (c, s, p, c * s * p)):
            assert abs(g - v) <= atol, (ion_id, col, g, v)
        n_pos += int(c * s * p > 0)
    return n_pos
