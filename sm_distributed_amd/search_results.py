"""Result-row wire format of the hot path's outputs (sm/engine/search_results.py:58-110).

The Postgres/Spark storage itself is out of scope; these generators produce the exact rows the reference
inserts so a storage backend can consume them:

* ``metrics_rows`` (:57-62): (job_id, db_id, sf_id, adduct, msm, fdr, json{chaos, spatial, spectral}, peaks_n),
  peaks_n positional as in the reference (or by key, a documented opt-in deviation)
* ``iso_image_rows`` (:88-97): per (ion, peak) with any pixel > 0.001: (job_id, db_id, sf_id, adduct, peak,
  flattened pixel indices, intensities, min over the full image, max over the full image)
"""
from __future__ import annotations

import json
from collections import OrderedDict

import numpy as np


def metrics_rows(job_id, db_id, sf_metrics_df, sf_adduct_peaksn, metrics=("chaos", "spatial", "spectral"),
                 peaks_n="positional"):
    """search_results.py:57-62.  ``peaks_n="positional"`` reproduces the reference exactly: row ``ind`` of the
    metrics table takes ``sf_adduct_peaksn[ind][2]``, the peak count of the ``ind``-th (sf_id, adduct) of the
    formula table -- which is the row's own count only when the two tables list the same ions in the same order
    (the metrics table is filtered to reported targets, so in a real search it usually is not).
    ``peaks_n="by_key"`` (documented deviation) looks the count up by the row's (sf_id, adduct) instead."""
    if peaks_n not in ("positional", "by_key"):
        raise ValueError("peaks_n must be 'positional' or 'by_key'")
    peaksn = list(sf_adduct_peaksn)
    by_key = {(s, a): n for s, a, n in peaksn} if peaks_n == "by_key" else None
    for ind, r in sf_metrics_df.reset_index().iterrows():
        metr_json = json.dumps(OrderedDict([(m, float(r[m])) for m in metrics]))
        n = peaksn[ind][2] if by_key is None else by_key[(r.sf_id, r.adduct)]
        yield (job_id, db_id, r.sf_id, r.adduct, float(r.msm), float(r.fdr), metr_json, n)


def iso_image_rows(job_id, db_id, sf_iso_images, nrows, ncols):
    """search_results.py:88-97 (iso_img_row_gen) without densifying any image.  A device ``IonImageSet`` (the
    output of compute_sf_images, possibly filtered) is reduced on the GPU (smg_iso_image_rows); any other iterable
    of ((sf_id, adduct), [sparse | None]) is reduced per image from its COO entries: duplicates summed
    (= toarray()), pixels > 0.001 in flattened row-major order, min / max over the nrows*ncols image (pixels without
    an entry are 0)."""
    from .formula_imager_segm import IonImageSet
    if isinstance(sf_iso_images, IonImageSet):
        yield from sf_iso_images.image_rows().rows(job_id, db_id)
        return
    npx = int(nrows) * int(ncols)
    items = sf_iso_images.collect() if hasattr(sf_iso_images, "collect") else sf_iso_images
    for (sf_id, adduct), img_list in items:
        for peak_i, img_sparse in enumerate(img_list):
            if img_sparse is None:
                continue  # np.zeros: no pixel > 0.001
            c = img_sparse.tocoo(copy=True)
            c.sum_duplicates()  # sorted by (row, col): flattened index ascending
            flat = c.row.astype(np.int64) * int(ncols) + c.col.astype(np.int64)
            v = np.asarray(c.data, dtype=np.float64)
            mask = v > 0.001
            if mask.sum() > 0:
                full = len(v) >= npx
                vmin = v.min() if full else min(0.0, v.min())
                vmax = v.max() if full else max(0.0, v.max())
                yield (job_id, db_id, sf_id, adduct, peak_i, flat[mask].tolist(), v[mask].tolist(),
                       np.float64(vmin), np.float64(vmax))
