"""Result-row wire format of the hot path's outputs (sm/engine/search_results.py:58-110).

The Postgres/Spark storage itself is out of scope; these generators produce the exact rows the reference
inserts so a storage backend can consume them:

* ``metrics_rows`` (:57-62): (job_id, db_id, sf_id, adduct, msm, fdr, json{chaos, spatial, spectral}, peaks_n)
* ``iso_image_rows`` (:88-97): per (ion, peak) with any pixel > 0.001: (job_id, db_id, sf_id, adduct, peak,
  flattened pixel indices, intensities, min over the full image, max over the full image)
"""
from __future__ import annotations

import json
from collections import OrderedDict

import numpy as np


def metrics_rows(job_id, db_id, sf_metrics_df, sf_adduct_peaksn, metrics=("chaos", "spatial", "spectral")):
    peaksn = {(s, a): n for s, a, n in sf_adduct_peaksn}
    for _, r in sf_metrics_df.reset_index().iterrows():
        metr_json = json.dumps(OrderedDict([(m, float(r[m])) for m in metrics]))
        yield (job_id, db_id, r.sf_id, r.adduct, float(r.msm), float(r.fdr), metr_json, peaksn[(r.sf_id, r.adduct)])


def iso_image_rows(job_id, db_id, sf_iso_images, nrows, ncols):
    items = sf_iso_images.collect() if hasattr(sf_iso_images, "collect") else sf_iso_images
    for (sf_id, adduct), img_list in items:
        for peak_i, img_sparse in enumerate(img_list):
            img_ints = np.zeros(int(nrows) * int(ncols)) if img_sparse is None else img_sparse.toarray().flatten()
            pixel_inds = np.arange(img_ints.shape[0])
            mask = img_ints > 0.001
            if mask.sum() > 0:
                yield (job_id, db_id, sf_id, adduct, peak_i, pixel_inds[mask].tolist(), img_ints[mask].tolist(),
                       img_ints.min(), img_ints.max())
