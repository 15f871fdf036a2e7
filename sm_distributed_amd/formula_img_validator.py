"""MSM scoring: drop-in for sm/engine/msm_basic/formula_img_validator.py.

* ``sf_image_metrics(sf_images, sc, formulas, ds, ds_config)`` (:93-122) -- one row per ion present in
  ``sf_images``, DataFrame indexed by [sf_id, adduct] with float64 columns chaos, spatial, spectral, msm.
  For an ``IonImageSet`` (the output of ``compute_sf_images``) the whole batch is scored by one fused
  device launch (libsmg ``smg_ion_metrics``); for any other iterable of ``((sf_id, adduct), [images])``
  the images are uploaded and scored by the same kernels.
* ``get_compute_img_metrics(empty_matrix, img_gen_conf)`` (:58-86) returns ``compute(iso_images_sparse,
  sf_ints) -> (chaos, spatial, spectral)``; it is looked up at call time so tests can patch it, exactly as
  the reference tests do (test_formula_img_validator.py:52-53).
* ``ImgMeasures`` (:13-55), ``sf_image_metrics_est_fdr`` (:125-130) unchanged in meaning.

Metric arithmetic = the pyImagingMSpec 0.1.1 / cpyImagingMSpec 0.0.4 restatement documented in
DESIGN.md §Oracle (chaos: threshold levels np.linspace(0, 1, nlevels), dilation 4-cross, erosion 3x3 box,
4-connected components; configurable via ``image_generation.chaos_connectivity`` / ``chaos_erosion_border``).
"""
from __future__ import annotations

import numpy as np
import pandas as pd


class ImgMeasures(object):
    """Container for isotope image metrics (formula_img_validator.py:13-55)."""

    def __init__(self, chaos, image_corr, pattern_match):
        self.chaos = chaos
        self.image_corr = image_corr
        self.pattern_match = pattern_match

    @staticmethod
    def _replace_nan(v, new_v=0):
        if v is None or not v or np.isinf(v) or np.isnan(v):
            return new_v
        return v

    def to_tuple(self, replace_nan=True):
        if replace_nan:
            return (self._replace_nan(self.chaos), self._replace_nan(self.image_corr),
                    self._replace_nan(self.pattern_match))
        return self.chaos, self.image_corr, self.pattern_match


def _chaos_opts(img_gen_conf):
    return dict(nlevels=int(img_gen_conf.get("nlevels", 30)), q=float(img_gen_conf.get("q", 99.0)),
                do_preprocessing=bool(img_gen_conf.get("do_preprocessing", False)),
                connectivity=int(img_gen_conf.get("chaos_connectivity", 4)),
                erosion_border=int(img_gen_conf.get("chaos_erosion_border", 0)))


def get_compute_img_metrics(empty_matrix, img_gen_conf):
    """formula_img_validator.py:58-86: per-ion metric function (device-backed)."""
    nrows, ncols = np.shape(empty_matrix)
    opts = _chaos_opts(img_gen_conf)

    def compute(iso_images_sparse, sf_ints):
        from .engine import metrics_from_images
        if len(sf_ints) == 0 and len(iso_images_sparse) == 0:
            return ImgMeasures(0, 0, 0).to_tuple()
        r = metrics_from_images([(list(iso_images_sparse), list(sf_ints))], nrows, ncols, **opts)
        return float(r["chaos"][0]), float(r["spatial"][0]), float(r["spectral"][0])

    compute.batched = True  # marks the library's own implementation (see sf_image_metrics)
    return compute


_default_get_compute = get_compute_img_metrics


def _calculate_msm(sf_metrics_df):
    return sf_metrics_df.chaos * sf_metrics_df.spatial * sf_metrics_df.spectral


def _frame(keys, chaos, spatial, spectral):
    df = pd.DataFrame({"sf_id": [k[0] for k in keys], "adduct": [k[1] for k in keys],
                       "chaos": np.asarray(chaos, dtype=np.float64), "spatial": np.asarray(spatial, dtype=np.float64),
                       "spectral": np.asarray(spectral, dtype=np.float64)},
                      columns=["sf_id", "adduct", "chaos", "spatial", "spectral"])
    df = df.set_index(["sf_id", "adduct"])
    df["msm"] = _calculate_msm(df)
    return df


def sf_image_metrics(sf_images, sc, formulas, ds, ds_config):
    """formula_img_validator.py:93-122.  ``sc`` is accepted and ignored."""
    from .formula_imager_segm import IonImageSet
    nrows, ncols = ds.get_dims()
    img_conf = ds_config["image_generation"]
    sf_ints = formulas.get_sf_peak_ints()
    patched = globals()["get_compute_img_metrics"] is not _default_get_compute
    if isinstance(sf_images, IonImageSet) and not patched:
        return _metrics_device_batch(sf_images, sf_ints, img_conf)
    compute = globals()["get_compute_img_metrics"](np.zeros((nrows, ncols)), img_conf)
    items = sf_images.collect() if hasattr(sf_images, "collect") else list(sf_images)
    if getattr(compute, "batched", False):
        from .engine import metrics_from_images
        opts = _chaos_opts(img_conf)
        keys = [k for k, _ in items]
        r = metrics_from_images([(imgs, sf_ints[k]) for k, imgs in items], nrows, ncols, **opts)
        return _frame(keys, r["chaos"], r["spatial"], r["spectral"])
    rows = [(k,) + tuple(compute(imgs, sf_ints[k])) for k, imgs in items]
    return _frame([r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows], [r[3] for r in rows])


def _metrics_device_batch(ims, sf_ints, img_conf):
    """Score every ion of an IonImageSet with one fused launch (rows only for ions with images)."""
    import torch

    from . import engine as E
    from ._lib import SMG_HITS_PACKED_F32
    opts = _chaos_opts(img_conf)
    ims.ensure_current()
    keys = ims.keys
    K = np.diff(ims.win_off)
    need = np.array([len(sf_ints[k]) for k in keys], dtype=np.int64)
    if np.any(need > K):
        # theoretical patterns longer than the windows of sf_peak_df: re-layout with empty padding windows
        lo = ims.lo.cpu().numpy()
        hi = ims.hi.cpu().numpy()
        Kn = np.maximum(K, need)
        off = np.zeros(len(keys) + 1, np.int64)
        np.cumsum(Kn, out=off[1:])
        nlo = np.zeros(off[-1], np.int64)
        nhi = np.zeros(off[-1], np.int64)
        for i in range(len(keys)):
            a, b = ims.win_off[i], ims.win_off[i + 1]
            nlo[off[i]:off[i] + (b - a)] = lo[a:b]
            nhi[off[i]:off[i] + (b - a)] = hi[a:b]
        win_off = off
        dev = ims.lo.device
        lo_d, hi_d = torch.from_numpy(nlo).to(dev), torch.from_numpy(nhi).to(dev)
    else:
        win_off, lo_d, hi_d = ims.win_off, ims.lo, ims.hi
        Kn = K
    theor = np.zeros(int(win_off[-1]))
    for i, k in enumerate(keys):
        v = sf_ints[k]
        theor[win_off[i]:win_off[i] + len(v)] = v
    # windows beyond len(sf_ints) (sf_peak_df longer than the pattern) keep theor 0 -- the reference would
    # use len(sf_ints) images only; trim them by giving the kernel exactly len(sf_ints) windows
    if np.any(need < Kn):
        sel = np.concatenate([np.arange(win_off[i], win_off[i] + need[i]) for i in range(len(keys))])
        off2 = np.zeros(len(keys) + 1, np.int64)
        np.cumsum(need, out=off2[1:])
        dev = ims.lo.device
        st = torch.from_numpy(sel).to(dev)
        lo_d, hi_d, theor, win_off = lo_d[st], hi_d[st], theor[sel], off2
    dev = ims.lo.device
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)
    nrows, ncols = ims.dims
    m = E.ion_metrics_raw(SMG_HITS_PACKED_F32, ims.peaks.hits_sorted, None, ims.peaks.sorted_cum(), lo_d, hi_d,
                          t(win_off, np.int64),
                          t(theor, np.float64), ims.ions_dev.ion_order, len(keys), nrows, ncols, **opts)
    r = m.to_numpy()
    has = (r["flags"] & 1) != 0
    sel = ims.ion_indices()
    sel = sel[has[sel]]
    return _frame([keys[i] for i in sel], r["chaos"][sel], r["spatial"][sel], r["spectral"][sel])


def sf_image_metrics_est_fdr(sf_metrics_df, formulas, fdr):
    """formula_img_validator.py:125-130."""
    sf_msm_df = formulas.get_sf_adduct_sorted_df()
    sf_msm_df = sf_msm_df.join(sf_metrics_df.msm).fillna(0)
    sf_adduct_fdr = fdr.estimate_fdr(sf_msm_df)
    return sf_metrics_df.join(sf_adduct_fdr, how="inner")[["chaos", "spatial", "spectral", "msm", "fdr"]]
