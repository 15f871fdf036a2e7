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


def _theor_arrays(ims, sf_ints, device):
    """Theoretical intensities aligned with the ions of ``ims``: device (Kt int64[n_ion], values f64[sum Kt])
    with Kt = len(sf_ints[key]).  A PeakInts mapping (FormulasSegm) is aligned on the device by key search; any
    other mapping is read key by key."""
    import torch

    from .formulas import PeakInts
    ik = ims.ion_keys
    n = len(ik)
    if isinstance(sf_ints, PeakInts):
        cache = sf_ints.__dict__.setdefault("_dev_cache", {})
        # keyed by the adduct list and the sf levels object itself: the entry holds a reference to the levels it
        # was built for and is used only for that same object (an id() alone can be reused after collection)
        sig = (str(device), tuple(ik.adducts), None if ik.sf_levels is None else id(ik.sf_levels))
        if sig in cache and cache[sig][4] is not ik.sf_levels:
            cache.clear()
        # the alignment is a function of the ion keys only: the last one is reused while they are the same
        # (a search per step over the same formula table), without its synchronisations
        last = cache.get(("last",) + sig)
        if (last is not None and last[4] is ik.sf_levels and len(last[0]) == n
                and (last[5] is ik.keys or np.array_equal(last[0], ik.keys))):
            return last[1], last[2], last[3]
        n_pk = len(sf_ints.sf_ids)
        if (sig not in cache and ik.sf_levels is None and n_pk == n and n > 0 and
                list(sf_ints.adducts) == list(ik.adducts)):
            # the common case: the layout's ions are exactly the table's ions, in the table's (sf_id, adduct)
            # order -- the alignment is the identity (no key search, no host synchronisation)
            own = np.asarray(sf_ints.sf_ids, np.int64) * ik.n_cat + np.asarray(sf_ints.adduct_codes, np.int64)
            if np.array_equal(own, ik.keys):
                off_t = torch.from_numpy(np.ascontiguousarray(sf_ints.off, np.int64)).to(device)
                vals = torch.from_numpy(np.ascontiguousarray(sf_ints.values, np.float64)).to(device)
                out = (off_t[1:] - off_t[:-1], vals, off_t)
                cache.clear()
                cache[("last",) + sig] = (np.array(ik.keys, copy=True),) + out + (ik.sf_levels, ik.keys)
                return out
        if sig not in cache:
            k, ok = ik.encode_codes(sf_ints.sf_ids, sf_ints.adduct_codes, sf_ints.adducts)
            rows = np.nonzero(ok)[0]
            k = k[rows]
            if len(k) > 1 and not (k[1:] > k[:-1]).all():
                o = np.argsort(k, kind="stable")
                k, rows = k[o], rows[o]
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
            cache.clear()
            cache[sig] = (t(k), t(rows), t(np.asarray(sf_ints.off, np.int64)), t(np.asarray(sf_ints.values, np.float64)),
                          ik.sf_levels)
        pk_key, pk_row, pk_off, pk_val, _ = cache[sig]
        ion_key = ik.keys_dev if ik.keys_dev is not None else torch.from_numpy(ik.keys).to(device)
        if n == 0:
            return (torch.zeros(0, dtype=torch.int64, device=device), torch.zeros(0, dtype=torch.float64, device=device),
                    torch.zeros(1, dtype=torch.int64, device=device))
        if pk_key.numel() == 0:
            raise KeyError(ims.keys[0])
        j = torch.searchsorted(pk_key, ion_key).clamp_(max=pk_key.numel() - 1)
        miss = pk_key[j] != ion_key
        if bool(miss.any().item()):  # formula_img_validator.py:117: sf_peak_ints[(sf_id, adduct)] raises
            raise KeyError(ims.keys[int(torch.nonzero(miss)[0].item())])
        row = pk_row[j]
        Kt = pk_off[row + 1] - pk_off[row]
        off_t = torch.zeros(n + 1, dtype=torch.int64, device=device)
        torch.cumsum(Kt, 0, out=off_t[1:])
        n_t = int(off_t[-1].item())
        owner = torch.repeat_interleave(torch.arange(n, device=device), Kt, output_size=n_t)
        k_in = torch.arange(n_t, device=device) - off_t[owner]
        out = (Kt, pk_val[pk_off[row][owner] + k_in], off_t)
        cache.pop(("last",) + sig, None)
        cache[("last",) + sig] = (np.array(ik.keys, copy=True),) + out + (ik.sf_levels, ik.keys)
        return out
    vals = [sf_ints[k] for k in ims.keys]
    Kt = np.array([len(v) for v in vals], dtype=np.int64)
    flat = np.concatenate([np.asarray(v, np.float64) for v in vals]) if n else np.zeros(0)
    off = np.zeros(n + 1, np.int64)
    np.cumsum(Kt, out=off[1:])
    return torch.from_numpy(Kt).to(device), torch.from_numpy(flat).to(device), torch.from_numpy(off).to(device)


def _metrics_device_rows(ims, sf_ints, img_conf, prelaunch=None):
    """Score every ion of an IonImageSet with one fused launch; returns (device bool[n_ion]: the ion gets a row,
    engine.IonMetrics).

    The kernel sees exactly len(sf_ints[key]) windows per ion: compute() pads the image list with empty images
    up to that length (formula_img_validator.py:73-75), and windows of sf_peak_df beyond it do not enter the
    metrics.  The alignment runs on the side stream (it needs only the layout, not the sorted peaks).

    Which ions get a row is known before the launch (an ion has images and >= 1 of its first min(Kt, 32) scored
    windows is non-empty: the kernel's SMG_ION_HAS_HITS flag); ``prelaunch(keep)`` is called with it just before
    the kernel is queued, so a caller can stage the table's index while the kernel runs."""
    import torch

    from . import engine as E
    from ._lib import SMG_HITS_PACKED_F32, check, lib
    from .engine import _p, _stream
    from .formula_imager_segm import _side_stream
    opts = _chaos_opts(img_conf)
    ims.ensure_current()
    dev = ims.lo.device
    n = ims.n_ions
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    with torch.cuda.stream(side):
        Kt, theor, off_t = _theor_arrays(ims, sf_ints, dev)
        sel_dev = None if ims._sel is None else torch.from_numpy(ims._sel.astype(np.uint8)).to(dev)
    main.wait_stream(side)
    for t in (Kt, theor, off_t) + ((sel_dev,) if sel_dev is not None else ()):
        t.record_stream(main)
    # the scored windows (the layout's, padded with empty runs up to len(sf_ints[key])) and the table-row flags
    # in one launch (smg_align_windows), on the main stream after the window search
    n_t = theor.numel()
    lo2 = torch.empty(n_t, dtype=torch.int64, device=dev)
    hi2 = torch.empty(n_t, dtype=torch.int64, device=dev)
    keep8 = torch.empty(n, dtype=torch.uint8, device=dev)
    check(lib().smg_align_windows(_p(ims.lo), _p(ims.hi), _p(ims.ions_dev.win_off), _p(off_t), _p(sel_dev), n,
                                  _p(lo2), _p(hi2), _p(keep8), _stream(None)), "smg_align_windows")
    keep = keep8.view(torch.bool)
    if prelaunch is not None:
        prelaunch(keep)
    nrows, ncols = ims.dims
    m = E.ion_metrics_raw(SMG_HITS_PACKED_F32, ims.peaks.hits_sorted, None, ims.peaks.sorted_cum(), lo2, hi2,
                          off_t, theor, ims.ions_dev.ion_order, n, nrows, ncols, **opts)
    return keep, m


def _metrics_device_batch(ims, sf_ints, img_conf):
    """The reference table (index [sf_id, adduct], columns chaos, spatial, spectral, msm) of an IonImageSet:
    one row per ion with images (formula_img_validator.py:115-121), built from codes, not tuples.  The row set
    is known before the scoring launch: its index codes are copied to the host and the MultiIndex is built
    there while the kernel runs; only the metric columns are copied after it."""
    import torch
    from .formula_imager_segm import FrameIndex
    fi = FrameIndex(ims.ion_keys)
    keep, m = _metrics_device_rows(ims, sf_ints, img_conf, prelaunch=fi.stage)
    return fi.frame(torch.stack([m.chaos, m.spatial, m.spectral, m.msm], 0))


def sf_image_metrics_est_fdr(sf_metrics_df, formulas, fdr):
    """formula_img_validator.py:125-130."""
    sf_msm_df = formulas.get_sf_adduct_sorted_df()
    sf_msm_df = sf_msm_df.join(sf_metrics_df.msm).fillna(0)
    sf_adduct_fdr = fdr.estimate_fdr(sf_msm_df)
    return sf_metrics_df.join(sf_adduct_fdr, how="inner")[["chaos", "spatial", "spectral", "msm", "fdr"]]
