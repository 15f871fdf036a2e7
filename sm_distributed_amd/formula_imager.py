"""Legacy imager: drop-in for sm/engine/msm_basic/formula_imager.py (not called by the live search, pinned
by the reference unit tests test_formula_imager.py:11-51).

* ``sample_spectra(sc, ds, formulas)`` (:62-80): for every spectrum and theoretical window, the window sum
  ``cum[searchsorted(mzs, upper, 'r')] - cum[searchsorted(mzs, lower, 'l')]`` kept if > 0.001 -- computed
  by the ``smg_sample_spectra`` HIP kernel; returns ``[((sf_i, peak_i), (sp_i, intensity)), ...]`` in the
  reference's flatMap order (spectrum order, then window order).
* ``compute_sf_peak_images(ds, sf_sp_intens)`` (:83-103): image by assignment into a dense array -> CSR.
* ``compute_sf_images(sf_peak_imgs)`` (:106-123): group per formula, list indexed by peak id.
"""
from __future__ import annotations

import ctypes
from collections import defaultdict

import numpy as np
import scipy.sparse

from .rdd import LocalRDD


def sample_spectra(sc, ds, formulas, device="cuda"):
    import torch

    from ._lib import check, lib
    from .engine import _p, _stream, require_gpu
    require_gpu()
    lower, upper = formulas.get_sf_peak_bounds()
    sf_peak_map = np.asarray(formulas.get_sf_peak_map())
    spectra = ds.get_spectra().collect()
    spectra = sorted(spectra, key=lambda t: t[0])
    off = np.zeros(len(spectra) + 1, np.int64)
    mzs, cums, sp_ids = [], [], []
    for i, (sp_i, mz, cum) in enumerate(spectra):
        mz = np.asarray(mz, np.float64)
        cum = np.asarray(cum, np.float64)
        if cum.shape[0] != mz.shape[0] + 1:
            raise ValueError("legacy spectra carry cumulative ints with one leading element")
        mzs.append(mz)
        cums.append(cum)
        sp_ids.append(sp_i)
        off[i + 1] = off[i] + mz.shape[0]
    n_sp, n_w = len(spectra), len(lower)
    if n_sp == 0 or n_w == 0:
        return LocalRDD([])
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(device)
    d_off, d_mz, d_cum = t(off, np.int64), t(np.concatenate(mzs), np.float64), t(np.concatenate(cums), np.float64)
    d_lo, d_hi = t(lower, np.float64), t(upper, np.float64)
    cap = n_sp * n_w
    ow = torch.empty(cap, dtype=torch.int64, device=device)
    os_ = torch.empty_like(ow)
    ov = torch.empty(cap, dtype=torch.float64, device=device)
    cnt = torch.zeros(1, dtype=torch.int64, device=device)
    check(lib().smg_sample_spectra(_p(d_off), _p(d_mz), _p(d_cum), n_sp, _p(d_lo), _p(d_hi), n_w, _p(ow), _p(os_),
                                   _p(ov), cap, _p(cnt), _stream()), "smg_sample_spectra")
    n = int(cnt.item())
    w, s, v = ow[:n].cpu().numpy(), os_[:n].cpu().numpy(), ov[:n].cpu().numpy()
    order = np.lexsort((w, s))  # flatMap order: spectrum, then window
    out = []
    for k in order:
        j = int(w[k])
        out.append(((int(sf_peak_map[j, 0]), int(sf_peak_map[j, 1])), (int(sp_ids[int(s[k])]), float(v[k]))))
    return LocalRDD(out)


def _coord_list_to_matrix(sp_iter, norm_img_pixel_inds, nrows, ncols):
    """formula_imager.py:41-47."""
    sp_intens_arr = np.array(list(sp_iter), dtype=[("sp", int), ("intens", float)])
    img_array = np.zeros(nrows * ncols)
    pixel_inds = np.asarray(norm_img_pixel_inds)[sp_intens_arr["sp"]]
    img_array[pixel_inds] = sp_intens_arr["intens"]
    return scipy.sparse.csr_matrix(img_array.reshape(nrows, ncols))


def _img_pairs_to_list(pairs):
    """formula_imager.py:50-58."""
    if not pairs:
        return None
    length = max(i for i, _ in pairs) + 1
    res = [None] * length
    for i, img in pairs:
        res[i] = img
    return res


def compute_sf_peak_images(ds, sf_sp_intens):
    nrows, ncols = ds.get_dims()
    pix = ds.get_norm_img_pixel_inds()
    groups = defaultdict(list)
    for key, sp_int in (sf_sp_intens.collect() if hasattr(sf_sp_intens, "collect") else sf_sp_intens):
        groups[key].append(sp_int)
    return LocalRDD((sf_i, (p_i, _coord_list_to_matrix(v, pix, nrows, ncols))) for (sf_i, p_i), v in groups.items())


def compute_sf_images(sf_peak_imgs):
    groups = defaultdict(list)
    for sf_i, pair in (sf_peak_imgs.collect() if hasattr(sf_peak_imgs, "collect") else sf_peak_imgs):
        groups[sf_i].append(pair)
    return LocalRDD((k, _img_pairs_to_list(v)) for k, v in groups.items())
