"""CPU oracle: a numpy/scipy restatement of SM_distributed's molecule-annotation hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``sm_distributed_amd`` imports this module.  It may be
used by ``tests/``, ``__graft_entry__.smoke()`` (as the checker) and ``bench.py``'s
``cpu_baseline`` leg (as the timed CPU port of the reference algorithm) -- never as the thing
measured for ``value`` and never as a fallback of the product path.

What it restates (citations are ``path:line`` under the reference repository):

* ion-image generation, live segmented imager -- ``sm/engine/msm_basic/formula_imager_segm.py``
  ``_gen_iso_images`` :66-92 (sort by m/z, f64 bounds ``mz - mz*ppm*1e-6``, inclusive
  searchsorted window, one COO per window with >=1 point, zero intensities included, pixel =
  ``pixel_map[sp_id]``, row = pix // ncols, col = pix % ncols) and ``_img_pairs_to_list``
  :95-109 (per peak_i keep the COO with larger nnz, ``None`` gaps, length max(peak_i)+1).
  Parity is defined on *complete-window* semantics: one chunk covering every spectrum
  (SURVEY.md §8a hazard H1), which is what the reference computes whenever
  ``int(1e7 / peaks_per_sp_segm) >= n_spectra``.
* legacy imager ``sm/engine/msm_basic/formula_imager.py`` :9-123 (prefix-sum window sums kept
  only if > 0.001; images built by assignment).
* image metrics ``sm/engine/msm_basic/formula_img_validator.py`` :58-122 (padding with the empty
  matrix, evaluation order spectral / spatial / chaos, ``isclose(moc, 1) -> 0``, NaN/inf/None/0
  -> 0, msm = chaos*spatial*spectral, DataFrame indexed by [sf_id, adduct]).
* the third-party metric functions it calls, restated from the published packages because they
  are NOT in /root/reference (parity for their arithmetic is therefore *unpinned*; see
  DESIGN.md §Oracle):
    - ``pyImagingMSpec==0.1.1  isotope_pattern_match``  (called formula_img_validator.py:80)
    - ``pyImagingMSpec==0.1.1  isotope_image_correlation`` (called :81)
    - ``cpyImagingMSpec==0.0.4 measure_of_chaos`` (C++ via cffi, called :82), restated from the
      pyImagingMSpec python version that the C++ ports.  Frozen choices: levels =
      ``np.linspace(0, 1, nlevels)``, ``B = im/max(im) > level``, binary dilation with the 4-cross,
      binary erosion with the 3x3 box (scipy ``border_value=0``), 4-connected components,
      ``chaos = 1 - sum(counts)/(nlevels * #(im > 0))``, NaN when ``sum(im) <= 0`` or
      ``#(im > 0) < 4``.  ``connectivity`` / ``erosion_border`` are exposed so a future pin of
      the C++ can be matched by a switch.
* FDR ``sm/engine/fdr.py`` :42-88 (for the "identical annotations at FDR 0.1" check).
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import pandas as pd
from scipy import ndimage
from scipy.sparse import coo_matrix

# --------------------------------------------------------------------------------------------
# imaging (formula_imager_segm.py)
# --------------------------------------------------------------------------------------------


def window_bounds(mz, ppm):
    """formula_imager_segm.py:79-80 -- ``mz - mz*ppm*1e-6`` / ``mz + mz*ppm*1e-6`` in float64."""
    mz = np.asarray(mz, dtype=np.float64)
    d = mz * ppm * 1e-6  # evaluated left to right as in the reference lambda
    return mz - d, mz + d


def flatten_spectra(spectra, pixel_map):
    """``_sp_df_gen`` (formula_imager_segm.py:60-63): one (pixel, mz f32, int f64) row per point."""
    pix, mzs, ints = [], [], []
    pixel_map = np.asarray(pixel_map)
    for sp_id, mz, it in spectra:
        mz = np.asarray(mz, dtype=np.float32)
        pix.append(np.full(mz.shape[0], pixel_map[sp_id], dtype=np.int64))
        mzs.append(mz)
        ints.append(np.asarray(it, dtype=np.float64))
    if not pix:
        return (np.zeros(0, np.int64), np.zeros(0, np.float32), np.zeros(0, np.float64))
    return np.concatenate(pix), np.concatenate(mzs), np.concatenate(ints)


def sort_points(pix, mz, ints):
    """formula_imager_segm.py:73-74 -- rows sorted by m/z (the reference sort is not stable, H3)."""
    order = np.argsort(mz, kind="stable")
    return pix[order], mz[order], ints[order]


def gen_iso_images(pix_s, mz_s, int_s, sf_ids, adducts, peak_is, peak_mzs, nrows, ncols, ppm):
    """formula_imager_segm.py:66-92 on a single chunk holding every spectrum.

    Yields ``((sf_id, adduct), (peak_i, coo_matrix))`` for every window with >= 1 point.
    ``searchsorted`` compares the f32 m/z column against f64 bounds in f64 (numpy promotion),
    i.e. the window is ``lower <= mz <= upper``.
    """
    if mz_s.shape[0] == 0:
        return
    lower, upper = window_bounds(peak_mzs, ppm)
    mz64 = mz_s.astype(np.float64)
    lo = np.searchsorted(mz64, lower, "left")
    hi = np.searchsorted(mz64, upper, "right")
    for i in range(len(peak_mzs)):
        l, u = lo[i], hi[i]
        if u - l >= 1:
            idx = pix_s[l:u]
            data = int_s[l:u]
            img = coo_matrix((data, (idx // ncols, idx % ncols)), shape=(nrows, ncols))
            yield (sf_ids[i], adducts[i]), (int(peak_is[i]), img)


def img_pairs_to_list(pairs, shape):
    """formula_imager_segm.py:95-109 -- duplicate peak_i: keep the COO with the larger nnz."""
    if not pairs:
        return None
    d = defaultdict(lambda: coo_matrix(shape))
    for k, m in pairs:
        _m = d[k]
        d[k] = _m if _m.nnz >= m.nnz else m
    res = [None] * (max(d.keys()) + 1)
    for i, m in d.items():
        res[i] = m
    return res


def compute_sf_images(spectra, pixel_map, dims, sf_peak_df, ppm):
    """formula_imager_segm.py:142-161 with complete-window semantics.

    ``sf_peak_df``: DataFrame with columns sf_id, adduct, peak_i, mz (as FormulasSegm.get_sf_peak_df,
    formulas_segm.py:61-63).  Returns ``dict[(sf_id, adduct)] -> list[coo | None]``.
    """
    nrows, ncols = dims
    pix, mz, ints = flatten_spectra(spectra, pixel_map)
    pix_s, mz_s, int_s = sort_points(pix, mz, ints)
    df = sf_peak_df.sort_values(by="mz", kind="stable")
    groups = defaultdict(list)
    for key, pair in gen_iso_images(pix_s, mz_s, int_s, df.sf_id.values, df.adduct.values,
                                    df.peak_i.values, df.mz.values, nrows, ncols, ppm):
        groups[key].append(pair)
    return {k: img_pairs_to_list(v, (nrows, ncols)) for k, v in groups.items()}


def window_ranges(mz_sorted, peak_mzs, ppm):
    """The searchsorted pair of formula_imager_segm.py:81-82 (inclusive window), as index ranges."""
    lower, upper = window_bounds(peak_mzs, ppm)
    mz64 = np.asarray(mz_sorted).astype(np.float64)
    return (np.searchsorted(mz64, lower, "left").astype(np.int64),
            np.searchsorted(mz64, upper, "right").astype(np.int64))


# --------------------------------------------------------------------------------------------
# legacy imager (formula_imager.py) -- pinned by test_formula_imager.py KATs
# --------------------------------------------------------------------------------------------


def legacy_peak_bounds(peak_mzs, ppm):
    """formulas.py:70-71 -- the legacy expression ``mz - ppm*mz/1e6``."""
    mz = np.asarray(peak_mzs, dtype=np.float64)
    return mz - ppm * mz / 1e6, mz + ppm * mz / 1e6


def sample_spectrum(sp, lower, upper, sf_peak_map):
    """formula_imager.py:9-38 -- window sums from cumulative ints, kept when > 0.001."""
    sp_i, mzs, cum_ints = sp
    mzs = np.asarray(mzs)
    cum_ints = np.asarray(cum_ints, dtype=np.float64)
    ints = cum_ints[mzs.searchsorted(upper, "right")] - cum_ints[mzs.searchsorted(lower, "left")]
    keep = ints > 0.001
    inds = np.arange(len(lower))[keep]
    sf_peak_map = np.asarray(sf_peak_map)
    return [((int(sf_peak_map[j, 0]), int(sf_peak_map[j, 1])), (sp_i, float(v)))
            for j, v in zip(inds, ints[keep])]


def sample_spectra(spectra, lower, upper, sf_peak_map):
    """formula_imager.py:62-80 (flatMap over spectra)."""
    out = []
    for sp in spectra:
        out.extend(sample_spectrum(sp, lower, upper, sf_peak_map))
    return out


def coord_list_to_matrix(sp_intens, pixel_map, nrows, ncols):
    """formula_imager.py:41-47 -- assignment (not sum) into a dense image, then CSR."""
    from scipy.sparse import csr_matrix
    img = np.zeros(nrows * ncols)
    sp = np.array([s for s, _ in sp_intens], dtype=np.int64)
    it = np.array([v for _, v in sp_intens], dtype=np.float64)
    img[np.asarray(pixel_map)[sp]] = it
    return csr_matrix(img.reshape(nrows, ncols))


# --------------------------------------------------------------------------------------------
# image metrics (formula_img_validator.py + restated third-party functions)
# --------------------------------------------------------------------------------------------


def isotope_pattern_match(images_flat, theor_iso_intensities):
    """pyImagingMSpec 0.1.1 ``isotope_pattern_match`` (restated; unpinned)."""
    t = np.asarray(theor_iso_intensities, dtype=np.float64)
    if len(images_flat) != len(t):
        raise ValueError("amount of images and theoretical intensities must be equal")
    not_null = images_flat[0] > 0
    image_ints = np.array([np.sum(images_flat[i][not_null]) for i in range(len(t))], dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        pattern_match = 1 - np.mean(np.abs(t / np.linalg.norm(t) - image_ints / np.linalg.norm(image_ints)))
    if pattern_match == 1.0:
        return 0
    return pattern_match


def isotope_image_correlation(images_flat, weights=None):
    """pyImagingMSpec 0.1.1 ``isotope_image_correlation`` (restated; unpinned).

    Pearson correlation of each isotope image with the principal one over ALL pixels (zeros
    included), inf -> 0, weighted average with ``weights`` (= theoretical ints[1:]).
    A constant image gives NaN, which propagates (and is turned into 0 by ImgMeasures).
    """
    if len(images_flat) < 2:
        return 0
    with np.errstate(divide="ignore", invalid="ignore"):
        iso_correlation = np.corrcoef(np.asarray(images_flat))[1:, 0]
    iso_correlation[np.isinf(iso_correlation)] = 0
    return np.average(iso_correlation, weights=weights)


CROSS = np.array([[0, 1, 0], [1, 1, 1], [0, 1, 0]], dtype=bool)
BOX = np.ones((3, 3), dtype=bool)


def measure_of_chaos(im, nlevels, connectivity=4, erosion_border=0):
    """cpyImagingMSpec 0.0.4 ``measure_of_chaos`` (restated from the pyImagingMSpec python version; unpinned).

    Per level: threshold the max-normalised image, dilate with the 4-cross, erode with the 3x3
    box, count connected components.  Independent of the GPU formulation (which uses grayscale
    morphology + a Kruskal pass), so agreement between the two is a real cross-check.
    """
    im = np.array(im, dtype=np.float64, copy=True)
    im[np.isnan(im)] = 0
    if np.sum(im) <= 0:
        return np.nan
    sum_notnull = int(np.sum(im > 0))
    if sum_notnull < 4:
        return np.nan
    im_clean = im / np.max(im)
    label_struct = CROSS if connectivity == 4 else BOX
    counts = []
    for lev in np.linspace(0, 1, nlevels):
        bw = im_clean > lev
        bw = ndimage.binary_dilation(bw, structure=CROSS, border_value=0)
        bw = ndimage.binary_erosion(bw, structure=BOX, border_value=erosion_border)
        counts.append(ndimage.label(bw, structure=label_struct)[1])
    return 1 - float(np.sum(counts)) / nlevels / float(sum_notnull)


def replace_nan(v, new_v=0):
    """ImgMeasures._replace_nan, formula_img_validator.py:32-36."""
    if v is None or not v or np.isinf(v) or np.isnan(v):
        return new_v
    return v


def quantile_clip(img, q):
    """Gated hot-spot clip (``image_generation.do_preprocessing``/``q``; never read by the reference,
    SURVEY.md §5): clamp every pixel above the q-th percentile of the image's positive pixels."""
    img = np.array(img, dtype=np.float64, copy=True)
    pos = img[img > 0]
    if pos.size == 0:
        return img
    thr = np.percentile(pos, q)
    img[img > thr] = thr
    return img


def compute_img_metrics(iso_images_sparse, sf_ints, nrows, ncols, nlevels, q=99.0,
                        do_preprocessing=False, connectivity=4, erosion_border=0):
    """formula_img_validator.py:72-84 ``compute``: returns the cleaned (chaos, spatial, spectral)."""
    empty = np.zeros((nrows, ncols))
    iso_images_sparse = list(iso_images_sparse)
    diff = len(sf_ints) - len(iso_images_sparse)
    iso_imgs = [empty if img is None else np.asarray(img.toarray(), dtype=np.float64)
                for img in iso_images_sparse + [None] * diff]
    if do_preprocessing:
        iso_imgs = [quantile_clip(img, q) for img in iso_imgs]
    iso_imgs_flat = [img.flat[:] for img in iso_imgs]
    chaos, spatial, spectral = 0, 0, 0
    if len(iso_imgs) > 0:
        spectral = isotope_pattern_match(iso_imgs_flat, sf_ints)
        spatial = isotope_image_correlation(iso_imgs_flat, weights=sf_ints[1:])
        moc = measure_of_chaos(iso_imgs[0], nlevels, connectivity, erosion_border)
        chaos = 0 if np.isclose(moc, 1.0) else moc
    return replace_nan(chaos), replace_nan(spatial), replace_nan(spectral)


def sf_image_metrics(sf_images, sf_peak_ints, nrows, ncols, nlevels, **kw):
    """formula_img_validator.py:93-122 -- one row per ion present in ``sf_images``."""
    rows = []
    for (sf, adduct), imgs in sf_images.items():
        rows.append((sf, adduct) + tuple(compute_img_metrics(imgs, sf_peak_ints[(sf, adduct)],
                                                            nrows, ncols, nlevels, **kw)))
    df = pd.DataFrame(rows, columns=["sf_id", "adduct", "chaos", "spatial", "spectral"])
    df = df.astype({"chaos": np.float64, "spatial": np.float64, "spectral": np.float64})
    df = df.set_index(["sf_id", "adduct"])
    df["msm"] = df.chaos * df.spatial * df.spectral
    return df


# --------------------------------------------------------------------------------------------
# FDR (fdr.py) -- for the annotation-parity check
# --------------------------------------------------------------------------------------------


def msm_fdr_map(target_msm, decoy_msm):
    """fdr.py:50-58."""
    target_hits = pd.Series(target_msm.msm.value_counts(), name="target")
    decoy_hits = pd.Series(decoy_msm.msm.value_counts(), name="decoy")
    msm_df = pd.concat([target_hits, decoy_hits], axis=1).fillna(0).sort_index(ascending=False)
    msm_df["target_cum"] = msm_df.target.cumsum()
    msm_df["decoy_cum"] = msm_df.decoy.cumsum()
    msm_df["fdr"] = msm_df.decoy_cum / msm_df.target_cum
    return msm_df.fdr


def digitize_fdr(fdr_df, fdr_levels):
    """fdr.py:60-68."""
    df = fdr_df.copy().sort_values(by="msm", ascending=False)
    msm_levels = [df[df.fdr < thr].msm.min() for thr in fdr_levels]
    df["fdr_d"] = 1.0
    for msm_thr, fdr_thr in zip(msm_levels, fdr_levels):
        row_mask = np.isclose(df.fdr_d, 1.0) & np.greater_equal(df.msm, msm_thr)
        df.loc[row_mask, "fdr_d"] = fdr_thr
    df["fdr"] = df.fdr_d
    return df.drop("fdr_d", axis=1)


def estimate_fdr(msm_df, td_df, target_adducts, decoy_sample_size, fdr_levels=(0.05, 0.1, 0.2, 0.5)):
    """fdr.py:70-88."""
    out = []
    for ta in target_adducts:
        target_msm = msm_df.loc(axis=0)[:, ta]
        fdr_list = []
        sub = td_df[td_df.ta == ta][["sf_id", "da"]]
        for i in range(decoy_sample_size):
            sf_da_list = list(map(tuple, sub[i::decoy_sample_size].values))
            decoy_msm = msm_df.loc[sf_da_list]
            fdr_list.append(msm_fdr_map(target_msm, decoy_msm))
        msm_fdr_avg = pd.Series(pd.concat(fdr_list, axis=1).median(axis=1), name="fdr")
        target_fdr = digitize_fdr(target_msm.join(msm_fdr_avg, on="msm"), list(fdr_levels))
        out.append(target_fdr.drop("msm", axis=1))
    return pd.concat(out, axis=0)
