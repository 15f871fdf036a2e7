"""Ion-image generation: drop-in for sm/engine/msm_basic/formula_imager_segm.py.

``compute_sf_images(sc, ds, sf_peak_df, ppm)`` (reference :142-161) returns an ``IonImageSet``: the images
stay in HBM as (window -> [lo, hi) run of the m/z-sorted hit array) and are materialised as scipy COO
matrices only when a caller iterates them.  Semantics (complete-window):

* window = points with ``mz - mz*ppm*1e-6 <= mz_point <= mz + mz*ppm*1e-6`` (f64 bounds, :79-82);
* an (ion, peak_i) image exists iff its window holds >= 1 point, zero intensities included (:85-86);
* an ion appears iff >= 1 of its images exists; its list has length max(peak_i with image)+1 with
  ``None`` gaps (:95-109); duplicate pixels are summed by ``toarray()``.

The reference's m/z segmentation and chunking (:9-49, :68-69) only partition this same computation
over Spark workers; on one GPU the whole sorted peak list is resident, so neither exists here.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
from scipy.sparse import coo_matrix

from .rdd import LocalRDD


class IonImageSet:
    """Device-resident ``RDD[((sf_id, adduct), [coo | None, ...])]``."""

    def __init__(self, peaks, keys, win_off, peak_i_max, lo, hi, dims, ions_dev, ppm=None):
        self.peaks = peaks              # DevicePeaks (sorted)
        self.ppm = ppm                  # the ppm of the duplicate flags and windows
        self.peaks_version = peaks.version if peaks is not None else 0
        self.keys = keys                # list[(sf_id, adduct)] ion-major
        self.win_off = win_off          # np.int64[n_ion+1]
        self.peak_i_max = peak_i_max    # np.int64[n_ion]: number of windows per ion
        self.lo = lo                    # device int64[n_win]
        self.hi = hi
        self.dims = dims
        self.ions_dev = ions_dev        # engine.DeviceIons (theor filled later)
        self._has = None
        self._sel = None                # optional ion subset (filter_by_keys)

    # ---- bookkeeping -------------------------------------------------------------------------
    def ensure_current(self):
        """Restore the sorted peaks this set was built on if another compute_sf_images (another ppm) re-flagged
        and re-sorted them since: the duplicate-candidate flags must be those of this set's windows.  The sort is
        stable and keyed by m/z only, so re-flagging at this ppm and re-sorting gives back the same positions."""
        p = self.peaks
        if p is not None and (p.version != self.peaks_version or p.flag_ppm != self.ppm):
            p.flag_duplicates(self.ppm)
            p.sort()
            p.prefix_sums()
            self.peaks_version = p.version
        return self

    def _counts(self):
        if self._has is None:
            cnt = (self.hi - self.lo).cpu().numpy()
            self._win_counts = cnt
            has = np.zeros(len(self.keys), dtype=bool)
            nz = np.nonzero(cnt)[0]
            if nz.size:
                owner = np.searchsorted(self.win_off, nz, side="right") - 1
                has[owner] = True
            self._has = has
        return self._win_counts, self._has

    def ion_indices(self):
        _, has = self._counts()
        idx = np.nonzero(has)[0]
        if self._sel is not None:
            idx = idx[self._sel[idx]]
        return idx

    def filter_by_keys(self, index) -> "IonImageSet":
        """Keep ions whose key is in ``index`` without materialising anything (filter_sf_images)."""
        keep = set(index)
        sel = np.array([k in keep for k in self.keys], dtype=bool)
        out = IonImageSet(self.peaks, self.keys, self.win_off, self.peak_i_max, self.lo, self.hi, self.dims,
                          self.ions_dev, self.ppm)
        out.peaks_version = self.peaks_version
        out._has, out._win_counts = self._has, getattr(self, "_win_counts", None)
        out._sel = sel if self._sel is None else (sel & self._sel)
        return out

    # ---- materialisation -----------------------------------------------------------------------
    def materialize(self, ion_idx):
        """[(key, [coo|None...])] for the given ions; gathers only their windows from HBM."""
        import torch
        cnt, _ = self._counts()
        self.ensure_current()
        nrows, ncols = self.dims
        wins = [np.arange(self.win_off[i], self.win_off[i + 1]) for i in ion_idx]
        if not wins:
            return []
        w = np.concatenate(wins)
        c = cnt[w]
        total = int(c.sum())
        out_hits = np.zeros(0, np.uint64)
        if total:
            dev = self.lo.device
            wt = torch.from_numpy(w).to(dev)
            ct = torch.from_numpy(c).to(dev)
            starts = self.lo[wt]
            base = torch.repeat_interleave(starts, ct)
            offs = torch.repeat_interleave(torch.cumsum(ct, 0) - ct, ct)
            idx = base + (torch.arange(total, device=dev) - offs)
            out_hits = self.peaks.hits_sorted[idx].cpu().numpy().view(np.uint64)
        pix = (out_hits & np.uint64(0x7FFFFFFF)).astype(np.int64)
        val = (out_hits >> np.uint64(32)).astype(np.uint32).view(np.float32).astype(np.float64)
        res = []
        pos = 0
        wpos = 0
        for i, ws in zip(ion_idx, wins):
            imgs = []
            for _ in ws:
                n = int(c[wpos])
                if n:
                    p = pix[pos:pos + n]
                    imgs.append(coo_matrix((val[pos:pos + n], (p // ncols, p % ncols)), shape=(nrows, ncols)))
                else:
                    imgs.append(None)
                pos += n
                wpos += 1
            last = max((j for j, m in enumerate(imgs) if m is not None), default=-1)
            res.append((self.keys[i], imgs[:last + 1]))
        return res

    def _items(self):
        return self.materialize(self.ion_indices())

    # ---- RDD surface ---------------------------------------------------------------------------
    def collect(self):
        return self._items()

    def take(self, n):
        return self.materialize(self.ion_indices()[:n])

    def count(self):
        return int(len(self.ion_indices()))

    def map(self, f):
        return LocalRDD(self._items()).map(f)

    def flatMap(self, f):
        return LocalRDD(self._items()).flatMap(f)

    def filter(self, f):
        return LocalRDD(self._items()).filter(f)

    def mapValues(self, f):
        return LocalRDD(self._items()).mapValues(f)

    def foreachPartition(self, f):
        f(iter(self._items()))

    def keys_with_images(self):
        return [self.keys[i] for i in self.ion_indices()]

    def cache(self):
        return self

    def __iter__(self):
        return iter(self._items())


def ion_layout(sf_peak_df: pd.DataFrame, sf_peak_ints: dict | None = None):
    """Ion-major window table from FormulasSegm.get_sf_peak_df rows (sf_id, adduct, peak_i, mz).

    Returns keys, win_off, peak_mz (window m/z, NaN for padding windows), theor ints (or NaN).
    An ion gets max(peak_i)+1 windows, or len(sf_ints) if larger (formula_img_validator.py:73-75 padding).
    """
    df = sf_peak_df[["sf_id", "adduct", "peak_i", "mz"]]
    keys_arr = list(zip(df.sf_id.tolist(), df.adduct.tolist()))
    codes, uniq = pd.factorize(pd.Series(keys_arr, dtype=object), sort=False)
    order = sorted(range(len(uniq)), key=lambda j: (uniq[j][0], str(uniq[j][1])))
    remap = np.empty(len(uniq), np.int64)
    remap[order] = np.arange(len(uniq))
    ion = remap[codes]
    keys = [tuple(uniq[j]) for j in order]
    pk = df.peak_i.to_numpy().astype(np.int64)
    K = np.zeros(len(keys), np.int64)
    np.maximum.at(K, ion, pk + 1)
    if sf_peak_ints is not None:
        K = np.maximum(K, np.array([len(sf_peak_ints[k]) for k in keys], dtype=np.int64))
    win_off = np.zeros(len(keys) + 1, np.int64)
    np.cumsum(K, out=win_off[1:])
    peak_mz = np.full(int(win_off[-1]), np.nan)
    slot = win_off[ion] + pk
    if len(np.unique(slot)) != len(slot):
        raise AssertionError("duplicate (sf_id, adduct, peak_i) rows in sf_peak_df")
    peak_mz[slot] = df.mz.to_numpy(np.float64)
    theor = np.full(int(win_off[-1]), np.nan)
    if sf_peak_ints is not None:
        for i, k in enumerate(keys):
            v = sf_peak_ints[k]
            theor[win_off[i]:win_off[i] + len(v)] = v
    return keys, win_off, peak_mz, theor


def compute_sf_images(sc, ds, sf_peak_df, ppm):
    """formula_imager_segm.py:142-161.  ``sc`` is accepted for signature compatibility and ignored."""
    from .engine import DeviceIons, DevicePeaks, window_bounds
    from .dataset import spectra_from_duck
    if hasattr(ds, "device_peaks"):
        peaks = ds.device_peaks()
    else:
        off, mz, it = spectra_from_duck(ds)
        peaks = DevicePeaks.from_arrays(off, mz, it, np.asarray(ds.norm_img_pixel_inds), ds.get_dims())
    peaks.flag_duplicates(ppm)
    peaks.sort()
    keys, win_off, peak_mz, _ = ion_layout(sf_peak_df)
    # padding windows (NaN m/z) must stay empty: give them an m/z no point can match
    pm = np.where(np.isnan(peak_mz), -1.0, peak_mz)
    dions = DeviceIons.from_arrays(win_off, pm, np.zeros_like(pm), device=peaks.device)
    lo, hi = window_bounds(peaks, dions, ppm)
    return IonImageSet(peaks, keys, win_off, np.diff(win_off), lo, hi, ds.get_dims(), dions, ppm)
