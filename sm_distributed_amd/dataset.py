"""Dataset duck type of the hot path (sm/engine/dataset.py:16-150 surface) backed by HBM.

The reference Dataset parses ``ds.txt`` into an RDD of ``(sp_id, mz f32[], int f64[])`` and builds the
row-major pixel map from the coordinate file (dataset.py:52-85, :106-120).  ``DeviceDataset`` keeps the
same accessors (``get_spectra``, ``norm_img_pixel_inds``, ``get_norm_img_pixel_inds``, ``get_dims``) and adds
``device_peaks()``: the resident m/z + packed-hit layout the kernels read (no text round trip).
"""
from __future__ import annotations

import numpy as np

from .rdd import LocalRDD
from .synthetic import SpectraSet, pixel_map_from_coords


class DeviceDataset:
    def __init__(self, spectra: SpectraSet, device="cuda"):
        self.spectra = spectra
        self.device = device
        self.norm_img_pixel_inds, dims = pixel_map_from_coords(spectra.coords)
        self._dims = dims
        c = np.asarray(spectra.coords)
        self.min_x, self.min_y = c.min(axis=0)
        self.max_x, self.max_y = c.max(axis=0)
        self._peaks = None

    # --- reference accessors -----------------------------------------------------------------
    def get_norm_img_pixel_inds(self):
        """dataset.py:68-75."""
        return self.norm_img_pixel_inds

    def get_dims(self):
        """dataset.py:77-85: (nrows, ncols)."""
        return self._dims

    def get_spectra(self):
        """dataset.py:110-120 (host view; the device path uses device_peaks())."""
        return LocalRDD(self.spectra.spectra())

    # --- device layout -------------------------------------------------------------------------
    def device_peaks(self):
        if self._peaks is None:
            from .engine import DevicePeaks
            s = self.spectra
            self._peaks = DevicePeaks.from_arrays(s.sp_off, s.mz, s.ints, self.norm_img_pixel_inds, self._dims,
                                                  device=self.device)
        return self._peaks

    @classmethod
    def from_spectra_list(cls, spectra, coords, device="cuda"):
        """Build from ``[(sp_id, mzs, ints), ...]`` in sp_id order and 1-based ``coords[sp_id] = (x, y)``."""
        spectra = sorted(spectra, key=lambda t: t[0])
        off = np.zeros(len(spectra) + 1, np.int64)
        mzs, its = [], []
        for i, (_, mz, it) in enumerate(spectra):
            mzs.append(to_f32(mz, "m/z"))
            its.append(to_f32(it, "intensity"))
            off[i + 1] = off[i] + len(mzs[-1])
        mz = np.concatenate(mzs) if mzs else np.zeros(0, np.float32)
        it = np.concatenate(its) if its else np.zeros(0, np.float32)
        return cls(SpectraSet(sp_off=off, mz=mz, ints=it, coords=np.asarray(coords)), device=device)

    @classmethod
    def from_imzml(cls, imzml_path, device="cuda"):
        from .imzml import read_imzml
        return cls(read_imzml(imzml_path), device=device)


_WARNED = set()


def to_f32(a, what):
    """``a`` as float32 (the resident format).  A lossy narrowing (f64 values that are not f32 values) is reported
    once per quantity: intensities change by <= 6e-8 relative (inside the 1e-6 / 1e-5 tolerances), but an m/z
    within that distance of a window bound can land on the other side of it."""
    src = np.asarray(a)
    out = src.astype(np.float32, copy=False)
    if src.dtype != np.float32 and what not in _WARNED and src.size and not np.array_equal(out, src):
        import warnings
        _WARNED.add(what)
        warnings.warn(f"{what}: {src.dtype} values rounded to float32 (resident format); relative change <= 6e-8",
                      RuntimeWarning, stacklevel=3)
    return out


def spectra_from_duck(ds):
    """Collect any reference-style dataset (get_spectra RDD + pixel map + dims) into a SpectraSet-like tuple."""
    items = ds.get_spectra().collect()
    items = sorted(items, key=lambda t: t[0])
    n = (max(t[0] for t in items) + 1) if items else 0
    off = np.zeros(n + 1, np.int64)
    mzs = [np.zeros(0, np.float32)] * n
    its = [np.zeros(0, np.float32)] * n
    for sp_id, mz, it in items:
        mzs[sp_id] = to_f32(mz, "m/z")
        its[sp_id] = to_f32(it, "intensity")
    for i in range(n):
        off[i + 1] = off[i] + len(mzs[i])
    mz = np.concatenate(mzs) if n else np.zeros(0, np.float32)
    it = np.concatenate(its) if n else np.zeros(0, np.float32)
    return off, mz, it


class ResidentDataset:
    """A dataset already resident in HBM (e.g. generated there, or loaded by another rank's reader): the same
    accessors as DeviceDataset over a DevicePeaks.  ``pixel_map`` defaults to the identity (spectrum i is
    pixel i, the row-major grid of dataset.py:52-66)."""

    def __init__(self, peaks, pixel_map=None):
        self._peaks = peaks
        self._dims = (peaks.nrows, peaks.ncols)
        n_sp = int(peaks.sp_off.numel()) - 1 if peaks.sp_off is not None else peaks.nrows * peaks.ncols
        self.norm_img_pixel_inds = (np.arange(n_sp, dtype=np.int32) if pixel_map is None
                                    else np.asarray(pixel_map, dtype=np.int32))

    def device_peaks(self):
        return self._peaks

    def get_norm_img_pixel_inds(self):
        return self.norm_img_pixel_inds

    def get_dims(self):
        return self._dims

    def get_spectra(self):
        raise NotImplementedError("ResidentDataset holds device arrays only")
