"""Theoretical isotope peaks: drop-in for sm/engine/isocalc_wrapper.py.

``IsocalcWrapper`` keeps the reference's constructor (the ``isotope_generation`` section of a dataset config),
``isotope_peaks(sf, adduct) -> Centroids`` (first six centroids, empty lists on an invalid formula,
isocalc_wrapper.py:42-70), ``slice_array``, ``_format_peak_str`` / ``formatted_iso_peaks`` (the tab-separated
theor_peaks row, :76-106).  The calculator behind it is native (``smg_isotope_centroids`` in libsmg.so, host
code): the reference called the third-party cpyMSpec ``complete_isodist``, which is not available here, so its
arithmetic is restated (oracle/isocalc_oracle.py, parity unpinned).  ``isotope_peaks_batch`` computes many
(sf, adduct) pairs on all host cores in one call (the Spark fan-out of theor_peaks_gen.py:129-133).
"""
from __future__ import annotations

import ctypes
import logging
from collections import namedtuple

import numpy as np

from . import _lib

logger = logging.getLogger("sm_distributed_amd")

Centroids = namedtuple("Centroids", ["mzs", "ints"])

WEIGHTED_BINS = 5   # centroid_kwargs={'weighted_bins': 5} (isocalc_wrapper.py:40)
MAX_PEAKS = 6       # l[:6] (isocalc_wrapper.py:62)


def list_of_floats_to_str(l):
    """isocalc_wrapper.py:14-15."""
    return ",".join("{:.6f}".format(x) for x in l)


class IsocalcWrapper(object):
    """Theoretical isotope centroids of (sum formula, adduct) pairs (isocalc_wrapper.py:18-106)."""

    def __init__(self, isocalc_config):
        self.charge = 0
        if "polarity" in isocalc_config["charge"]:
            polarity = isocalc_config["charge"]["polarity"]
            self.charge = (-1 if polarity == "-" else 1) * isocalc_config["charge"]["n_charges"]
        self.sigma = isocalc_config["isocalc_sigma"]
        self.pts_per_mz = isocalc_config["isocalc_pts_per_mz"]
        self.prof_pts_per_centr = 6

    def _isodist(self, sf_adduct: str, cap: int = 256):
        """All centroids (mzs, ints) of one formula string in m/z order; raises ValueError when invalid."""
        lib = _lib.lib()
        while True:
            mzs = np.empty(cap, dtype=np.float64)
            ints = np.empty(cap, dtype=np.float64)
            n = ctypes.c_int32(0)
            rc = lib.smg_isotope_centroids(sf_adduct.encode(), int(self.charge), float(self.sigma),
                                           int(self.pts_per_mz), WEIGHTED_BINS, cap, mzs.ctypes.data,
                                           ints.ctypes.data, ctypes.byref(n))
            if rc != _lib.SMG_OK:
                raise ValueError(lib.smg_last_error().decode(errors="replace"))
            if n.value < cap:
                return mzs[:n.value], ints[:n.value]
            cap *= 4

    def isotope_peaks(self, sf, adduct):
        """First six centroids of ``sf + adduct``; ``Centroids([], [])`` on any error (isocalc_wrapper.py:42-70)."""
        centroids = Centroids([], [])
        try:
            if not isinstance(sf, str) or not isinstance(adduct, str):
                raise TypeError("sum formula and adduct must be strings, got {!r}, {!r}".format(sf, adduct))
            lib = _lib.lib()
            mzs = np.empty(MAX_PEAKS, dtype=np.float64)
            ints = np.empty(MAX_PEAKS, dtype=np.float64)
            n = ctypes.c_int32(0)
            rc = lib.smg_isotope_centroids((sf + adduct).encode(), int(self.charge), float(self.sigma),
                                           int(self.pts_per_mz), WEIGHTED_BINS, MAX_PEAKS, mzs.ctypes.data,
                                           ints.ctypes.data, ctypes.byref(n))
            if rc != _lib.SMG_OK:
                logger.warning("(%s, %s) - %s", sf, adduct, lib.smg_last_error().decode(errors="replace"))
            else:
                centroids = Centroids(mzs[:n.value], ints[:n.value])
        except _lib.SmgLibraryError:
            raise  # the native calculator is the product path: no silent fallback
        except Exception as e:
            logger.error("(%s, %s) - %s", sf, adduct, e)
        return centroids

    def isotope_peaks_batch(self, pairs, n_threads: int = 0):
        """``[isotope_peaks(sf, adduct) for sf, adduct in pairs]`` on ``n_threads`` host threads (0 = all)."""
        pairs = list(pairs)
        out = [Centroids([], [])] * len(pairs)
        ok = [i for i, (sf, a) in enumerate(pairs) if isinstance(sf, str) and isinstance(a, str)]
        if not ok:
            return out
        raw = [(pairs[i][0] + pairs[i][1]).encode() for i in ok]
        offs = np.zeros(len(raw) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(r) for r in raw])
        buf = ctypes.create_string_buffer(b"".join(raw), int(offs[-1]) + 1)
        mzs = np.empty((len(raw), MAX_PEAKS), dtype=np.float64)
        ints = np.empty((len(raw), MAX_PEAKS), dtype=np.float64)
        n_out = np.empty(len(raw), dtype=np.int32)
        _lib.check(_lib.lib().smg_isotope_centroids_batch(
            ctypes.addressof(buf), offs.ctypes.data, len(raw), int(self.charge), float(self.sigma),
            int(self.pts_per_mz), WEIGHTED_BINS, MAX_PEAKS, mzs.ctypes.data, ints.ctypes.data, n_out.ctypes.data,
            int(n_threads)), "smg_isotope_centroids_batch")
        for j, i in enumerate(ok):
            if n_out[j] < 0:
                logger.warning("(%s, %s) - invalid sum formula", *pairs[i])
            else:
                out[i] = Centroids(mzs[j, :n_out[j]].copy(), ints[j, :n_out[j]].copy())
        return out

    @staticmethod
    def slice_array(mzs, lower, upper):
        """isocalc_wrapper.py:72-74."""
        return np.hstack([mzs[l:u] for l, u in zip(lower, upper)])

    def _format_peak_str(self, db_id, sf_id, adduct, centroids):
        """isocalc_wrapper.py:76-84: one theor_peaks row (profile columns empty)."""
        return "%d\t%d\t%s\t%.6f\t%d\t%d\t{%s}\t{%s}\t{%s}\t{%s}" % (
            db_id, sf_id, adduct,
            round(self.sigma, 6), self.charge, self.pts_per_mz,
            list_of_floats_to_str(centroids.mzs),
            list_of_floats_to_str(centroids.ints),
            "",
            "",
        )

    def formatted_iso_peaks(self, db_id, sf_id, sf, adduct):
        """isocalc_wrapper.py:86-106: yields the row if the pattern is non-empty."""
        centroids = self.isotope_peaks(sf, adduct)
        if len(centroids.mzs) > 0:
            yield self._format_peak_str(db_id, sf_id, adduct, centroids)
