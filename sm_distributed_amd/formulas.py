"""Theoretical-peak tables: the data contract of sm/engine/formulas_segm.py (and legacy formulas.py).

``FormulasSegm`` exposes what the hot path consumes (formulas_segm.py:56-79): ``sf_df`` with columns
(sf_id, adduct, centr_mzs, centr_ints) sorted by (sf_id, adduct), ``get_sf_peak_df`` (one row per
theoretical peak, sorted by mz), ``get_sf_peak_ints`` ({(sf_id, adduct): ints}),
``get_sf_adduct_sorted_df`` and ``get_sf_adduct_peaksn``.  The Postgres load (:25-47) is out of scope:
construct from a DataFrame, an ``IonTable`` or flat arrays instead.

At ~1M ions the reference's representation (a DataFrame of Python lists, a dict of 1M tuples) costs seconds
per access, so the table is held columnar -- ion-major flat arrays, ions sorted by (sf_id, adduct) -- and
the accessors are built from it without per-ion Python work:

* ``get_sf_peak_df`` carries ``adduct`` as a pandas Categorical (string categories, sorted), so the device
  layout of compute_sf_images reads integer codes instead of hashing 5M strings;
* ``get_sf_peak_ints`` returns a ``PeakInts`` read-only mapping with the dict interface the reference uses
  (``sf_ints[(sf_id, adduct)]``) whose flat arrays sf_image_metrics aligns on the device.

Legacy ``Formulas`` (formulas.py) adds ``get_sf_peak_bounds`` (mz -/+ ppm*mz/1e6) and ``get_sf_peak_map``.
"""
from __future__ import annotations

from collections.abc import Mapping

import numpy as np
import pandas as pd


class PeakInts(Mapping):
    """{(sf_id, adduct): [theoretical intensities]} backed by flat arrays (formulas_segm.py:68-69).

    ``sf_ids`` int64[n], ``adduct_codes`` int32[n] into ``adducts`` (sorted unique strings), ions sorted by
    (sf_id, adduct); ion i's intensities are ``values[off[i]:off[i+1]]``.
    """

    def __init__(self, sf_ids, adduct_codes, adducts, off, values):
        self.sf_ids = sf_ids
        self.adduct_codes = adduct_codes
        self.adducts = adducts
        self.off = off
        self.values = values
        self._index = None

    def _lookup(self):
        if self._index is None:
            ad = np.asarray(self.adducts, dtype=object)[self.adduct_codes]
            self._index = {k: i for i, k in enumerate(zip(self.sf_ids.tolist(), ad.tolist()))}
        return self._index

    def __getitem__(self, key):
        i = self._lookup()[key]
        return self.values[self.off[i]:self.off[i + 1]].tolist()

    def __iter__(self):
        return iter(self._lookup())

    def __len__(self):
        return len(self.sf_ids)

    def __contains__(self, key):
        return key in self._lookup()


def _sorted_categories(values):
    """(codes int32, sorted unique strings) of an adduct column."""
    codes, uniq = pd.factorize(pd.Series(values, dtype=object), sort=True)
    if (codes < 0).any():
        raise ValueError("missing adduct")
    return codes.astype(np.int32), [str(u) for u in uniq]


class FormulasSegm(object):
    def __init__(self, sf_df: pd.DataFrame, ppm: float = 2.0):
        """From the reference's list-column table (sf_id, adduct, centr_mzs, centr_ints)."""
        df = sf_df[["sf_id", "adduct", "centr_mzs", "centr_ints"]]
        K = np.array([len(m) for m in df.centr_mzs], dtype=np.int64)
        if (np.array([len(t) for t in df.centr_ints], dtype=np.int64) != K).any():
            raise ValueError("centr_mzs and centr_ints lengths differ")
        mz = np.concatenate([np.asarray(m, np.float64) for m in df.centr_mzs]) if len(df) else np.zeros(0)
        it = np.concatenate([np.asarray(t, np.float64) for t in df.centr_ints]) if len(df) else np.zeros(0)
        off = np.zeros(len(df) + 1, np.int64)
        np.cumsum(K, out=off[1:])
        self._init_columns(df.sf_id.to_numpy(), df.adduct.to_numpy(dtype=object), off, mz, it, ppm)

    @classmethod
    def from_arrays(cls, sf_ids, adducts, win_off, peak_mz, peak_int, ppm=2.0):
        """Ion-major flat arrays: ion i = (sf_ids[i], adducts[i]) with peaks [win_off[i], win_off[i+1])."""
        self = cls.__new__(cls)
        self._init_columns(np.asarray(sf_ids), np.asarray(adducts, dtype=object), np.asarray(win_off, np.int64),
                           np.asarray(peak_mz, np.float64), np.asarray(peak_int, np.float64), ppm)
        return self

    @classmethod
    def from_ion_table(cls, ions, ppm=2.0):
        return cls.from_arrays(ions.sf_ids, ions.adducts, ions.win_off, ions.peak_mz, ions.peak_int, ppm)

    def _init_columns(self, sf_ids, adducts, off, mz, it, ppm):
        self.ppm = ppm
        codes, cats = _sorted_categories(adducts)
        if sf_ids.dtype.kind not in "iu":
            raise ValueError("sf_id must be integer")
        sf_ids = sf_ids.astype(np.int64)
        order = np.lexsort((codes, sf_ids))  # formulas_segm.py:47: sort_values(['sf_id', 'adduct'])
        K = np.diff(off)
        if not (order == np.arange(len(order))).all():
            sf_ids, codes, Ko = sf_ids[order], codes[order], K[order]
            noff = np.zeros(len(Ko) + 1, np.int64)
            np.cumsum(Ko, out=noff[1:])
            sel = np.repeat(off[:-1][order], Ko) + np.arange(noff[-1]) - np.repeat(noff[:-1], Ko)
            mz, it, off = mz[sel], it[sel], noff
        # formulas_segm.py:49-53
        dup = (sf_ids[1:] == sf_ids[:-1]) & (codes[1:] == codes[:-1])
        assert not dup.any(), "Not unique formula-adduct combinations {} != {}".format(
            len(sf_ids) - int(dup.sum()), len(sf_ids))
        self.ion_sf = sf_ids
        self.ion_adduct_code = codes
        self.adducts = cats
        self.ion_off = off
        self.peak_mz = mz
        self.peak_int = it
        self._peak_df = None
        self._peak_ints = None
        self._sf_df = None

    @property
    def n_ions(self):
        return len(self.ion_sf)

    @property
    def sf_df(self):
        """The reference's list-column table (built on first use)."""
        if self._sf_df is None:
            o = self.ion_off
            self._sf_df = pd.DataFrame({
                "sf_id": self.ion_sf,
                "adduct": np.asarray(self.adducts, dtype=object)[self.ion_adduct_code],
                "centr_mzs": [self.peak_mz[a:b].tolist() for a, b in zip(o[:-1], o[1:])],
                "centr_ints": [self.peak_int[a:b].tolist() for a, b in zip(o[:-1], o[1:])],
            }, columns=["sf_id", "adduct", "centr_mzs", "centr_ints"])
        return self._sf_df

    @staticmethod
    def check_formula_uniqueness(sf_df):
        """formulas_segm.py:49-53."""
        uniq = len(set(zip(sf_df.sf_id.tolist(), sf_df.adduct.tolist())))
        assert uniq == sf_df.shape[0], "Not unique formula-adduct combinations {} != {}".format(uniq, sf_df.shape[0])

    def get_sf_peak_df(self):
        """formulas_segm.py:55-63: (sf_id, adduct, peak_i, mz), one row per theoretical peak, sorted by mz.
        ``adduct`` is Categorical (string categories).  Built once and cached: do not modify it in place."""
        if self._peak_df is None:
            K = np.diff(self.ion_off)
            owner = np.repeat(np.arange(self.n_ions), K)
            peak_i = np.arange(len(self.peak_mz), dtype=np.int64) - np.repeat(self.ion_off[:-1], K)
            order = np.argsort(self.peak_mz, kind="stable")
            owner = owner[order]
            self._peak_df = pd.DataFrame({
                "sf_id": self.ion_sf[owner],
                "adduct": pd.Categorical.from_codes(self.ion_adduct_code[owner], categories=self.adducts),
                "peak_i": peak_i[order],
                "mz": self.peak_mz[order],
            }, columns=["sf_id", "adduct", "peak_i", "mz"])
        return self._peak_df

    def get_sf_adduct_sorted_df(self):
        """formulas_segm.py:65-66: the (sf_id, adduct) index of every ion, sorted."""
        idx = pd.MultiIndex.from_arrays([self.ion_sf, np.asarray(self.adducts, dtype=object)[self.ion_adduct_code]],
                                        names=["sf_id", "adduct"])
        return pd.DataFrame(index=idx)

    def get_sf_peak_ints(self):
        """formulas_segm.py:68-69 as a read-only mapping backed by flat arrays (PeakInts)."""
        if self._peak_ints is None:
            self._peak_ints = PeakInts(self.ion_sf, self.ion_adduct_code, self.adducts, self.ion_off, self.peak_int)
        return self._peak_ints

    def get_sf_adduct_peaksn(self):
        """formulas_segm.py:71-79: (sf_id, adduct, number of theoretical peaks) in sf_df order."""
        ad = np.asarray(self.adducts, dtype=object)[self.ion_adduct_code]
        return list(zip(self.ion_sf.tolist(), ad.tolist(), np.diff(self.ion_off).tolist()))

    def subset(self, ion_idx):
        """The formulas of the given ions (positions in sf_df order): a rank's shard."""
        ion_idx = np.asarray(ion_idx, dtype=np.int64)
        K = np.diff(self.ion_off)[ion_idx]
        off = np.zeros(len(ion_idx) + 1, np.int64)
        np.cumsum(K, out=off[1:])
        sel = (np.repeat(self.ion_off[ion_idx], K) + np.arange(off[-1]) - np.repeat(off[:-1], K))
        ad = np.asarray(self.adducts, dtype=object)[self.ion_adduct_code[ion_idx]]
        return FormulasSegm.from_arrays(self.ion_sf[ion_idx], ad, off, self.peak_mz[sel], self.peak_int[sel],
                                        self.ppm)


class Formulas(object):
    """Legacy molecule table (formulas.py:24-110) for the legacy imager."""

    def __init__(self, sf_ids, adducts, sf_theor_peaks, sf_theor_peak_ints, ppm):
        self.ppm = ppm
        self.sf_ids, self.adducts = list(sf_ids), list(adducts)
        self.sf_theor_peaks, self.sf_theor_peak_ints = list(sf_theor_peaks), list(sf_theor_peak_ints)
        pairs = list(zip(self.sf_ids, self.adducts))
        assert len(set(pairs)) == len(pairs), "Not unique formula-adduct combinations"

    def get_sf_peak_bounds(self):
        """formulas.py:64-72: ``mz - ppm*mz/1e6`` / ``mz + ppm*mz/1e6``."""
        lower = np.array([mz - self.ppm * mz / 1e6 for peaks in self.sf_theor_peaks for mz in peaks])
        upper = np.array([mz + self.ppm * mz / 1e6 for peaks in self.sf_theor_peaks for mz in peaks])
        return lower, upper

    def get_sf_peak_map(self):
        return np.array([(i, j) for i, peaks in enumerate(self.sf_theor_peaks) for j, _ in enumerate(peaks)])

    def get_sf_peak_ints(self):
        return self.sf_theor_peak_ints

    def get_sf_peaks(self):
        return self.sf_theor_peaks

    def get_sf_adduct_peaksn(self):
        return list(zip(self.sf_ids, self.adducts, map(len, self.sf_theor_peaks)))
