"""Theoretical-peak tables: the data contract of sm/engine/formulas_segm.py (and legacy formulas.py).

``FormulasSegm`` exposes what the hot path consumes (formulas_segm.py:56-79): ``sf_df`` with columns
(sf_id, adduct, centr_mzs, centr_ints) sorted by (sf_id, adduct), ``get_sf_peak_df`` (one row per
theoretical peak, sorted by mz), ``get_sf_peak_ints`` ({(sf_id, adduct): ints}),
``get_sf_adduct_sorted_df`` and ``get_sf_adduct_peaksn``.  The Postgres load (:25-47) is out of scope:
construct from a DataFrame / an ``IonTable`` instead.  Legacy ``Formulas`` (formulas.py) adds
``get_sf_peak_bounds`` (mz -/+ ppm*mz/1e6) and ``get_sf_peak_map``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd


class FormulasSegm(object):
    def __init__(self, sf_df: pd.DataFrame, ppm: float = 2.0):
        self.ppm = ppm
        self.sf_df = sf_df[["sf_id", "adduct", "centr_mzs", "centr_ints"]].sort_values(["sf_id", "adduct"])
        self.check_formula_uniqueness(self.sf_df)

    @classmethod
    def from_ion_table(cls, ions, ppm=2.0):
        return cls(ions.sf_df(), ppm)

    @staticmethod
    def check_formula_uniqueness(sf_df):
        """formulas_segm.py:49-53."""
        uniq = len(set(zip(sf_df.sf_id.tolist(), sf_df.adduct.tolist())))
        assert uniq == sf_df.shape[0], "Not unique formula-adduct combinations {} != {}".format(uniq, sf_df.shape[0])

    @staticmethod
    def sf_peak_gen(sf_df):
        for sf_id, adduct, mzs, _ in sf_df.values:
            for pi, mz in enumerate(mzs):
                yield sf_id, adduct, pi, mz

    def get_sf_peak_df(self):
        return pd.DataFrame(self.sf_peak_gen(self.sf_df),
                            columns=["sf_id", "adduct", "peak_i", "mz"]).sort_values(by="mz", kind="stable")

    def get_sf_adduct_sorted_df(self):
        return self.sf_df[["sf_id", "adduct"]].copy().set_index(["sf_id", "adduct"]).sort_index()

    def get_sf_peak_ints(self):
        return dict(zip(zip(self.sf_df.sf_id, self.sf_df.adduct), self.sf_df.centr_ints))

    def get_sf_adduct_peaksn(self):
        return list(zip(self.sf_df.sf_id, self.sf_df.adduct, self.sf_df.centr_mzs.map(len)))


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
