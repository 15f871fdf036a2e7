"""Theoretical peak generation for a formula database: drop-in for sm/engine/theor_peaks_gen.py (§8f row 3).

``TheorPeaksGenerator`` keeps the reference's methods and their behaviour (theor_peaks_gen.py:18-146):
``_sf_elements``, ``_valid_sf_adduct``, ``apply_database_filters`` ('organic' filter), ``find_sf_adduct_cand``
(targets + DECOY_ADDUCTS not yet stored) and ``generate_theor_peaks`` (formatted theor_peaks rows, computed in
chunks of 10,000).  Persistence is out of scope: the reference's ``run`` SELECTs formulas and
stored peaks from Postgres and ``_import_theor_peaks_to_db`` COPYs the rows back (theor_peaks_gen.py:57-74,
136-146); here the caller passes the formula list and the stored (sf, adduct) set and receives the rows.  The
Spark fan-out becomes one native multi-threaded call per chunk (``IsocalcWrapper.isotope_peaks_batch``).

``theor_peaks_df`` builds the (sf_id, adduct, centr_mzs, centr_ints) table that ``FormulasSegm`` (and so the
GPU search) consumes, straight from formula strings.
"""
from __future__ import annotations

import logging
import os
import pandas as pd

from .fdr import DECOY_ADDUCTS
from .isocalc_wrapper import IsocalcWrapper

logger = logging.getLogger("sm_distributed_amd")

def _parse_elements(sf):
    """Element symbols of a sum formula in order of first appearance (pyMSpec parseSumFormula segments)."""
    import re
    if not isinstance(sf, str):
        raise ValueError("invalid sum formula {!r}".format(sf))
    seen = []
    for e in re.findall(r"[A-Z][a-z]*", sf):
        if e not in seen:
            seen.append(e)
    return seen


class TheorPeaksGenerator(object):
    """Generator of theoretical isotope peaks for all molecules in a database (theor_peaks_gen.py:18-146)."""

    CHUNK = 10000  # theor_peaks_gen.py:128

    def __init__(self, sc, sm_config, ds_config, n_threads: int = 0, db_id: int = 0):
        self.sc = sc
        self.sm_config = sm_config
        self.ds_config = ds_config
        self.theor_peaks_tmp_dir = os.path.join(sm_config.get("fs", {}).get("base_path", ""), "tmp_theor_peaks_gen")
        self.db_id = db_id  # formula database id written into the rows
        self.n_threads = n_threads
        self.adducts = self.ds_config["isotope_generation"]["adducts"]
        self.isocalc_wrapper = IsocalcWrapper(self.ds_config["isotope_generation"])

    @staticmethod
    def _sf_elements(sf):
        return _parse_elements(sf)

    @classmethod
    def _valid_sf_adduct(cls, sf, adduct):
        """theor_peaks_gen.py:45-55."""
        if sf is None or adduct is None or sf == "None" or adduct == "None":
            logger.warning("Invalid sum formula or adduct: sf=%s, adduct=%s", sf, adduct)
            return False
        if "-" in adduct and adduct.strip("-") not in cls._sf_elements(sf):
            logger.info("No negative adduct element in the sum formula: sf=%s, adduct=%s", sf, adduct)
            return False
        return True

    def run(self, formula_list, stored_sf_adduct=()):
        """theor_peaks_gen.py:57-74 without the database: rows for the (sf, adduct) pairs not stored yet."""
        logger.info("Running theoretical peaks generation")
        formula_list = self.apply_database_filters(formula_list)
        sf_adduct_cand = self.find_sf_adduct_cand(formula_list, set(map(tuple, stored_sf_adduct)))
        logger.info("%d saved (sf, adduct)s, %s not saved (sf, adduct)s", len(stored_sf_adduct), len(sf_adduct_cand))
        return self.generate_theor_peaks(sf_adduct_cand) if sf_adduct_cand else []

    def apply_database_filters(self, formula_list):
        """theor_peaks_gen.py:76-92: the 'organic' filter keeps formulas containing carbon."""
        if "organic" in [s.lower() for s in self.ds_config["database"].get("filters", [])]:
            logger.info("Organic sum formula filter has been applied")
            return [(i, sf) for i, sf in formula_list if "C" in self._sf_elements(sf)]
        return formula_list

    def find_sf_adduct_cand(self, formula_list, stored_sf_adduct):
        """theor_peaks_gen.py:94-111: (id, sf, adduct) for target + decoy adducts not stored yet."""
        assert formula_list, "Emtpy agg_formula table!"
        adducts = set(self.adducts) | set(DECOY_ADDUCTS)
        cand = [(i, sf, a) for (i, sf) in formula_list for a in sorted(adducts)]
        return [(i, sf, a) for (i, sf, a) in cand if (sf, a) not in stored_sf_adduct]

    def generate_theor_peaks(self, sf_adduct_cand):
        """theor_peaks_gen.py:113-134: formatted theor_peaks rows, computed in chunks."""
        logger.info("Generating missing peaks")
        all_lines = []
        for i in range(0, len(sf_adduct_cand), self.CHUNK):
            chunk = sf_adduct_cand[i:i + self.CHUNK]
            cents = self.isocalc_wrapper.isotope_peaks_batch([(sf, a) for _, sf, a in chunk], self.n_threads)
            all_lines.extend(self.isocalc_wrapper._format_peak_str(self.db_id, sf_id, a, c)
                             for (sf_id, _, a), c in zip(chunk, cents) if len(c.mzs) > 0)
        return all_lines


def theor_peaks_df(formulas, adducts, isocalc_config, n_threads: int = 0) -> pd.DataFrame:
    """(sf_id, adduct, centr_mzs, centr_ints) for every (id, sum formula) x adduct with a non-empty pattern --
    the table FormulasSegm (formulas_segm.py:25-47) loads from theor_peaks."""
    w = IsocalcWrapper(isocalc_config)
    pairs = [(i, sf, a) for i, sf in formulas for a in adducts]
    cents = w.isotope_peaks_batch([(sf, a) for _, sf, a in pairs], n_threads)
    rows = [(i, a, list(map(float, c.mzs)), list(map(float, c.ints)))
            for (i, _, a), c in zip(pairs, cents) if len(c.mzs) > 0]
    return pd.DataFrame(rows, columns=["sf_id", "adduct", "centr_mzs", "centr_ints"])
