"""Target/decoy FDR: drop-in for sm/engine/fdr.py (host-side pandas).

Runs on rank 0 after the metric rows are gathered.  Behaviour follows fdr.py:15-88:
``decoy_adduct_selection`` draws ``decoy_sample_size`` decoy adducts per (sf, target adduct) without
replacement from the 80 element adducts minus the targets; ``estimate_fdr`` computes, per target adduct,
the decoy_cum/target_cum curve over msm for each of the decoy_sample_size decoy draws, takes the
median, and digitizes it to ``fdr_levels``.  The reference draws with the unseeded global
``np.random``; here the draw takes an explicit seed so every rank (and the oracle) shares one table.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from .synthetic import DECOY_ADDUCTS

SF_LIST_SEL = ('SELECT af.id FROM agg_formula af JOIN formula_db db ON db.id = af.db_id WHERE db.id = %s')


class FDR(object):
    def __init__(self, job_id, db_id, decoy_sample_size, target_adducts, db, seed=None):
        self.job_id = job_id
        self.db_id = db_id
        self.decoy_sample_size = decoy_sample_size
        self.db = db
        self.target_adducts = target_adducts
        self.td_df = None
        self.fdr_levels = [0.05, 0.1, 0.2, 0.5]
        self.seed = seed

    @staticmethod
    def _decoy_adduct_gen(sf_ids, target_adducts, decoy_adducts_cand, decoy_sample_size, rng=None):
        choice = (rng or np.random).choice
        for sf_id in sf_ids:
            for ta in target_adducts:
                for da in choice(decoy_adducts_cand, size=decoy_sample_size, replace=False):
                    yield (sf_id, ta, da)

    def _save_target_decoy_df(self):
        if self.db is None or not hasattr(self.db, "copy"):
            return
        import io
        buf = io.StringIO()
        df = self.td_df.copy()
        df.insert(0, "db_id", self.db_id)
        df.insert(0, "job_id", self.job_id)
        df.to_csv(buf, index=False, header=False)
        buf.seek(0)
        self.db.copy(buf, "target_decoy_add", sep=",")

    def decoy_adduct_selection(self, sf_ids=None):
        """fdr.py:42-48; ``sf_ids`` may be given directly instead of selected from the DB."""
        if sf_ids is None:
            sf_ids = [r[0] for r in self.db.select(SF_LIST_SEL, self.db_id)]
        decoy_adduct_cand = sorted(set(DECOY_ADDUCTS) - set(self.target_adducts))
        rng = np.random.default_rng(self.seed) if self.seed is not None else None
        self.td_df = pd.DataFrame(self._decoy_adduct_gen(sf_ids, self.target_adducts, decoy_adduct_cand,
                                                         self.decoy_sample_size, rng),
                                  columns=["sf_id", "ta", "da"])
        self._save_target_decoy_df()

    @staticmethod
    def _msm_fdr_map(target_msm, decoy_msm):
        target_msm_hits = pd.Series(target_msm.msm.value_counts(), name="target")
        decoy_msm_hits = pd.Series(decoy_msm.msm.value_counts(), name="decoy")
        msm_df = pd.concat([target_msm_hits, decoy_msm_hits], axis=1).fillna(0).sort_index(ascending=False)
        msm_df["target_cum"] = msm_df.target.cumsum()
        msm_df["decoy_cum"] = msm_df.decoy.cumsum()
        msm_df["fdr"] = msm_df.decoy_cum / msm_df.target_cum
        return msm_df.fdr

    def _digitize_fdr(self, fdr_df):
        df = fdr_df.copy().sort_values(by="msm", ascending=False)
        msm_levels = [df[df.fdr < fdr_thr].msm.min() for fdr_thr in self.fdr_levels]
        df["fdr_d"] = 1.0
        for msm_thr, fdr_thr in zip(msm_levels, self.fdr_levels):
            row_mask = np.isclose(df.fdr_d, 1.0) & np.greater_equal(df.msm, msm_thr)
            df.loc[row_mask, "fdr_d"] = fdr_thr
        df["fdr"] = df.fdr_d
        return df.drop("fdr_d", axis=1)

    def estimate_fdr(self, msm_df):
        """fdr.py:70-88: msm_df indexed by (sf_id, adduct) with column msm (targets + decoys)."""
        target_fdr_df_list = []
        for ta in self.target_adducts:
            target_msm = msm_df.loc(axis=0)[:, ta]
            msm_fdr_list = []
            sub = self.td_df[self.td_df.ta == ta][["sf_id", "da"]]
            for i in range(self.decoy_sample_size):
                sf_da_list = list(map(tuple, sub[i::self.decoy_sample_size].values))
                decoy_msm = msm_df.loc[sf_da_list]
                msm_fdr_list.append(self._msm_fdr_map(target_msm, decoy_msm))
            msm_fdr_avg = pd.Series(pd.concat(msm_fdr_list, axis=1).median(axis=1), name="fdr")
            target_fdr = self._digitize_fdr(target_msm.join(msm_fdr_avg, on="msm"))
            target_fdr_df_list.append(target_fdr.drop("msm", axis=1))
        return pd.concat(target_fdr_df_list, axis=0)
