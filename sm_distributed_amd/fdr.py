"""Target/decoy FDR: the behaviour of sm/engine/fdr.py, vectorised for ~1M ions.

Runs on rank 0 after the metric rows are gathered.  Semantics (fdr.py:15-88):

* ``decoy_adduct_selection`` draws ``decoy_sample_size`` decoy adducts without replacement per
  (sf, target adduct) from the 80 element adducts minus the targets (fdr.py:26-31, 42-48).  The reference
  uses the unseeded global ``np.random``; here one seeded generator draws the whole table at once, so every
  rank (and the oracle) can share it.  Writing the table to Postgres (fdr.py:33-40) is out of scope.
* ``estimate_fdr(msm_df)`` (fdr.py:70-88): for target adduct ``ta`` and decoy draw ``i`` (row ``i`` of every
  sf's block of the ta-rows of ``td_df``), the FDR at a target's msm value ``v`` is
  ``#{decoys of draw i with msm >= v} / #{targets with msm >= v}`` -- exactly what the value_counts /
  cumsum table of ``_msm_fdr_map`` (fdr.py:51-58) evaluates at ``v``, since every target value is in that
  table's index.  The per-target FDR is the median over the draws (fdr.py:83), then digitised to
  ``fdr_levels`` (fdr.py:60-68): level ``l`` goes to every still-undigitised target whose msm is >= the
  smallest msm with FDR < ``l``.  Decoy keys missing from ``msm_df`` are not counted (old-pandas ``.loc``
  with missing labels gave NaN rows, which ``value_counts`` drops).

Instead of 2 x decoy_sample_size pandas value_counts / concat / join passes per target adduct, each draw is
one sorted array and every count is a ``searchsorted``: O((n_targets + n_decoys) log n) per draw.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from .synthetic import DECOY_ADDUCTS


class FDR(object):
    def __init__(self, job_id, db_id, decoy_sample_size, target_adducts, db=None, seed=None):
        self.job_id = job_id
        self.db_id = db_id
        self.decoy_sample_size = decoy_sample_size
        self.db = db  # accepted for signature compatibility; nothing is read from or written to it
        self.target_adducts = target_adducts
        self.td_df = None
        self.fdr_levels = [0.05, 0.1, 0.2, 0.5]
        self.seed = seed

    def decoy_adduct_selection(self, sf_ids=None):
        """fdr.py:42-48 for the given formula ids (the reference SELECTs them from Postgres)."""
        if sf_ids is None:
            raise ValueError("decoy_adduct_selection needs sf_ids (formula DB access is out of scope)")
        sf_ids = np.asarray(sf_ids)
        cand = np.array(sorted(set(DECOY_ADDUCTS) - set(self.target_adducts)), dtype=object)
        n_ta, k = len(self.target_adducts), self.decoy_sample_size
        if k > len(cand):
            raise ValueError("decoy_sample_size %d > %d decoy candidates" % (k, len(cand)))
        rng = np.random.default_rng(self.seed)
        # one draw without replacement per (sf, ta) row: the first k of a random permutation of the candidates
        draws = np.argsort(rng.random((len(sf_ids) * n_ta, len(cand))), axis=1)[:, :k]
        self.td_df = pd.DataFrame({
            "sf_id": np.repeat(sf_ids, n_ta * k),
            "ta": np.tile(np.repeat(np.array(self.target_adducts, dtype=object), k), len(sf_ids)),
            "da": cand[draws.reshape(-1)],
        }, columns=["sf_id", "ta", "da"])

    # ---- estimate_fdr --------------------------------------------------------------------------
    @staticmethod
    def _keyer(index: pd.MultiIndex):
        """Integer keys for (sf_id, adduct) pairs: sorted keys of ``index`` and a function mapping pairs to
        positions in ``index`` (-1 when absent)."""
        sf_lv = index.levels[0]
        ad_lv = index.levels[1]
        n_ad = max(len(ad_lv), 1)
        own = index.codes[0].astype(np.int64) * n_ad + index.codes[1].astype(np.int64)
        order = np.argsort(own, kind="stable")
        own_sorted = own[order]

        def lookup(sf, ad):
            if len(own_sorted) == 0:
                return np.full(len(sf), -1, np.int64)
            a = sf_lv.get_indexer(pd.Index(sf))
            b = ad_lv.get_indexer(pd.Index(ad))
            key = a.astype(np.int64) * n_ad + b
            pos = np.searchsorted(own_sorted, key)
            pos_c = np.minimum(pos, len(own_sorted) - 1)
            ok = (a >= 0) & (b >= 0) & (own_sorted[pos_c] == key)
            return np.where(ok, order[pos_c], -1)

        return lookup

    def _digitize(self, msm, fdr):
        """fdr.py:60-68 on arrays already sorted by msm descending."""
        fdr_d = np.ones_like(fdr)
        for thr in self.fdr_levels:
            sel = fdr < thr
            if not sel.any():
                continue  # min() of an empty selection is NaN: no msm is >= NaN
            msm_thr = msm[sel].min()
            fdr_d[np.isclose(fdr_d, 1.0) & (msm >= msm_thr)] = thr
        return fdr_d

    def estimate_fdr(self, msm_df):
        """fdr.py:70-88: ``msm_df`` indexed by (sf_id, adduct) with column msm (targets + decoys); returns the
        digitised fdr of every target ion, indexed by (sf_id, adduct), grouped by target adduct, msm descending."""
        if not isinstance(msm_df.index, pd.MultiIndex):
            raise ValueError("msm_df must be indexed by (sf_id, adduct)")
        index = msm_df.index.remove_unused_levels()
        msm_all = msm_df["msm"].to_numpy(dtype=np.float64)
        lookup = self._keyer(index)
        ad_of_row = index.levels[1].to_numpy()[index.codes[1]]
        sf_of_row = index.levels[0].to_numpy()[index.codes[0]]
        td = self.td_df
        k = self.decoy_sample_size
        parts = []
        for ta in self.target_adducts:
            rows = np.nonzero(ad_of_row == ta)[0]
            t = msm_all[rows]
            t_sorted = np.sort(t)
            target_cum = len(t) - np.searchsorted(t_sorted, t, side="left")  # #targets with msm >= t (>= 1)
            sub = td[td.ta == ta]
            sub_sf, sub_da = sub.sf_id.to_numpy(), sub.da.to_numpy()
            fdr_draws = np.empty((k, len(t)))
            for i in range(k):
                pos = lookup(sub_sf[i::k], sub_da[i::k])
                d = np.sort(msm_all[pos[pos >= 0]])
                decoy_cum = len(d) - np.searchsorted(d, t, side="left")
                fdr_draws[i] = decoy_cum / target_cum
            fdr = np.median(fdr_draws, axis=0) if k > 0 else np.full(len(t), np.nan)
            order = np.argsort(-t, kind="stable")
            fdr_d = self._digitize(t[order], fdr[order])
            r = rows[order]
            parts.append(pd.DataFrame({"sf_id": sf_of_row[r], "adduct": ad_of_row[r], "fdr": fdr_d},
                                      columns=["sf_id", "adduct", "fdr"]))
        out = pd.concat(parts, axis=0, ignore_index=True) if parts else \
            pd.DataFrame(columns=["sf_id", "adduct", "fdr"])
        return out.set_index(["sf_id", "adduct"])
