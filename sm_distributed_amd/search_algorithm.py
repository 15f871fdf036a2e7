"""Search-algorithm plugin interface: drop-in for sm/engine/search_algorithm.py:2-25.  The MSM plugin,
``MSMBasicSearch``, is in msm_basic_search.py (sm/engine/msm_basic/msm_basic_search.py:7-31).
"""
from __future__ import annotations


class SearchAlgorithm(object):
    def __init__(self, sc, ds, formulas, fdr, ds_config):
        self.sc = sc
        self.ds = ds
        self.formulas = formulas
        self.fdr = fdr
        self.ds_config = ds_config
        self.metrics = []

    def search(self):
        pass

    def calc_metrics(self, sf_images):
        pass

    def estimate_fdr(self, all_sf_metrics_df):
        pass

    def filter_sf_metrics(self, sf_metrics_df):
        return sf_metrics_df[sf_metrics_df.msm > 0]

    def filter_sf_images(self, sf_images, sf_metrics_df):
        """search_algorithm.py:24-25 -- keep ions present in the metrics index."""
        if hasattr(sf_images, "filter_by_keys"):
            return sf_images.filter_by_keys(sf_metrics_df.index)
        index = set(sf_metrics_df.index)
        return sf_images.filter(lambda kv: kv[0] in index)


def __getattr__(name):
    # MSMBasicSearch lives in msm_basic_search.py as in the reference layout; importable from here as before
    if name == "MSMBasicSearch":
        from .msm_basic_search import MSMBasicSearch
        return MSMBasicSearch
    raise AttributeError(name)
