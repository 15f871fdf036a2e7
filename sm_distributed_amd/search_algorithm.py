"""Search-algorithm plugin interface: drop-in for sm/engine/search_algorithm.py:2-25 and
sm/engine/msm_basic/msm_basic_search.py:7-31.

``MSMBasicSearch(sc, ds, formulas, fdr, ds_config).search()`` runs compute_sf_images ->
sf_image_metrics -> sf_image_metrics_est_fdr -> filter (chaos>0 | spatial>0 | spectral>0) and returns
``(sf_metrics_fdr_df, filtered sf_images)`` exactly as the reference plugin does; the images and the
scoring live on the GPU.
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


class MSMBasicSearch(SearchAlgorithm):
    def __init__(self, sc, ds, formulas, fdr, ds_config):
        super(MSMBasicSearch, self).__init__(sc, ds, formulas, fdr, ds_config)
        self.metrics = ["chaos", "spatial", "spectral"]

    def search(self):
        from .formula_imager_segm import compute_sf_images
        sf_images = compute_sf_images(self.sc, self.ds, self.formulas.get_sf_peak_df(),
                                      self.ds_config["image_generation"]["ppm"])
        all_sf_metrics_df = self.calc_metrics(sf_images)
        sf_metrics_fdr_df = self.estimate_fdr(all_sf_metrics_df)
        sf_metrics_fdr_df = self.filter_sf_metrics(sf_metrics_fdr_df)
        return sf_metrics_fdr_df, self.filter_sf_images(sf_images, sf_metrics_fdr_df)

    def calc_metrics(self, sf_images):
        from .formula_img_validator import sf_image_metrics
        return sf_image_metrics(sf_images, self.sc, self.formulas, self.ds, self.ds_config)

    def estimate_fdr(self, all_sf_metrics_df):
        from .formula_img_validator import sf_image_metrics_est_fdr
        return sf_image_metrics_est_fdr(all_sf_metrics_df, self.formulas, self.fdr)

    def filter_sf_metrics(self, sf_metrics_df):
        return sf_metrics_df[(sf_metrics_df.chaos > 0) | (sf_metrics_df.spatial > 0) | (sf_metrics_df.spectral > 0)]
