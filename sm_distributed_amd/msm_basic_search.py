"""MSM plugin: drop-in for sm/engine/msm_basic/msm_basic_search.py:7-31.

``MSMBasicSearch(sc, ds, formulas, fdr, ds_config).search()`` runs compute_sf_images ->
sf_image_metrics -> sf_image_metrics_est_fdr -> filter (chaos>0 | spatial>0 | spectral>0) and returns
``(sf_metrics_fdr_df, filtered sf_images)`` exactly as the reference plugin does; the images and the
scoring live on the GPU.
"""
from __future__ import annotations

from .search_algorithm import SearchAlgorithm


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
