"""sm_distributed_amd -- MI355X-native molecule-annotation hot path of SM_distributed.

Ion-image generation (``formula_imager_segm.compute_sf_images``) and MSM scoring
(``formula_img_validator.sf_image_metrics``) as HIP kernels for gfx950 behind the reference's own
Python interface.  See DESIGN.md.
"""
__version__ = "0.2.0"  # = the library's smg_version() (smg_prep.hip)

