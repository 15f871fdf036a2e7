"""End to end through the drop-in plugin (GPU): ``MSMBasicSearch(sc, ds, formulas, fdr, ds_config).search()``
(msm_basic_search.py:13-31: compute_sf_images -> sf_image_metrics -> sf_image_metrics_est_fdr -> filter) on
the device against the oracle pipeline (oracle images + metrics, oracle ``estimate_fdr`` = fdr.py:70-88) with
the same target/decoy table.  Bar (BASELINE.json north_star): identical annotations at FDR 0.1, identical
digitized FDR for every reported target ion, metrics within 1e-5.
"""
import numpy as np
import pandas as pd
import pytest

from tests.parity_cases import oracle_run

pytestmark = pytest.mark.gpu

FDR_LEVEL = 0.1


def _search_case():
    from sm_distributed_amd import synthetic as syn
    ions = syn.make_ion_table(40, seed=131, decoy_seed=132)
    ds = syn.make_dataset_np(48, 56, 300, seed=133, ions=ions, plant_fraction=0.35, plant_seed=134)
    return ds, ions, 5.0


def _fdr(ions):
    from sm_distributed_amd.fdr import FDR
    fdr = FDR(0, 0, ions.decoy_sample_size, list(ions.target_adducts), None)
    sf, ta, da = ions.td
    fdr.td_df = pd.DataFrame({"sf_id": sf, "ta": ta, "da": da})
    return fdr


def test_search_annotations_at_fdr_match_oracle():
    from oracle import msm_oracle as O
    from sm_distributed_amd.dataset import DeviceDataset
    from sm_distributed_amd.formulas import FormulasSegm
    from sm_distributed_amd.search_algorithm import MSMBasicSearch

    ds, ions, ppm = _search_case()
    ds_config = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    formulas = FormulasSegm.from_ion_table(ions, ppm)
    fdr = _fdr(ions)

    got, images = MSMBasicSearch(None, DeviceDataset(ds), formulas, fdr, ds_config).search()

    # oracle pipeline with the same inputs and decoy table
    _, om = oracle_run(ds, ions, ppm)
    sf_msm = formulas.get_sf_adduct_sorted_df().join(om.msm).fillna(0)
    ofdr = O.estimate_fdr(sf_msm, fdr.td_df, list(ions.target_adducts), ions.decoy_sample_size)
    exp = om.join(ofdr, how="inner")[["chaos", "spatial", "spectral", "msm", "fdr"]]
    exp = exp[(exp.chaos > 0) | (exp.spatial > 0) | (exp.spectral > 0)]

    got, exp = got.sort_index(), exp.sort_index()
    assert list(got.index) == list(exp.index), "reported target ions differ"
    for col in ("chaos", "spatial", "spectral", "msm"):
        assert np.abs(got[col].to_numpy() - exp[col].to_numpy()).max(initial=0.0) <= 1e-5, col
    np.testing.assert_array_equal(got.fdr.to_numpy(), exp.fdr.to_numpy())
    ann = set(got.index[got.fdr <= FDR_LEVEL])
    assert ann == set(exp.index[exp.fdr <= FDR_LEVEL])
    assert len(ann) >= 5, "the case must produce annotations at FDR 0.1"
    # the filtered image set holds exactly the reported ions
    assert set(k for k, _ in images.collect()) == set(got.index)
