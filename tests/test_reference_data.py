"""Pins against data the reference itself holds, read IN PLACE from /root/reference (CPU only; skipped where the
reference tree is absent, e.g. on the GPU box -- nothing is copied into this repository).

* config 1: the bundled example dataset tests/data/imzml_example_ds/Example_Continuous.imzML with its
  config.json, searched for C12H24O (sf_id 10007) with metrics mocked to 0.9 as the reference's regression test
  does (tests/test_search_job_imzml_example.py:39-42), asserting that test's facts (:51-86): image bounds
  x, y in 1..3; 3 target + 80 decoy theoretical-peak rows, each with centroids; metric rows for sf 10007 with
  stats {chaos, spatial, spectral}; image rows for sf 10007 with max intensity > 0.  Imaging runs on the oracle
  here (no GPU in this container); the same reader + API run on the device in test_gpu_api.py.
* the golden scientific table tests/reports/spheroid_12h_search_res.csv: every positive chaos value has the
  measure_of_chaos structure 1 - (sum of component counts) / (nlevels * #positive pixels) with nlevels = 30,
  the structure of the restated measure_of_chaos (oracle/msm_oracle.py).
* search_results.py:57-62 wire format of the metric rows, positional peaks_n.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest

REF = "/root/reference"
EXAMPLE = os.path.join(REF, "tests", "data", "imzml_example_ds")
SPHEROID_CSV = os.path.join(REF, "tests", "reports", "spheroid_12h_search_res.csv")

needs_ref = pytest.mark.skipif(not os.path.isdir(EXAMPLE), reason="reference tree not present")


@needs_ref
def test_config1_imzml_example_facts(monkeypatch):
    from oracle import msm_oracle as O
    from sm_distributed_amd import formula_img_validator as V
    from sm_distributed_amd import theor_peaks_gen as T
    from sm_distributed_amd.fdr import FDR
    from sm_distributed_amd.formulas import FormulasSegm
    from sm_distributed_amd.imzml import read_imzml
    from sm_distributed_amd.rdd import LocalRDD
    from sm_distributed_amd.search_results import iso_image_rows, metrics_rows
    from sm_distributed_amd.synthetic import DECOY_ADDUCTS

    cfg = json.load(open(os.path.join(EXAMPLE, "config.json")))
    spectra = read_imzml(os.path.join(EXAMPLE, "Example_Continuous.imzML"))
    # dataset meta (:51-56): img_bounds x, y in 1..3
    c = np.asarray(spectra.coords)
    assert spectra.n_spectra == 9
    assert (c[:, 0].min(), c[:, 0].max(), c[:, 1].min(), c[:, 1].max()) == (1, 3, 1, 3)
    pm, dims = spectra.pixel_map_dims()
    assert dims == (3, 3) and sorted(pm.tolist()) == list(range(9))
    assert spectra.n_points == 9 * 8399 and 100.0 < spectra.mz.min() and spectra.mz.max() < 800.0

    # theoretical patterns (:58-65): 3 + 80 rows with centroids
    iso = cfg["isotope_generation"]
    targets = iso["adducts"]
    tp = T.theor_peaks_df([(10007, "C12H24O")], targets + DECOY_ADDUCTS, iso)
    assert len(tp) == 3 + len(DECOY_ADDUCTS)
    assert all(len(m) > 0 and len(i) > 0 for m, i in zip(tp.centr_mzs, tp.centr_ints))
    formulas = FormulasSegm(tp, cfg["image_generation"]["ppm"])

    # the search with the metrics mocked as the reference test does (:39-42)
    monkeypatch.setattr(V, "get_compute_img_metrics", lambda *a: (lambda *args: (0.9, 0.9, 0.9)))
    ppm = cfg["image_generation"]["ppm"]
    imgs = O.compute_sf_images(spectra.spectra(), pm, dims, formulas.get_sf_peak_df(), ppm)
    rdd = LocalRDD(list(imgs.items()))

    class DS:
        def get_dims(self):
            return dims

    metrics = V.sf_image_metrics(rdd, None, formulas, DS(), cfg)
    fdr = FDR(0, 0, 20, targets, seed=0)
    fdr.decoy_adduct_selection(sf_ids=[10007])
    res = V.sf_image_metrics_est_fdr(metrics, formulas, fdr)
    res = res[(res.chaos > 0) | (res.spatial > 0) | (res.spectral > 0)]
    rows = list(metrics_rows(0, 0, res, formulas.get_sf_adduct_peaksn()))
    # image metric rows (:67-76): rows exist, (db_id, sf_id) = (0, 10007), stats keys
    assert rows and tuple(rows[0][:3][1:]) == (0, 10007)
    assert set(json.loads(rows[0][6]).keys()) == {"chaos", "spatial", "spectral"}
    # image rows (:78-87): rows exist for sf 10007, max intensity > 0
    img_rows = list(iso_image_rows(0, 0, [(k, v) for k, v in imgs.items() if k in set(res.index)], *dims))
    assert img_rows and all(r[2] == 10007 for r in img_rows)
    assert max(r[-1] for r in img_rows) > 0


@pytest.mark.skipif(not os.path.exists(SPHEROID_CSV), reason="reference tree not present")
def test_reference_golden_chaos_has_the_restated_structure():
    df = pd.read_csv(SPHEROID_CSV, sep="\t")
    assert list(df.columns) == ["sf", "adduct", "chaos", "spatial", "spectral"] and len(df) == 2780
    c = df.chaos.to_numpy()
    assert (c >= 0).all() and (c <= 1).all()
    pos = c[c > 0]
    assert len(pos) > 1000
    n = np.arange(4, 5001)
    for v in pos:
        x = (1.0 - v) * 30.0 * n          # sum of component counts over the 30 levels, if #pixels = n
        ok = np.abs(x - np.round(x)) <= 30.0 * n * 1e-12 + 1e-9   # the CSV carries 12 significant digits
        assert ok.any(), v
    # a random value in the same range fits this often by chance: < 1e-3 per value
    rng = np.random.default_rng(0)
    fits = 0
    for v in rng.uniform(0.85, 1.0, 2000):
        x = (1.0 - v) * 30.0 * n
        fits += bool((np.abs(x - np.round(x)) <= 30.0 * n * 1e-12 + 1e-9).any())
    assert fits < 10


def test_metrics_rows_positional_peaks_n_and_by_key():
    """search_results.py:57-62: peaks_n = sf_adduct_peaksn[ind][2] by row position (the reference), or by key."""
    from sm_distributed_amd.search_results import metrics_rows
    df = pd.DataFrame([[2, "+K", 0.9, 0.8, 0.7, 0.504, 0.1], [1, "+H", 0.5, 0.5, 0.5, 0.125, 0.5]],
                      columns=["sf_id", "adduct", "chaos", "spatial", "spectral", "msm", "fdr"]) \
        .set_index(["sf_id", "adduct"])
    peaksn = [(1, "+H", 4), (1, "+Na", 5), (2, "+K", 6)]
    pos = list(metrics_rows(7, 3, df, peaksn))
    assert [r[7] for r in pos] == [4, 5]                    # rows 0 and 1 of the formula table's list
    assert pos[0][:6] == (7, 3, 2, "+K", 0.504, 0.1)
    assert json.loads(pos[0][6]) == {"chaos": 0.9, "spatial": 0.8, "spectral": 0.7}
    assert list(json.loads(pos[0][6]).keys()) == ["chaos", "spatial", "spectral"]
    key = list(metrics_rows(7, 3, df, peaksn, peaks_n="by_key"))
    assert [r[7] for r in key] == [6, 4]
    with pytest.raises(ValueError):
        list(metrics_rows(7, 3, df, peaksn, peaks_n="other"))
