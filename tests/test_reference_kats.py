"""The reference's known-answer tests (tests/golden/kats.json), run against the oracle and the host-side
parts of the drop-in API.  CPU only (no GPU): device-backed KATs live in test_gpu_api.py."""
import json
import os

import numpy as np
import pandas as pd
import pytest
from scipy.sparse import coo_matrix, csr_matrix

from oracle import msm_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KATS = json.load(open(os.path.join(GOLDEN, "kats.json")))


def test_oracle_sample_spectra_kat():
    k = KATS["sample_spectra_2by3"]
    spectra = [(sp, np.array(mz), np.array(cum)) for sp, mz, cum in k["spectra"]]
    got = O.sample_spectra(spectra, np.array(k["lower"]), np.array(k["upper"]), np.array(k["sf_peak_map"]))
    exp = [((a, b), (c, d)) for (a, b), (c, d) in k["expected"]]
    assert got == exp


def test_oracle_coord_list_to_matrix_kat():
    k = KATS["compute_sf_peak_images_2by3"]
    nrows, ncols = k["dims"]
    groups = {}
    for (sf, p), (sp, v) in k["sf_sp_intens"]:
        groups.setdefault(p, []).append((sp, v))
    for p, pairs in groups.items():
        img = O.coord_list_to_matrix(pairs, np.array(k["pixel_inds"]), nrows, ncols)
        np.testing.assert_array_almost_equal(img.toarray(), np.array(k["expected"][str(p)]))


def test_api_legacy_grouping_kat():
    from sm_distributed_amd.formula_imager import compute_sf_images, compute_sf_peak_images
    from sm_distributed_amd.rdd import LocalRDD

    class DS:
        def get_dims(self):
            return (2, 3)

        def get_norm_img_pixel_inds(self):
            return np.array([1, 2, 3, 4, 5])

    k = KATS["compute_sf_peak_images_2by3"]
    pairs = LocalRDD([((a, b), (c, d)) for (a, b), (c, d) in k["sf_sp_intens"]])
    imgs = dict((p, m) for _, (p, m) in compute_sf_peak_images(DS(), pairs).collect())
    np.testing.assert_array_almost_equal(imgs[0].toarray(), k["expected"]["0"])
    np.testing.assert_array_almost_equal(imgs[1].toarray(), k["expected"]["1"])
    sf_imgs = compute_sf_images(LocalRDD([(0, (0, imgs[0])), (0, (1, imgs[1]))])).collect()
    assert sf_imgs[0][0] == 0 and len(sf_imgs[0][1]) == 2


def test_img_pairs_to_list_kat():
    k = KATS["gen_iso_sf_images"]
    pairs = [(p, coo_matrix(np.array(m))) for p, m in k["pairs"]]
    got = O.img_pairs_to_list(pairs, tuple(k["shape"]))
    assert len(got) == len(k["expected"])
    for m, e in zip(got, k["expected"]):
        if e is None:
            assert m is None
        else:
            assert (m.toarray() == np.array(e)).all()


def test_img_measures_replace_invalid():
    from sm_distributed_amd.formula_img_validator import ImgMeasures
    for v in (None, np.nan, np.inf):
        assert ImgMeasures(v, v, v).to_tuple(replace_nan=True) == (0.0, 0.0, 0.0)
    assert ImgMeasures(-0.5, 0.2, 0.3).to_tuple() == (-0.5, 0.2, 0.3)


def test_compute_plumbing_order_with_patched_measures(monkeypatch):
    """test_formula_img_validator.py:17-34: spectral, spatial, chaos order and the tuple layout."""
    k = KATS["compute_img_measures_plumbing"]
    imgs = [csr_matrix(np.array(m)) for m in k["images"]]
    monkeypatch.setattr(O, "isotope_pattern_match", lambda *a: k["mocked"]["spectral"])
    monkeypatch.setattr(O, "isotope_image_correlation", lambda *a, **kw: k["mocked"]["spatial"])
    monkeypatch.setattr(O, "measure_of_chaos", lambda *a, **kw: k["mocked"]["chaos"])
    got = O.compute_img_metrics(imgs, k["sf_ints"], 2, 3, 30)
    np.testing.assert_array_almost_equal(got, k["expected"])


def test_sf_image_metrics_table_with_patched_compute(monkeypatch):
    """test_formula_img_validator.py:51-64: the API keeps get_compute_img_metrics patchable."""
    from sm_distributed_amd import formula_img_validator as V
    from sm_distributed_amd.rdd import LocalRDD
    k = KATS["sf_image_metrics_table"]
    monkeypatch.setattr(V, "get_compute_img_metrics", lambda *a: (lambda *args: tuple(k["mocked"])))

    class DS:
        def get_dims(self):
            return tuple(k["dims"])

    class F:
        def get_sf_peak_ints(self):
            return {(0, "+H"): [100, 10, 1], (1, "+H"): [100, 10, 1]}

    imgs = [csr_matrix([[0, 100, 100], [10, 0, 3]]), csr_matrix([[0, 50, 50], [0, 20, 0]])]
    rdd = LocalRDD([((0, "+H"), imgs), ((1, "+H"), imgs)])
    df = V.sf_image_metrics(rdd, None, F(), DS(), {"image_generation": {"ppm": 1.0, "nlevels": 30, "q": 99,
                                                                          "do_preprocessing": False}})
    exp = pd.DataFrame(k["expected"], columns=["sf_id", "adduct", "chaos", "spatial", "spectral", "msm"]) \
        .set_index(["sf_id", "adduct"])
    pd.testing.assert_frame_equal(df, exp)


def test_sf_image_metrics_est_fdr_join():
    from sm_distributed_amd.formula_img_validator import sf_image_metrics_est_fdr
    df = pd.DataFrame([[0, "+H", 0.9, 0.9, 0.9, 0.9 ** 3], [1, "+H", 0.5, 0.5, 0.5, 0.5 ** 3]],
                      columns=["sf_id", "adduct", "chaos", "spatial", "spectral", "msm"]).set_index(["sf_id", "adduct"])

    class F:
        def get_sf_adduct_sorted_df(self):
            return pd.DataFrame([[0, "+H"], [1, "+H"]], columns=["sf_id", "adduct"]).set_index(["sf_id", "adduct"])

    class Fdr:
        def estimate_fdr(self, msm_df):
            return pd.DataFrame([[0, "+H", 0.99], [1, "+H", 0.5]], columns=["sf_id", "adduct", "fdr"]) \
                .set_index(["sf_id", "adduct"])

    res = sf_image_metrics_est_fdr(df, F(), Fdr())
    assert list(res.columns) == ["chaos", "spatial", "spectral", "msm", "fdr"]
    np.testing.assert_array_almost_equal(res.fdr.values, [0.99, 0.5])


@pytest.mark.parametrize("name", ["estimate_fdr_1", "estimate_fdr_digitize"])
def test_fdr_kats(name):
    from sm_distributed_amd.fdr import FDR
    k = KATS[name]
    fdr = FDR(0, 0, k["decoy_sample_size"], k["target_adducts"], None)
    fdr.fdr_levels = k["fdr_levels"]
    fdr.td_df = pd.DataFrame(k["td"], columns=["sf_id", "ta", "da"])
    msm = pd.DataFrame(k["msm"], columns=["sf_id", "adduct", "msm"]).set_index(["sf_id", "adduct"]).sort_index()
    exp = pd.DataFrame(k["expected"], columns=["sf_id", "adduct", "fdr"]).set_index(["sf_id", "adduct"])
    pd.testing.assert_frame_equal(fdr.estimate_fdr(msm), exp)
    # the oracle's restatement agrees
    o = O.estimate_fdr(msm, fdr.td_df, k["target_adducts"], k["decoy_sample_size"], k["fdr_levels"])
    pd.testing.assert_frame_equal(o, exp)


def test_fdr_decoy_selection(monkeypatch):
    from sm_distributed_amd import fdr as F
    k = KATS["decoy_selection"]
    monkeypatch.setattr(F, "DECOY_ADDUCTS", k["decoy_adducts"])
    fdr = F.FDR(0, 0, k["decoy_sample_size"], k["target_adducts"], None, seed=1)
    fdr.decoy_adduct_selection(sf_ids=k["sf_ids"])
    assert set(map(tuple, fdr.td_df.values.tolist())) == set(map(tuple, k["expected"]))


def test_legacy_ppm_bounds():
    from sm_distributed_amd.formulas import Formulas
    k = KATS["legacy_ppm_bounds"]
    f = Formulas([0], ["+H"], [[k["mz"]]], [[100.0]], k["ppm"])
    lo, hi = f.get_sf_peak_bounds()
    assert lo[0] == pytest.approx(k["expected_lower"], abs=1e-12)
    assert hi[0] == pytest.approx(k["expected_upper"], abs=1e-12)


def test_iso_image_rows_kat():
    from sm_distributed_amd.search_results import iso_image_rows
    k = KATS["iso_image_rows"]
    imgs = [((1, "+H"), [csr_matrix(np.array(m)) for m in k["images"]])]
    rows = list(iso_image_rows(0, 0, imgs, *k["dims"]))
    assert [list(r) for r in rows] == k["expected"]


def test_filter_sf_images_keeps_indexed_ions():
    from sm_distributed_amd.rdd import LocalRDD
    from sm_distributed_amd.search_algorithm import MSMBasicSearch
    imgs = LocalRDD([((0, "+H"), [csr_matrix([[0, 100]])]), ((1, "+H"), [csr_matrix([[0, 0]])])])
    df = pd.DataFrame([[0, "+H", 0.9, 0.9, 0.9, 0.729]],
                      columns=["sf_id", "adduct", "chaos", "spatial", "spectral", "msm"]).set_index(["sf_id", "adduct"])
    out = MSMBasicSearch(None, None, None, None, None).filter_sf_images(imgs, df).collect()
    assert [k for k, _ in out] == [(0, "+H")]


def test_fdr_at_config3_scale_with_zero_ties_matches_oracle():
    """estimate_fdr (vectorised, fdr.py:70-88) vs the oracle's pandas restatement on a config-3-sized table
    (0.98M ions, 60k targets, 20 decoy draws per target adduct) whose msm vector has the device table's shape:
    most ions at exactly 0 (no hits / no signal) and many exact ties elsewhere.  Identical digitised FDR for
    every target ion, identical annotations at FDR 0.1."""
    import pandas as pd
    from oracle import msm_oracle as O
    from sm_distributed_amd import synthetic as syn
    from sm_distributed_amd.fdr import FDR
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
    f = FormulasSegm.from_ion_table(ions, 2.0)
    rng = np.random.default_rng(1)
    msm = np.where(rng.random(ions.n_ions) < 0.7, 0.0, np.round(0.8 * rng.random(ions.n_ions) ** 3, 3))
    tgt = ions.target_mask()
    msm[tgt] = np.where(rng.random(tgt.sum()) < 0.1, np.round(0.75 + 0.25 * rng.random(tgt.sum()), 3), msm[tgt])
    df = f.get_sf_adduct_sorted_df().copy()
    df["msm"] = msm
    fdr = FDR(0, 0, 20, list(ions.target_adducts))
    sf, ta, da = ions.td
    fdr.td_df = pd.DataFrame({"sf_id": sf, "ta": ta, "da": da})
    got = fdr.estimate_fdr(df).sort_index()
    exp = O.estimate_fdr(df, fdr.td_df, list(ions.target_adducts), 20).sort_index()
    assert got.index.equals(exp.index) and len(got) == 60000
    np.testing.assert_array_equal(got.fdr.to_numpy(), exp.fdr.to_numpy())
    ann = got.index[got.fdr <= 0.1]
    assert len(ann) > 100 and ann.equals(exp.index[exp.fdr <= 0.1])


def _dense_rows(job_id, db_id, items, nrows, ncols):
    """search_results.py:88-97 verbatim in meaning: densify, mask > 0.001, min/max over the full image."""
    for (sf_id, adduct), img_list in items:
        for peak_i, img in enumerate(img_list):
            ints = np.zeros(nrows * ncols) if img is None else img.toarray().flatten()
            inds = np.arange(ints.shape[0])
            m = ints > 0.001
            if m.sum() > 0:
                yield (job_id, db_id, sf_id, adduct, peak_i, inds[m].tolist(), ints[m].tolist(), ints.min(),
                       ints.max())


def test_iso_image_rows_sparse_equals_dense_restatement():
    """The sparse host path (no densifying) gives the reference's rows: duplicates summed, explicit zeros,
    values at/below the 0.001 threshold, a fully covered image (min > 0), None gaps."""
    from scipy.sparse import coo_matrix, csr_matrix
    from sm_distributed_amd.search_results import iso_image_rows
    rng = np.random.default_rng(9)
    nr, nc = 7, 9
    items = []
    for i in range(30):
        n = int(rng.integers(0, 40))
        r, c = rng.integers(0, nr, n), rng.integers(0, nc, n)
        v = rng.choice([0.0, 0.0005, 0.001, 0.002, 1.0, 37.5], n)
        imgs = [coo_matrix((v, (r, c)), shape=(nr, nc)), None, csr_matrix(coo_matrix((v[::-1], (r, c)), shape=(nr, nc)))]
        if i % 5 == 0:  # every pixel covered
            imgs.append(coo_matrix((rng.uniform(0.5, 2, nr * nc), (np.repeat(np.arange(nr), nc), np.tile(np.arange(nc), nr))),
                                   shape=(nr, nc)))
        items.append(((i, "+H"), imgs))
    got = list(iso_image_rows(3, 4, items, nr, nc))
    exp = list(_dense_rows(3, 4, items, nr, nc))
    assert len(got) == len(exp) and len(exp) > 20
    for g, e in zip(got, exp):
        assert g[:6] == e[:6]
        np.testing.assert_allclose(g[6], e[6], rtol=1e-15, atol=0)
        assert g[7] == e[7] and g[8] == e[8]
