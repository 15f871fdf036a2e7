"""Theoretical isotope patterns: the native calculator (smg_isotope_centroids, host code in
libsmg.so) against the oracle restatement (oracle/isocalc_oracle.py), physical known answers, and the reference's
own wrapper / generator tests (sm/engine/tests/test_isocalc_wrapper.py, test_theor_peaks_gen.py) transcribed.

Parity with the third-party calculator the reference used (cpyMSpec complete_isodist) is UNPINNED: it is not in
/root/reference or this image and every reference test mocks it.  The known answers pin what physics fixes:
monoisotopic m/z of common ions (literature values) and isotope abundance ratios.  CPU-only: no GPU needed."""
import numpy as np
import pytest
from unittest import mock

from oracle import isocalc_oracle as O
from sm_distributed_amd import theor_peaks_gen as TPG
from sm_distributed_amd.isocalc_wrapper import Centroids, IsocalcWrapper


def ds_config():  # sm/engine/tests/util.py:40-62
    return {
        "database": {"name": "HMDB"},
        "isotope_generation": {"adducts": ["+H", "+Na"], "charge": {"polarity": "+", "n_charges": 1},
                               "isocalc_sigma": 0.01, "isocalc_pts_per_mz": 10000},
        "image_generation": {"ppm": 1.0, "nlevels": 30, "q": 99, "do_preprocessing": False},
    }


FORMULAS = [("C6H12O6+H", 1), ("C6H12O6+Na", 1), ("C6H12O6-H", -1), ("C12H24O+K", 1), ("C40H80NO8P+H", 1),
            ("C10H16N5O13P3+H", 1), ("Au+H", 1), ("C6H12O6+Cu", 1), ("CH3(CH2)10COOH+H", 1),
            ("C60H100N20O30S5+H", 1), ("C20H30Br2Cl3FeSe+K", 2), ("H2O", 0), ("C((CH3)2)3+Li", 1),
            ("C27H46O+Cl", -1), ("C55H72MgN4O5+H", 1), ("C63H88CoN14O14P+H", 2)]
SETTINGS = [(0.01, 10000), (0.006728, 1750), (0.00094192, 12500)]  # default + generate_ds_config.py 70K / 500K


def _native_all(sf, z, sigma, pts, cap=2048):
    w = IsocalcWrapper({"charge": {"polarity": "+" if z >= 0 else "-", "n_charges": abs(z)},
                        "isocalc_sigma": sigma, "isocalc_pts_per_mz": pts})
    w.charge = z
    return w._isodist(sf, cap)


@pytest.mark.parametrize("sigma,pts", SETTINGS)
def test_native_matches_oracle(sigma, pts):
    for sf, z in FORMULAS:
        got_m, got_i = _native_all(sf, z, sigma, pts)
        ref_m, ref_i = O.isotope_centroids(sf, z, sigma, pts)
        assert len(got_m) == len(ref_m), sf
        np.testing.assert_allclose(got_m, ref_m, rtol=0, atol=1e-9, err_msg=sf)
        np.testing.assert_allclose(got_i, ref_i, rtol=1e-9, atol=1e-9, err_msg=sf)
        assert np.all(np.diff(got_m) > 0) and got_i.max() == pytest.approx(100.0)


def test_random_formulas_match_oracle():
    rng = np.random.default_rng(5)
    for _ in range(40):
        c, h, n, o = rng.integers(1, 40), rng.integers(1, 80), rng.integers(0, 6), rng.integers(0, 15)
        p, s = rng.integers(0, 3), rng.integers(0, 3)
        sf = f"C{c}H{h}" + (f"N{n}" if n else "") + (f"O{o}" if o else "") + (f"P{p}" if p else "") + \
            (f"S{s}" if s else "")
        ad = ["+H", "+Na", "+K", "-H"][rng.integers(0, 4)]
        z = -1 if ad == "-H" else 1
        got_m, got_i = _native_all(sf + ad, z, 0.01, 10000)
        ref_m, ref_i = O.isotope_centroids(sf + ad, z, 0.01, 10000)
        assert len(got_m) == len(ref_m)
        np.testing.assert_allclose(got_m, ref_m, atol=1e-9)
        np.testing.assert_allclose(got_i, ref_i, rtol=1e-9, atol=1e-9)


def test_monoisotopic_known_answers():
    # literature [M+H]+ / [M-H]- values (electron mass included)
    kat = {("C6H12O6+H", 1): 181.070665, ("C6H12O6-H", -1): 179.056113, ("C6H12O6+Na", 1): 203.052609,
           ("C40H80NO8P+H", 1): 734.569432, ("C10H16N5O13P3+H", 1): 508.00302}
    w = IsocalcWrapper(ds_config()["isotope_generation"])
    for (sf, z), mz in kat.items():
        assert O.monoisotopic_mz(sf, z) == pytest.approx(mz, abs=5e-6)
        w.charge = z
        m, _ = w._isodist(sf)
        assert m[0] == pytest.approx(mz, abs=1e-4), sf  # first centroid = monoisotopic peak at 10000 pts/mz


def test_isotope_ratio_known_answer():
    # C60: M+1/M = 60 * 1.07/98.93 (binomial) -> 64.9 %; resolved carbon envelope at sigma 0.01
    m, i = _native_all("C60", 0, 0.01, 10000)
    assert i[0] == pytest.approx(100.0)
    assert i[1] == pytest.approx(100 * 60 * 0.0107 / 0.9893, rel=2e-3)
    assert m[1] - m[0] == pytest.approx(1.0033548, abs=1e-4)


def test_parse_and_invalid_formulas():
    assert O.parse_sum_formula("CH3(CH2)10COOH") == {"C": 12, "H": 24, "O": 2}
    assert O.parse_sum_formula("C6H12O6+Na-H") == {"C": 6, "H": 11, "O": 6, "Na": 1}
    for bad in ["", "Xy2", "C6H12O6-Na", "C(", "2C", "C6H12O6+", "C)"]:
        with pytest.raises(O.InvalidFormulaError):
            O.parse_sum_formula(bad)
        with pytest.raises(ValueError):
            _native_all(bad, 1, 0.01, 10000)


def test_wrapper_first_six_and_invalid():
    w = IsocalcWrapper(ds_config()["isotope_generation"])
    c = w.isotope_peaks("C60H100N20O30S5", "+H")
    ref_m, ref_i = O.isotope_centroids("C60H100N20O30S5+H", 1, 0.01, 10000)
    assert len(c.mzs) == 6
    np.testing.assert_allclose(c.mzs, ref_m[:6], atol=1e-9)
    np.testing.assert_allclose(c.ints, ref_i[:6], rtol=1e-9)
    # test_isocalc_wrapper.py:27-28: invalid input -> empty centroids
    assert w.isotope_peaks(None, "+H") == Centroids([], [])
    assert w.isotope_peaks("Au", None) == Centroids([], [])
    assert w.isotope_peaks("C6H12O6", "-Na") == Centroids([], [])


def test_batch_equals_single():
    w = IsocalcWrapper(ds_config()["isotope_generation"])
    pairs = [("C6H12O6", "+H"), ("Xy", "+H"), (None, "+Na"), ("C40H80NO8P", "+K"), ("C6H12O6", "-Na")] * 7
    batch = w.isotope_peaks_batch(pairs, n_threads=4)
    for (sf, a), b in zip(pairs, batch):
        s = w.isotope_peaks(sf, a)
        assert len(s.mzs) == len(b.mzs)
        np.testing.assert_array_equal(np.asarray(s.mzs), np.asarray(b.mzs))
        np.testing.assert_array_equal(np.asarray(s.ints), np.asarray(b.ints))


def test_formatted_iso_peaks_correct_input():
    # test_theor_peaks_gen.py:30-37
    w = IsocalcWrapper(ds_config()["isotope_generation"])
    with mock.patch.object(IsocalcWrapper, "isotope_peaks", return_value=Centroids([100.], [1000.])):
        assert list(w.formatted_iso_peaks(0, 9, "Au", "+H"))[0] == \
            "0\t9\t+H\t0.010000\t1\t10000\t{100.000000}\t{1000.000000}\t{}\t{}"


def test_find_sf_adduct_cand_and_filters():
    # test_theor_peaks_gen.py:40-69
    with mock.patch.object(TPG, "DECOY_ADDUCTS", []):
        gen = TPG.TheorPeaksGenerator(None, {"fs": {"base_path": ""}}, ds_config())
        with pytest.raises(AssertionError):
            gen.find_sf_adduct_cand([], {})
        assert gen.find_sf_adduct_cand([(0, "He"), (9, "Au")], {("He", "+H"), ("Au", "+H")}) == \
            [(0, "He", "+Na"), (9, "Au", "+Na")]
    cfg = ds_config()
    cfg["isotope_generation"]["adducts"] = ["+H"]
    cfg["database"]["filters"] = ["Organic"]
    gen = TPG.TheorPeaksGenerator(None, {"fs": {"base_path": ""}}, cfg)
    assert gen.apply_database_filters([(0, "He"), (9, "CO2")]) == [(9, "CO2")]
    assert not gen._valid_sf_adduct(None, "+H") and not gen._valid_sf_adduct("C6H12O6", "-Na")
    assert gen._valid_sf_adduct("C6H12O6", "-H")


def test_generate_theor_peaks():
    # test_theor_peaks_gen.py:72-87: one formatted row per (sf_id, sf, adduct); the rows are returned (the
    # reference COPYs them into Postgres, which is out of scope)
    gen = TPG.TheorPeaksGenerator(None, {"fs": {"base_path": ""}}, ds_config())
    with mock.patch.object(IsocalcWrapper, "isotope_peaks_batch",
                           lambda self, pairs, n_threads=0: [Centroids([100.], [1000.])] * len(pairs)):
        lines = gen.generate_theor_peaks([(9, "Au", "+Na")])
        assert lines == ["0\t9\t+Na\t0.010000\t1\t10000\t{100.000000}\t{1000.000000}\t{}\t{}"]
        # run(): only the pairs not stored yet
        stored = {("Au", a) for a in gen.adducts} | {("Au", a) for a in TPG.DECOY_ADDUCTS if a != "+He"}
        rows = gen.run([(9, "Au")], stored)
        assert [r.split("\t")[2] for r in rows] == ["+He"]


def test_theor_peaks_df_feeds_formulas_segm():
    from sm_distributed_amd.formulas import FormulasSegm
    df = TPG.theor_peaks_df([(1, "C6H12O6"), (2, "C40H80NO8P"), (3, "Xy")], ["+H", "+Na"],
                            ds_config()["isotope_generation"])
    assert sorted(zip(df.sf_id, df.adduct)) == [(1, "+H"), (1, "+Na"), (2, "+H"), (2, "+Na")]
    f = FormulasSegm(df)
    peaks = f.get_sf_peak_df()
    assert peaks.mz.is_monotonic_increasing and len(peaks) == sum(len(m) for m in df.centr_mzs)
    assert f.get_sf_peak_ints()[(1, "+H")][0] == pytest.approx(100.0)
