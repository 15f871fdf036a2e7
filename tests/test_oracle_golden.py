"""The oracle is pinned: it reproduces the committed golden tables, the structural facts of the
reference's golden CSV, and the imzML reader round-trips our own synthetic example.  CPU only."""
import os

import numpy as np
import pandas as pd
import pytest

from oracle import msm_oracle as O
from tests.parity_cases import make_case, oracle_run, sf_peak_df, sf_peak_ints

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", ["basic", "dups", "conn8_border1"])
def test_oracle_reproduces_golden(name):
    ds, ions, ppm, kw = make_case(name)
    _, df = oracle_run(ds, ions, ppm, **kw)
    exp = pd.read_csv(os.path.join(GOLDEN, f"synth_{name}_expected.csv"))
    got = df.reset_index()
    assert list(zip(got.sf_id, got.adduct)) == list(zip(exp.sf_id, exp.adduct))
    for c in ("chaos", "spatial", "spectral", "msm"):
        np.testing.assert_allclose(got[c].values, exp[c].values, rtol=0, atol=1e-12)


def test_imzml_reader_on_synthetic_example():
    from scripts.make_golden import example_ions, synthetic_example_spectra
    from sm_distributed_amd.imzml import read_imzml
    s = read_imzml(os.path.join(GOLDEN, "synthetic_example.imzML"))
    ref = synthetic_example_spectra()
    np.testing.assert_array_equal(s.sp_off, ref.sp_off)
    np.testing.assert_array_equal(s.mz, ref.mz)
    np.testing.assert_array_equal(s.ints, ref.ints)
    assert s.coords.tolist() == ref.coords.tolist()
    pm, dims = s.pixel_map_dims()
    assert dims == (3, 3) and pm.tolist() == list(range(9))
    ions = example_ions()
    imgs = O.compute_sf_images(s.spectra(), pm, dims, sf_peak_df(ions), 100.0)
    df = O.sf_image_metrics(imgs, sf_peak_ints(ions), 3, 3, 30).reset_index()
    exp = pd.read_csv(os.path.join(GOLDEN, "synthetic_example_expected.csv"))
    for c in ("chaos", "spatial", "spectral", "msm"):
        np.testing.assert_allclose(df[c].values, exp[c].values, atol=1e-12)


def test_imzml_processed_roundtrip(tmp_path):
    from sm_distributed_amd import synthetic as syn
    from sm_distributed_amd.imzml import read_imzml
    from tests.imzml_writer import write_imzml
    ds = syn.make_dataset_np(4, 5, 50, seed=9)
    write_imzml(str(tmp_path / "p.imzML"), ds, continuous=False)
    s = read_imzml(str(tmp_path / "p.imzML"))
    np.testing.assert_array_equal(s.mz, ds.mz)
    np.testing.assert_array_equal(s.ints, ds.ints)
    np.testing.assert_array_equal(s.sp_off, ds.sp_off)


def test_measure_of_chaos_structure():
    """Every chaos value is 1 - int/(nlevels*int) (the structure of the reference golden CSV)."""
    ds, ions, ppm, kw = make_case("basic")
    exp = pd.read_csv(os.path.join(GOLDEN, "synth_basic_expected.csv"))
    for c in exp.chaos.values[exp.chaos.values > 0][:50]:
        found = any(abs((1 - c) * 30 * n - round((1 - c) * 30 * n)) < 1e-6 for n in range(4, 1025))
        assert found


def test_chaos_small_known_images():
    # a solid 5x5 block inside a 9x9 image: every level keeps one component after dilate/erode
    im = np.zeros((9, 9))
    im[2:7, 2:7] = 1.0
    # 25 positive pixels, levels 0..28/29 keep the block (1 component each), level 1.0 empty -> 29/(30*25)
    assert O.measure_of_chaos(im, 30) == pytest.approx(1 - 29 / (30 * 25))
    assert np.isnan(O.measure_of_chaos(np.zeros((4, 4)), 30))
    im2 = np.zeros((5, 5))
    im2[0, 0] = im2[4, 4] = im2[2, 2] = 1.0
    assert np.isnan(O.measure_of_chaos(im2, 30))  # < 4 positive pixels


def test_isotope_metrics_restatement():
    imgs = [np.array([0.0, 2.0, 4.0, 0.0]), np.array([0.0, 1.0, 2.0, 0.0]), np.zeros(4)]
    theor = [100.0, 50.0, 10.0]
    # spatial: image 2 is constant -> corrcoef NaN -> average NaN
    assert np.isnan(O.isotope_image_correlation(imgs, weights=theor[1:]))
    assert O.isotope_image_correlation(imgs[:2], weights=theor[1:2]) == pytest.approx(1.0)
    s = np.array([6.0, 3.0, 0.0])
    t = np.array(theor)
    exp = 1 - np.mean(np.abs(t / np.linalg.norm(t) - s / np.linalg.norm(s)))
    assert O.isotope_pattern_match(imgs, theor) == pytest.approx(exp)
