"""The drop-in API's device paths against the oracle and the committed fixtures (GPU only).

* legacy ``formula_imager.sample_spectra`` -> ``smg_sample_spectra``: the reference KAT
  (sm/engine/tests/msm_basic/test_formula_imager.py:11-26, transcribed in tests/golden/kats.json) and random
  spectra against the oracle (formula_imager.py:9-38); window sums are the same f64 subtraction, so bit-exact;
* the generic ``compute(iso_images_sparse, sf_ints)`` path (formula_img_validator.py:58-86):
  ``get_compute_img_metrics`` and ``sf_image_metrics`` over a LocalRDD of scipy images ->
  ``engine.metrics_from_images`` -> ``smg_ion_metrics`` with SMG_HITS_SPLIT_F64 hits;
* ``IonImageSet.collect()`` (compute_sf_images' lazily materialised image lists) against the oracle's
  ``_img_pairs_to_list`` semantics (formula_imager_segm.py:95-109): same ions, list lengths, None gaps,
  identical pixel multisets, values within 1e-6 relative (coo.toarray() sums);
* the committed golden tables (tests/golden/synth_*_expected.csv, synthetic_example_expected.csv) through
  compute_sf_images + sf_image_metrics on the device.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest
from scipy.sparse import coo_matrix

from tests.parity_cases import make_case, oracle_run, sf_peak_df, sf_peak_ints

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
METRIC_ATOL = 1e-5


class _DS:
    def __init__(self, spectra, dims=(1, 1)):
        self._spectra = spectra
        self._dims = dims

    def get_spectra(self):
        from sm_distributed_amd.rdd import LocalRDD
        return LocalRDD(self._spectra)

    def get_dims(self):
        return self._dims


class _Formulas:
    def __init__(self, lower, upper, peak_map):
        self.lower, self.upper, self.peak_map = np.asarray(lower), np.asarray(upper), np.asarray(peak_map)

    def get_sf_peak_bounds(self):
        return self.lower, self.upper

    def get_sf_peak_map(self):
        return self.peak_map


def test_sample_spectra_kat():
    """test_formula_imager.py:11-26 through the HIP sampler."""
    from sm_distributed_amd.formula_imager import sample_spectra
    k = json.load(open(os.path.join(GOLDEN, "kats.json")))["sample_spectra_2by3"]
    spectra = [(sp, np.array(mz, np.float64), np.array(cum, np.float64)) for sp, mz, cum in k["spectra"]]
    got = sample_spectra(None, _DS(spectra), _Formulas(k["lower"], k["upper"], k["sf_peak_map"])).collect()
    assert got == [((a, b), (c, d)) for (a, b), (c, d) in k["expected"]]


def test_sample_spectra_random_matches_oracle():
    from oracle import msm_oracle as O
    from sm_distributed_amd.formula_imager import sample_spectra
    rng = np.random.default_rng(17)
    spectra = []
    for sp in range(300):
        n = int(rng.integers(0, 60))
        mz = np.sort(rng.uniform(100, 110, n))
        it = np.where(rng.random(n) < 0.1, 0.0, rng.lognormal(0, 3, n))   # zeros and tiny values (< 0.001 cut)
        spectra.append((sp, mz, np.concatenate([[0.0], np.cumsum(it)])))
    centers = rng.uniform(100, 110, 80)
    lower, upper = O.legacy_peak_bounds(centers, 2000.0)
    peak_map = np.stack([np.arange(80) // 4, np.arange(80) % 4], axis=1)
    got = sample_spectra(None, _DS(spectra), _Formulas(lower, upper, peak_map)).collect()
    exp = O.sample_spectra(spectra, lower, upper, peak_map)
    assert len(exp) > 100
    assert got == exp  # same f64 subtraction of the same cumulative values: bit-exact, same flatMap order


def _scored(df):
    return df.sort_index()


@pytest.mark.parametrize("name", ["basic", "dups", "kmix"])
def test_sf_image_metrics_generic_images_match_oracle(name):
    """sf_image_metrics over a LocalRDD of scipy images (not an IonImageSet): the metrics_from_images path."""
    from sm_distributed_amd.formula_img_validator import get_compute_img_metrics, sf_image_metrics
    from sm_distributed_amd.rdd import LocalRDD
    ds, ions, ppm, kw = make_case(name)
    imgs, exp = oracle_run(ds, ions, ppm, **kw)
    ints = sf_peak_ints(ions)
    pm, dims = ds.pixel_map_dims()

    class F:
        def get_sf_peak_ints(self):
            return ints

    conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    got = sf_image_metrics(LocalRDD(list(imgs.items())), None, F(), _DS([], dims), conf)
    got, exp = _scored(got), _scored(exp)
    assert list(got.index) == list(exp.index)
    for c in ("chaos", "spatial", "spectral", "msm"):
        err = np.abs(got[c].to_numpy() - exp[c].to_numpy())
        assert err.max(initial=0.0) <= METRIC_ATOL, (c, float(err.max()))
    # and ion by ion through compute() (formula_img_validator.py:72-84)
    compute = get_compute_img_metrics(np.zeros(dims), conf["image_generation"])
    for key in list(imgs)[:6]:
        c, s, p = compute(imgs[key], ints[key])
        np.testing.assert_allclose([c, s, p], exp.loc[key, ["chaos", "spatial", "spectral"]].to_numpy(),
                                   atol=METRIC_ATOL, rtol=0)


def test_compute_pads_short_image_lists():
    """compute() pads the image list with empty images up to len(sf_ints) (formula_img_validator.py:73-75)."""
    from oracle import msm_oracle as O
    from sm_distributed_amd.formula_img_validator import get_compute_img_metrics
    rng = np.random.default_rng(3)
    dims = (12, 14)
    a = rng.random(dims) * (rng.random(dims) < 0.4)
    b = a * 0.5 + rng.random(dims) * (rng.random(dims) < 0.1)
    imgs = [coo_matrix(a), None, coo_matrix(b)]
    ints = [100.0, 30.0, 10.0, 2.0, 0.5]
    compute = get_compute_img_metrics(np.zeros(dims), {"nlevels": 30})
    got = compute(imgs, ints)
    exp = O.compute_img_metrics(imgs, ints, dims[0], dims[1], 30)
    np.testing.assert_allclose(got, exp, atol=METRIC_ATOL, rtol=0)


@pytest.mark.parametrize("name", ["basic", "dups", "zeros_rect", "kmix", "boundary"])
def test_ion_image_set_collect_matches_oracle(name):
    from sm_distributed_amd.dataset import DeviceDataset
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    ds, ions, ppm, kw = make_case(name)
    ref, _ = oracle_run(ds, ions, ppm, **kw)
    ims = compute_sf_images(None, DeviceDataset(ds), sf_peak_df(ions), ppm)
    got = dict(ims.collect())
    assert set(got) == set(ref)
    assert ims.count() == len(ref)
    nrows, ncols = ds.pixel_map_dims()[1]
    checked = 0
    for key, rl in ref.items():
        gl = got[key]
        assert len(gl) == len(rl), key
        for g, r in zip(gl, rl):
            assert (g is None) == (r is None), key
            if r is None:
                continue
            gc, rc = g.tocoo(), r.tocoo()
            assert g.shape == r.shape == (nrows, ncols)
            assert sorted((gc.row * ncols + gc.col).tolist()) == sorted((rc.row * ncols + rc.col).tolist())
            np.testing.assert_allclose(g.toarray(), r.toarray(), rtol=1e-6, atol=0)
            checked += 1
    assert checked > 0
    # take() / keys_with_images() agree with collect()
    assert [k for k, _ in ims.take(3)] == [k for k, _ in ims.collect()[:3]]
    assert sorted(ims.keys_with_images()) == sorted(ref)


def _api_table(spectra, ions, ppm, img_conf):
    from sm_distributed_amd.dataset import DeviceDataset
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    from sm_distributed_amd.formula_img_validator import sf_image_metrics
    from sm_distributed_amd.formulas import FormulasSegm
    dds = DeviceDataset(spectra)
    formulas = FormulasSegm.from_ion_table(ions, ppm)
    ims = compute_sf_images(None, dds, formulas.get_sf_peak_df(), ppm)
    return sf_image_metrics(ims, None, formulas, dds, {"image_generation": img_conf})


def _check_against_csv(df, csv):
    exp = pd.read_csv(csv).set_index(["sf_id", "adduct"]).sort_index()
    got = df.sort_index()
    assert list(got.index) == list(exp.index)
    for c in ("chaos", "spatial", "spectral", "msm"):
        err = np.abs(got[c].to_numpy() - exp[c].to_numpy())
        assert err.max(initial=0.0) <= METRIC_ATOL, (c, float(err.max()))


@pytest.mark.parametrize("name", ["basic", "dups", "conn8_border1"])
def test_golden_tables_through_device_api(name):
    ds, ions, ppm, kw = make_case(name)
    conf = {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False,
            "chaos_connectivity": kw.get("connectivity", 4), "chaos_erosion_border": kw.get("erosion_border", 0)}
    _check_against_csv(_api_table(ds, ions, ppm, conf), os.path.join(GOLDEN, f"synth_{name}_expected.csv"))


def test_synthetic_example_imzml_through_device_api():
    """Config-1 shaped input (3x3 continuous imzML written by our writer) read by our imzML reader, scored on the
    device, against the committed table."""
    from scripts.make_golden import example_ions
    from sm_distributed_amd.imzml import read_imzml
    spectra = read_imzml(os.path.join(GOLDEN, "synthetic_example.imzML"))
    df = _api_table(spectra, example_ions(), 100.0, {"ppm": 100.0, "nlevels": 30, "q": 99,
                                                    "do_preprocessing": False})
    _check_against_csv(df, os.path.join(GOLDEN, "synthetic_example_expected.csv"))


def test_image_set_survives_a_later_search_at_another_ppm():
    """An IonImageSet keeps its own duplicate flags: scoring it after another compute_sf_images on the same
    resident dataset (another ppm re-flags and re-sorts it) gives the same table as scoring it right away."""
    from sm_distributed_amd.dataset import DeviceDataset
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    from sm_distributed_amd.formula_img_validator import sf_image_metrics
    from sm_distributed_amd.formulas import FormulasSegm
    ds, ions, ppm, kw = make_case("dups")
    dds = DeviceDataset(ds)
    formulas = FormulasSegm.from_ion_table(ions, ppm)
    conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    first = compute_sf_images(None, dds, formulas.get_sf_peak_df(), ppm)
    ref = sf_image_metrics(first, None, formulas, dds, conf).sort_index()
    compute_sf_images(None, dds, formulas.get_sf_peak_df(), ppm / 5.0)   # narrower windows, fewer flags
    again = sf_image_metrics(first, None, formulas, dds, conf).sort_index()
    pd.testing.assert_frame_equal(again, ref)
    _, exp = oracle_run(ds, ions, ppm)
    assert list(ref.index) == list(exp.sort_index().index)


def _align_reference(lo, hi, win_off, kt_off, sel):
    """formula_img_validator.py:73-75 / 115-118 restated: the scored windows of ion i are its first
    kt_off[i+1] - kt_off[i] layout windows, empty runs past them; a row iff some layout window and some of the
    first 32 scored windows are non-empty (and sel)."""
    n = len(win_off) - 1
    lo2 = np.zeros(kt_off[-1], np.int64)
    hi2 = np.zeros(kt_off[-1], np.int64)
    keep = np.zeros(n, bool)
    for i in range(n):
        w = np.arange(win_off[i], win_off[i + 1])
        kt = kt_off[i + 1] - kt_off[i]
        m = min(kt, len(w))
        lo2[kt_off[i]:kt_off[i] + m] = lo[w[:m]]
        hi2[kt_off[i]:kt_off[i] + m] = hi[w[:m]]
        has = bool((hi[w] > lo[w]).any())
        hit = bool((hi2[kt_off[i]:kt_off[i] + min(kt, 32)] > lo2[kt_off[i]:kt_off[i] + min(kt, 32)]).any())
        keep[i] = has and hit and (sel is None or bool(sel[i]))
    return lo2, hi2, keep


@pytest.mark.parametrize("with_sel", [False, True])
def test_align_windows_matches_reference(with_sel):
    """smg_align_windows on ragged layouts: more theoretical peaks than layout windows (padding), fewer
    (truncation), ions without windows, empty windows only, > 32 scored windows."""
    import torch
    from sm_distributed_amd import engine as E
    from sm_distributed_amd._lib import check, lib
    rng = np.random.default_rng(11)
    n = 3000
    k_img = rng.integers(0, 9, n)
    k_img[:5] = [0, 40, 1, 3, 0]
    kt = rng.integers(0, 9, n)
    kt[:5] = [2, 40, 0, 5, 0]
    win_off = np.concatenate([[0], np.cumsum(k_img)]).astype(np.int64)
    kt_off = np.concatenate([[0], np.cumsum(kt)]).astype(np.int64)
    lo = rng.integers(0, 1000, win_off[-1]).astype(np.int64)
    hi = lo + rng.integers(0, 3, win_off[-1]) * rng.integers(0, 2, win_off[-1])
    hi[win_off[1]:win_off[2]][:33] = lo[win_off[1]:win_off[2]][:33]  # ion 1: only its 34th+ windows may hit
    sel = rng.integers(0, 2, n).astype(np.uint8) if with_sel else None
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    lo2 = torch.empty(kt_off[-1], dtype=torch.int64, device="cuda")
    hi2 = torch.empty_like(lo2)
    keep = torch.empty(n, dtype=torch.uint8, device="cuda")
    sel_d = d(sel) if sel is not None else None
    lo_d, hi_d, wo_d, kt_d = d(lo), d(hi), d(win_off), d(kt_off)  # held until the launch has completed
    check(lib().smg_align_windows(E._p(lo_d), E._p(hi_d), E._p(wo_d), E._p(kt_d), E._p(sel_d), n,
                                  E._p(lo2), E._p(hi2), E._p(keep), E._stream(None)), "smg_align_windows")
    torch.cuda.synchronize()
    rl, rh, rk = _align_reference(lo, hi, win_off, kt_off, sel)
    assert np.array_equal(lo2.cpu().numpy(), rl) and np.array_equal(hi2.cpu().numpy(), rh)
    assert np.array_equal(keep.cpu().numpy().astype(bool), rk)


@pytest.mark.parametrize("name", ["basic", "dups", "zeros_rect", "kmix"])
def test_device_iso_image_rows_match_dense_rows_of_oracle_images(name):
    """search_results.iso_image_rows over a device IonImageSet (smg_iso_image_rows: duplicates summed, pixels >
    0.001 ascending, min / max over the whole image; nothing densified) equals search_results.py:88-97 applied to
    the oracle's images (densified there, as the reference does); also after filter_sf_images-style selection."""
    from sm_distributed_amd.dataset import DeviceDataset
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    from sm_distributed_amd.search_results import iso_image_rows
    from tests.test_reference_kats import _dense_rows
    ds, ions, ppm, kw = make_case(name)
    ref, _ = oracle_run(ds, ions, ppm, **kw)
    nrows, ncols = ds.pixel_map_dims()[1]
    ims = compute_sf_images(None, DeviceDataset(ds), sf_peak_df(ions), ppm)
    keys = sorted(ref)
    for sel in (keys, keys[::3]):
        sub = ims if sel is keys else ims.filter_by_keys(pd.MultiIndex.from_tuples(sel, names=["sf_id", "adduct"]))
        got = sorted(iso_image_rows(1, 2, sub, nrows, ncols), key=lambda r: (r[2], r[3], r[4]))
        exp = sorted(_dense_rows(1, 2, [(k, ref[k]) for k in sel], nrows, ncols), key=lambda r: (r[2], r[3], r[4]))
        assert [r[:6] for r in got] == [r[:6] for r in exp]
        assert len(got) > 0
        for g, e in zip(got, exp):
            np.testing.assert_allclose(g[6], e[6], rtol=1e-12, atol=0)
            np.testing.assert_allclose([g[7], g[8]], [e[7], e[8]], rtol=1e-12, atol=0)


def test_device_iso_image_rows_reference_kat():
    """tests/test_search_results.py:59-77 of the reference (2x3 images [[100,0,0],[0,0,0]] and [[0,0,0],[0,0,10]])
    through the device reducer: rows (.., 0, [0], [100], 0, 100) and (.., 1, [5], [10], 0, 10)."""
    import torch
    from sm_distributed_amd import _lib
    from sm_distributed_amd.engine import _p, workspace
    import ctypes
    # packed hits: window 0 = pixel 0 (100), window 1 = pixel 5 (10) split into two duplicates 4 + 6
    f = lambda x: int(np.array([x], np.float32).view(np.uint32)[0])
    hits = np.array([0 | (f(100.0) << 32), (5 | 0x80000000) | (f(4.0) << 32), (5 | 0x80000000) | (f(6.0) << 32)],
                    dtype=np.uint64)
    d = lambda a, dt: torch.from_numpy(np.asarray(a, dtype=dt)).cuda()
    h = d(hits.view(np.int64), np.int64)
    lo, hi = d([0, 1], np.int64), d([1, 3], np.int64)
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    mn, mx = torch.zeros(2, dtype=torch.float64, device="cuda"), torch.zeros(2, dtype=torch.float64, device="cuda")
    pix, val = torch.zeros(3, dtype=torch.int32, device="cuda"), torch.zeros(3, dtype=torch.float64, device="cuda")
    L = _lib.lib()
    sz = ctypes.c_size_t(0)
    _lib.check(L.smg_iso_image_rows_workspace_size(2, 3, ctypes.byref(sz)))
    ws = workspace(sz.value, "cuda", "rows_kat")
    _lib.check(L.smg_iso_image_rows(_p(h), _p(lo), _p(hi), 2, 3, 6, 0.001, _p(cnt), _p(mn), _p(mx), _p(pix), _p(val),
                                    _p(ws), ws.numel(), None))
    torch.cuda.synchronize()
    assert cnt.tolist() == [1, 1] and pix[:2].tolist() == [0, 5] and val[:2].tolist() == [100.0, 10.0]
    assert mn.tolist() == [0.0, 0.0] and mx.tolist() == [100.0, 10.0]


@pytest.mark.gpu
def test_frame_index_stages_in_flight_do_not_share_a_buffer():
    """Three FrameIndex stages queued before any frame() (the staging ring had two buffers and no
    ownership): each frame() returns exactly its own mask's rows, framed in reverse order."""
    import torch

    from sm_distributed_amd.formula_imager_segm import FrameIndex, IonKeys
    dev = torch.device("cuda", 0)
    n = 5000
    keys = np.arange(n, dtype=np.int64) * 3  # sf codes 0..n-1, adduct 0 of 3
    ik = IonKeys(keys, ["+H", "+K", "+Na"])
    rng = np.random.default_rng(7)
    masks = [rng.random(n) < f for f in (0.2, 0.5, 0.8)]
    cols = [torch.from_numpy(rng.random((4, n))).to(dev) for _ in masks]
    fis = []
    for m in masks:
        fi = FrameIndex(ik)
        fi.stage(torch.from_numpy(m).to(dev))
        fis.append(fi)
    for fi, m, c in reversed(list(zip(fis, masks, cols))):
        df = fi.frame(c)
        assert len(df) == int(m.sum())
        np.testing.assert_array_equal(df.to_numpy(), c.cpu().numpy()[:, m].T)
