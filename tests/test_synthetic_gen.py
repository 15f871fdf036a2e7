"""Synthetic dataset generator (host logic, runs on CPU): the block-by-block recipe used for config-5-sized
datasets yields the same resident layout as the one-shot recipe (spectrum-major, m/z-sorted spectra, pixel
field = spectrum index, planted points inside their spectra)."""
import numpy as np
import pytest
import torch

from sm_distributed_amd import synthetic as syn


def _check_layout(mz, hits, sp_off, n_sp):
    mz = mz.numpy()
    h = hits.numpy().view(np.uint64)
    off = sp_off.numpy()
    assert off[0] == 0 and off[-1] == mz.size == h.size
    pix = (h & np.uint64(0xFFFFFFFF)).astype(np.int64)
    sp = np.repeat(np.arange(n_sp), np.diff(off))
    np.testing.assert_array_equal(pix, sp)
    # m/z non-decreasing inside every spectrum
    d = np.diff(mz)
    same = sp[1:] == sp[:-1]
    assert np.all(d[same] >= 0)
    ints = (h >> np.uint64(32)).astype(np.uint32).view(np.float32)
    assert np.all(np.isfinite(ints)) and np.all(ints >= 0)


@pytest.mark.parametrize("plant", [0.0, 0.2])
def test_chunked_generator_layout(monkeypatch, plant):
    ions = syn.make_ion_table(40, seed=43, decoy_seed=44)
    ref = syn.make_dataset_torch(12, 10, 50, seed=42, device="cpu", ions=ions, plant_fraction=plant)
    monkeypatch.setattr(syn, "CHUNKED_GEN_POINTS", 1)
    monkeypatch.setattr(syn, "CHUNK_POINTS", 700)  # many blocks, some spectra straddling a block edge
    mz, hits, dims, info = syn.make_dataset_torch(12, 10, 50, seed=42, device="cpu", ions=ions,
                                                  plant_fraction=plant)
    assert dims == (12, 10)
    _check_layout(mz, hits, info["sp_off"], 120)
    _check_layout(ref[0], ref[1], ref[3]["sp_off"], 120)
    # same spectrum sizes (the Poisson counts come first from the same generator) and the same planted points
    np.testing.assert_array_equal(info["sp_off"].numpy(), ref[3]["sp_off"].numpy())
    assert info["n_planted_points"] == ref[3]["n_planted_points"]
    assert info["n_planted_ions"] == ref[3]["n_planted_ions"]
    if plant:
        assert info["n_planted_points"] > 0


def test_device_layout_fast_paths_match_generic():
    """device_layout (on CPU tensors): the dense-key, compaction-ordered path for an m/z-sorted sf_peak_df and
    the sort-based path for a shuffled one (or sparse keys) give the same layout; duplicate rows are refused."""
    import pandas as pd
    import pytest as _pt
    from sm_distributed_amd import formula_imager_segm as FIS
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table(300, seed=3, decoy_seed=4)
    df = FormulasSegm.from_ion_table(ions, 2.0).get_sf_peak_df()
    k1, d1, K1 = FIS.device_layout(df, "cpu")
    shuffled = df.sample(frac=1.0, random_state=1)
    sparse = df.copy()
    sparse["sf_id"] = sparse["sf_id"] * 1000003
    for other, scale in ((shuffled, 1), (sparse, 1000003)):
        k2, d2, K2 = FIS.device_layout(other, "cpu")
        assert np.array_equal(k1.keys // k1.n_cat, k2.keys // k2.n_cat // scale)
        assert np.array_equal(K1.numpy(), K2.numpy())
        assert np.array_equal(d1.peak_mz.numpy(), d2.peak_mz.numpy())
        first = d1.peak_mz[d1.win_off[:-1]].numpy()
        assert np.array_equal(first[d1.ion_order.numpy()], first[d2.ion_order.numpy()])
    assert np.all(np.diff(first[d1.ion_order.numpy()]) >= 0)
    with _pt.raises(AssertionError):
        FIS.device_layout(pd.concat([df, df.iloc[:1]]), "cpu")
    with _pt.raises(AssertionError):  # a duplicate that keeps rows == windows: one window left empty
        FIS.device_layout(pd.concat([df.iloc[:-1], df.iloc[:1]]), "cpu")


def test_adduct_shift_follows_polarity():
    """isocalc_wrapper.py:28-32: charge sign from the polarity; m/z = (M - z*m_e)/|z| (the isotope calculator's
    monoisotopic m/z of the same sum formula agrees)."""
    from oracle import isocalc_oracle as I
    M = sum(syn.ELEMENT_MASS[e] * n for e, n in (("C", 6), ("H", 12), ("O", 6)))
    for add, z in (("+H", 1), ("+Na", 1), ("+K", 1), ("-H", -1), ("+Cl", -1), ("+Br", -1)):
        got = M + syn.adduct_shift(add, z)
        exp = I.monoisotopic_mz("C6H12O6" + add, z)
        assert abs(got - exp) < 2e-5, (add, z, got, exp)
    assert syn.adduct_shift("-H", -1) == -syn.ELEMENT_MASS["H"] + syn.ELECTRON_MASS
    assert syn.adduct_shift("+H") == syn.ELEMENT_MASS["H"] - syn.ELECTRON_MASS


def test_config5_ion_table_both_polarities():
    """BASELINE config 5's table: 6 target adducts in both polarities, '-H' only for formulas with hydrogen
    (theor_peaks_gen.py:46-51), decoys per search from DECOY_ADDUCTS minus its targets (fdr.py:42-48), unique
    (sf_id, adduct) keys, negative-mode ions two electron masses off the positive-mode m/z of the same adduct."""
    n = 400
    t = syn.make_ion_table_both_polarities(n, seed=7, decoy_seed=8)
    fs = syn.make_formulas(n, seed=7 + 1000)
    keys = set(zip(t.sf_ids.tolist(), t.adducts.tolist()))
    assert len(keys) == t.n_ions
    tgt = t.target_mask()
    pos, neg = t.sf_ids < n, t.sf_ids >= n
    assert set(t.adducts[tgt & pos]) == {"+H", "+Na", "+K"} and set(t.adducts[tgt & neg]) == {"-H", "+Cl", "+Br"}
    # -H only where the formula has hydrogen; every formula has its +Cl / +Br negative targets
    with_h = fs.has_element("H")
    assert (~with_h).any(), "the generator must produce some formulas without H"
    minus_h = t.sf_ids[tgt & (t.adducts == "-H")] - n
    np.testing.assert_array_equal(np.sort(minus_h), np.nonzero(with_h)[0])
    assert (tgt & neg & (t.adducts == "+Cl")).sum() == n
    # decoys: positive-mode decoys never +H/+Na/+K, negative-mode decoys never +Cl/+Br
    assert not np.isin(t.adducts[~tgt & pos], ["+H", "+Na", "+K"]).any()
    assert not np.isin(t.adducts[~tgt & neg], ["+Cl", "+Br", "-H"]).any()
    td_sf, td_ta, td_da = t.td
    assert len(td_sf) == 2 * n * 3 * 20
    # principal m/z = neutral mass + shift at the ion's charge
    first = t.peak_mz[t.win_off[:-1]]
    i = np.nonzero(tgt & neg & (t.adducts == "+Cl"))[0][0]
    sf = int(t.sf_ids[i]) - n
    assert abs(first[i] - round(fs.mass[sf] + syn.ELEMENT_MASS["Cl"] + syn.ELECTRON_MASS, 6)) < 1e-6
    j = np.nonzero((t.sf_ids == sf) & (t.adducts == "+Cl"))[0]  # the positive-mode '+Cl' decoy, if drawn
    if len(j):
        assert abs((first[i] - first[j[0]]) - 2 * syn.ELECTRON_MASS) < 2e-6
    # the config-3 table is unchanged by the polarity support (same RNG stream, charge +1)
    c3 = syn.make_ion_table(50, seed=43, decoy_seed=44)
    assert c3.charge is None and c3.is_target is None


def test_formulas_are_unique_compositions_in_range():
    fs = syn.make_formulas(3000, seed=3)
    assert len(set(fs.sf.tolist())) == 3000
    assert fs.mass.min() >= 150.0 and fs.mass.max() <= 900.0
    el = np.array([syn.ELEMENT_MASS[e] for e in syn.FORMULA_ELEMENTS])
    np.testing.assert_allclose(fs.counts @ el, fs.mass)


def test_theor_alignment_identity_fast_path_matches_generic():
    """sf_image_metrics' theoretical-intensity alignment (formula_img_validator._theor_arrays, run here on CPU
    tensors): the identity fast path (layout ions == the table's ions) and the key-search path give the
    intensities of every ion (formula_img_validator.py:112: sf_peak_ints[(sf_id, adduct)])."""
    from types import SimpleNamespace

    from sm_distributed_amd.formula_imager_segm import IonKeys
    from sm_distributed_amd.formula_img_validator import _theor_arrays
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table(60, seed=3, decoy_seed=4)
    f = FormulasSegm.from_ion_table(ions)
    pk = f.get_sf_peak_ints()
    keys = f.ion_sf.astype(np.int64) * len(f.adducts) + f.ion_adduct_code
    for sel in (np.arange(f.n_ions), np.arange(0, f.n_ions, 3)):  # identity, then a subset (key search)
        ims = SimpleNamespace(ion_keys=IonKeys(keys[sel], f.adducts))
        ims.keys = ims.ion_keys.tuples()
        Kt, vals, off = _theor_arrays(ims, pk, "cpu")
        Kt2, vals2, off2 = _theor_arrays(ims, pk, "cpu")  # the cached alignment
        for (a, b) in ((Kt, Kt2), (vals, vals2), (off, off2)):
            assert torch.equal(a, b)
        exp = [pk[k] for k in ims.keys]
        np.testing.assert_array_equal(Kt.numpy(), [len(e) for e in exp])
        np.testing.assert_array_equal(vals.numpy(), np.concatenate(exp))
        np.testing.assert_array_equal(off.numpy(), np.concatenate([[0], np.cumsum([len(e) for e in exp])]))


def test_layout_cache_is_content_addressed():
    """cached_device_layout: a table with the same contents (another object, e.g. a copy) gets the cached layout; an
    edited table (even in place, same object and buffers) or another adduct category order gets its own; a table with
    a non-Categorical adduct column is never cached."""
    from sm_distributed_amd import formula_imager_segm as FIS
    from sm_distributed_amd.formulas import FormulasSegm
    FIS._LAYOUT_CACHE.clear()
    ions = syn.make_ion_table(200, seed=5, decoy_seed=6)
    df = FormulasSegm.from_ion_table(ions, 2.0).get_sf_peak_df()
    a = FIS.cached_device_layout(df, "cpu")
    assert FIS.cached_device_layout(df.copy(), "cpu") is a
    edited = df.copy()
    mz = edited["mz"].to_numpy()
    mz[5] += 1e-9  # in place: same object, same buffer, other contents
    b = FIS.cached_device_layout(edited, "cpu")
    assert b is not a and not np.array_equal(a[1].peak_mz.numpy(), b[1].peak_mz.numpy())
    renamed = df.copy()
    renamed["adduct"] = renamed["adduct"].cat.rename_categories(lambda c: c + "x")
    assert FIS.cached_device_layout(renamed, "cpu") is not a
    plain = df.copy()
    plain["adduct"] = plain["adduct"].astype(object)
    assert FIS._layout_key(plain, "cpu") is None
    c = FIS.cached_device_layout(plain, "cpu")
    assert np.array_equal(c[0].keys, a[0].keys) and c is not FIS.cached_device_layout(plain, "cpu")
    assert len(FIS._LAYOUT_CACHE) <= FIS._LAYOUT_KEEP
