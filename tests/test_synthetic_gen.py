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
