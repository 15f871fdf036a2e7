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
