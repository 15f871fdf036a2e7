"""Config 5 (stress) on one GPU: one rank's shard of the 8-way plan of BASELINE config 5 (GPU only).

1000x1000 px, Poisson(5000) centroids per spectrum (~5e9 points, 60 GB resident: every rank holds the whole
dataset), 40,000 synthetic formulas searched in both polarities (+H/+Na/+K at charge +1, -H/+Cl/+Br at charge -1,
'-H' vetted by the formula's composition as theor_peaks_gen.py:46-51 does, distinct decoys per fdr.py:42-48) =
3.9M ions; plan_shards cuts them into 8 m/z-contiguous shards.  Rank 0's shard (the low-m/z end, where windows are
narrowest and ions most numerous) is scored by the product per-rank scorer (distributed._device_rows: m/z slice,
sort, images on the wide and LDS passes, scores) and a seeded sample of its ions (16 uniform + up to 8 planted) is
imaged and scored by the oracle from every point of their windows: metrics within 1e-5, identical scored set.
H1 (formula_imager_segm.py:68-69 chunking) does not arise: windows are complete on the device by construction.
"""
import numpy as np
import pytest

from tests.sample_check import assert_rows_match, oracle_rows, planted_ions

pytestmark = pytest.mark.gpu

PPM, NLEVELS, WORLD, RANK = 2.0, 30, 8, 0


@pytest.mark.timeout(1100)
def test_config5_rank_shard_sample_matches_oracle():
    import torch
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    from sm_distributed_amd import synthetic as syn
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table_both_polarities(40000, seed=43, decoy_seed=44)
    assert ions.n_ions > 3.5e6 and set(ions.target_adducts) == {"+H", "+Na", "+K", "-H", "+Cl", "+Br"}
    mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 5000.0, seed=42, device="cuda", ions=ions,
                                                  plant_fraction=0.02, plant_seed=45)
    assert info["n_points"] > 4.9e9
    peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    formulas = FormulasSegm.from_ion_table(ions, PPM)
    conf = {"image_generation": {"ppm": PPM, "nlevels": NLEVELS, "q": 99, "do_preprocessing": False}}
    plan = D.plan_shards(formulas, peaks, PPM, WORLD, RANK)
    rows, _ = D._device_rows(plan, peaks, conf)
    rows = rows.cpu().numpy()
    torch.cuda.synchronize()
    n_shard = len(plan.ion_idx)
    assert 0.05 * ions.n_ions < n_shard < 0.5 * ions.n_ions
    got = {int(r[0]): r[1:5] for r in rows if r[0] >= 0}  # global ion index (table order) -> metrics
    assert len(got) > 0.5 * n_shard

    # sample: uniform over the shard + planted targets in it (table order == ion table order)
    rng = np.random.default_rng(55)
    pick = rng.choice(plan.ion_idx, size=16, replace=False)
    planted = np.intersect1d(planted_ions(ions), plan.ion_idx)
    pick = np.unique(np.concatenate([pick, planted[:8]]))
    res, wins, sizes, npts, wall = oracle_rows(ions, pick, peaks, dims, PPM, NLEVELS)
    assert {r[0] for r in res} == {int(i) for i in pick if int(i) in got}
    n_pos = assert_rows_match(res, lambda i: got[i])
    assert len(res) >= 10
    print(f"config 5 rank {RANK}/{WORLD}: shard {n_shard:,} of {ions.n_ions:,} ions ({len(got):,} scored), "
          f"{len(res)} sampled ions within 1e-5 of the oracle ({n_pos} with msm > 0), oracle wall {wall:.1f}s, "
          f"{npts:,} window points")
