"""Config 5 (stress) on one GPU: every rank's shard of the 8-way plan of BASELINE config 5 (GPU only).

1000x1000 px, Poisson(5000) centroids per spectrum (~5e9 points, 60 GB resident: every rank holds the whole
dataset), 40,000 synthetic formulas searched in both polarities (+H/+Na/+K at charge +1, -H/+Cl/+Br at charge -1,
'-H' vetted by the formula's composition as theor_peaks_gen.py:46-51 does, distinct decoys per fdr.py:42-48) =
3.9M ions; plan_shards cuts them into 8 m/z-contiguous shards (the 8-GPU run of config 5).  Each shard is scored in
turn by the product per-rank scorer (distributed._device_rows: m/z slice, sort, window search, images on the wide
pass with the pixel-indexed pass taking its rejects, scores), as rank r of the 8-GPU run would, and:

* the slice holds exactly the dataset's points in the shard's m/z range (f64 comparison over all 5e9 points);
* every window's [lo, hi) equals an independent torch.searchsorted of its f64 bounds (formula_imager_segm.py:79-82)
  over the slice's sorted m/z: window membership bit-exact;
* the shard's rows are exactly its ions with >= 1 non-empty window (formula_img_validator.py:115-118);
* the rows of all 8 shards, reassembled by rows_to_frame (the rank-0 assembly), cover every ion with a hit once;
* a seeded sample of every shard (32 uniform ions, up to 8 planted targets, and ions of every pass that scored some: wide
  pass and pixel-indexed pass, up to 4 each; both polarities) is imaged and scored by the oracle from every point of its
  windows (formula_imager_segm.py:66-92 + formula_img_validator.py:72-84): metrics within 1e-5.
H1 (formula_imager_segm.py:68-69 chunking) does not arise: windows are complete on the device by construction.
"""
import numpy as np
import pytest

from tests.sample_check import assert_rows_match, oracle_rows, planted_ions

pytestmark = pytest.mark.gpu

PPM, NLEVELS, WORLD = 2.0, 30, 8
SMG_ION_DENSE, SMG_ION_WIDE = 0x2, 0x20


@pytest.fixture(scope="module")
def c5():
    import torch
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
    torch.cuda.synchronize()
    return dict(ions=ions, peaks=peaks, formulas=formulas, conf=conf, dims=dims)


def _range_count(mz, lo, hi, block=1 << 28):
    """#points with lo <= mz <= hi, compared in float64, over a device f32 tensor."""
    import torch
    n = 0
    for a in range(0, mz.numel(), block):
        x = mz[a:a + block].to(torch.float64)
        n += int(((x >= lo) & (x <= hi)).sum().item())
    return n


@pytest.mark.timeout(1100)
def test_config5_all_eight_shards(c5):
    import torch
    from sm_distributed_amd import distributed as D
    ions, peaks, formulas, conf = c5["ions"], c5["peaks"], c5["formulas"], c5["conf"]
    rng = np.random.default_rng(55)
    planted = planted_ions(ions)
    rows_all, picks, stats = [], [], []
    n_seen = 0
    for r in range(WORLD):
        plan = D.plan_shards(formulas, peaks, PPM, WORLD, r)
        n_shard = len(plan.ion_idx)
        assert 0.02 * ions.n_ions < n_shard < 0.5 * ions.n_ions, (r, n_shard)
        n_seen += n_shard
        rows, ims = D._device_rows(plan, peaks, conf)
        sl = ims.peaks
        # the slice: exactly the points in [mz_lo, mz_hi] of the whole dataset
        assert sl.n_points == _range_count(peaks.mz, plan.mz_lo, plan.mz_hi), r
        # window membership: an independent f64 searchsorted over the slice's sorted m/z
        pmz = ims.ions_dev.peak_mz
        lower = pmz - pmz * PPM * 1e-6
        upper = pmz + pmz * PPM * 1e-6
        s64 = sl.mz_sorted.to(torch.float64)
        lo = torch.searchsorted(s64, lower, right=False)
        hi = torch.searchsorted(s64, upper, right=True)
        pad = pmz < 0  # padding windows of the layout (no theoretical peak): empty
        lo = torch.where(pad, ims.lo, lo)
        hi = torch.where(pad, ims.lo, hi)
        assert torch.equal(ims.lo[~pad], lo[~pad]) and torch.equal(ims.hi - ims.lo, hi - lo), f"rank {r} windows"
        del s64
        # rows = the shard's ions with >= 1 non-empty window (their global table index)
        cnt = torch.zeros(lo.numel() + 1, dtype=torch.int64, device=lo.device)
        torch.cumsum((hi - lo > 0).to(torch.int64), 0, out=cnt[1:])
        woff = ims.ions_dev.win_off
        has = ((cnt[woff[1:]] - cnt[woff[:-1]]) > 0).cpu().numpy()
        rr = rows.cpu().numpy()
        k = len(has)
        glob = rr[:k, 0]
        assert ((glob >= 0) == has).all(), f"rank {r}: rows != ions with hits"
        assert (rr[k:, 0] < 0).all()
        kept = glob[glob >= 0].astype(np.int64)
        assert np.isin(kept, plan.ion_idx).all()
        # sample: uniform, planted, and ions of each pass that scored some (flags of this shard's launch)
        fl = ims.score_flags.cpu().numpy()[:k].astype(np.int64)
        g = glob.astype(np.int64)
        wide = g[(glob >= 0) & ((fl & SMG_ION_WIDE) != 0)]
        pix = g[(glob >= 0) & ((fl & SMG_ION_DENSE) != 0) & ((fl & SMG_ION_WIDE) == 0)]
        lds = g[(glob >= 0) & ((fl & SMG_ION_DENSE) == 0)]
        pick = [rng.choice(plan.ion_idx, size=32, replace=False), np.intersect1d(planted, plan.ion_idx)[:8]]
        for cat in (wide, pix, lds):
            if len(cat):
                pick.append(rng.choice(cat, size=min(4, len(cat)), replace=False))
        picks.append(np.unique(np.concatenate(pick)))
        stats.append((r, n_shard, int(has.sum()), len(wide), len(pix), len(lds), sl.n_points, plan.mz_lo, plan.mz_hi))
        rows_all.append(rows)
        gkeys = plan.global_keys
        del ims, sl, lo, hi, lower, upper
        torch.cuda.synchronize()
    assert n_seen == ions.n_ions
    # the rank-0 assembly of all shards: one row per ion with a hit, each exactly once
    table = torch.cat(rows_all)
    df = D.rows_to_frame(table, gkeys)
    assert len(df) == sum(s[2] for s in stats)
    gi = table[:, 0].cpu().numpy()
    gi = gi[gi >= 0].astype(np.int64)
    assert len(np.unique(gi)) == len(gi)
    assert list(df.columns) == ["chaos", "spatial", "spectral", "msm"] and np.isfinite(df.to_numpy()).all()
    np.testing.assert_array_equal(df.msm.to_numpy(), (df.chaos * df.spatial * df.spectral).to_numpy())
    # the sampled ions: the oracle from every point of their windows
    pick = np.unique(np.concatenate(picks))
    res, wins, sizes, npts, wall = oracle_rows(ions, pick, peaks, c5["dims"], PPM, NLEVELS)
    tab = table.cpu().numpy()
    got = {int(x[0]): x[1:5] for x in tab if x[0] >= 0}
    assert {x[0] for x in res} == {int(i) for i in pick if int(i) in got}
    n_pos = assert_rows_match(res, lambda i: got[i])
    pol = {ions.adducts[x[0]] for x in res}
    assert pol & {"+H", "+Na", "+K"} and pol & {"-H", "+Cl", "+Br"}, pol
    for s in stats:
        print("rank %d/8: %s ions, %s with rows (wide %s, pixel-indexed %s, LDS %s), slice %s points [%.2f, %.2f]"
              % (s[0], f"{s[1]:,}", f"{s[2]:,}", f"{s[3]:,}", f"{s[4]:,}", f"{s[5]:,}", f"{s[6]:,}", s[7], s[8]))
    print(f"config 5, 8 shards: {len(df):,} rows reassembled of {ions.n_ions:,} ions; {len(res)} sampled ions within "
          f"1e-5 of the oracle ({n_pos} with msm > 0; {sum(len(p) for p in picks)} picks), oracle wall {wall:.1f}s, "
          f"{npts:,} window points")
