"""Config 3 at full size through the benched path (GPU only): the drop-in API exactly as bench.py times it, the
8-way sharded path reassembled on one GPU, and the FDR of the full ~1M-row msm table.

* ``compute_sf_images(None, ResidentDataset(peaks), formulas.get_sf_peak_df(), 2.0)`` + ``sf_image_metrics(...)``
  with ``FormulasSegm.from_ion_table`` (bench.py's step; formula_imager_segm.py:142-161,
  formula_img_validator.py:93-122): the table's rows are exactly the ions with >= 1 non-empty window, and a seeded
  ~4600-ion sample across the whole m/z range (4096 uniform + 512 planted) matches the oracle within 1e-5 in the
  DataFrame.  This covers the device layout's fast paths (dense key table, stable compaction of ion_order),
  smg_align_windows, the PeakInts alignment and FrameIndex at 0.98M ions.
* An 8-way plan (distributed.plan_shards): every rank's shard scored on this GPU by the product per-rank scorer
  (``_device_rows``: m/z slice, sort, images, scores) and reassembled by ``rows_to_frame`` gives the single-GPU
  table: the same index in the same order, and metrics equal to 1e-12 (the slice's block prefix sums start at
  other points, so tail-window sums may differ in the last bit; the count of bit-identical values is printed).
* The whole table again with every ion forced onto each dense kernel (smg_debug_force_dense: 1 = the rank-indexed
  wide pass, 2 = the pixel-indexed kernel), independent implementations of the same metrics: the same rows and
  every metric of all ~0.95M rows within 1e-9 of the LDS passes' table (and, with the hot-spot clip, of each
  other), a whole-table cross-check beyond the oracle sample.
* ``estimate_fdr`` (fdr.py:70-88) of the full msm table (sf_image_metrics_est_fdr's join, its exact-zero ties)
  vs the oracle's pandas restatement: identical digitised FDR for every target ion, identical annotations at
  FDR 0.1.
"""
import numpy as np
import pandas as pd
import pytest

from tests.sample_check import assert_rows_match, oracle_rows, planted_ions

pytestmark = pytest.mark.gpu

PPM, NLEVELS = 2.0, 30


@pytest.fixture(scope="module")
def c3():
    import torch
    from sm_distributed_amd import engine as E
    from sm_distributed_amd import synthetic as syn
    from sm_distributed_amd.dataset import ResidentDataset
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    from sm_distributed_amd.formula_img_validator import sf_image_metrics
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table(20000, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(500, 500, 2000.0, seed=42, device="cuda", ions=ions,
                                                  plant_fraction=0.02, plant_seed=45)
    assert info["n_points"] > 4.9e8 and ions.n_ions > 9.5e5
    peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    formulas = FormulasSegm.from_ion_table(ions, PPM)
    conf = {"image_generation": {"ppm": PPM, "nlevels": NLEVELS, "q": 99, "do_preprocessing": False}}
    dds = ResidentDataset(peaks)
    sf_peak_df = formulas.get_sf_peak_df()
    ims = compute_sf_images(None, dds, sf_peak_df, PPM)
    df = sf_image_metrics(ims, None, formulas, dds, conf)
    df2 = sf_image_metrics(compute_sf_images(None, dds, sf_peak_df, PPM), None, formulas, dds, conf)  # warm caches
    torch.cuda.synchronize()
    cnt = (ims.hi - ims.lo).cpu().numpy()
    win_off = ims.ions_dev.win_off.cpu().numpy()
    return dict(ions=ions, peaks=peaks, formulas=formulas, conf=conf, dims=dims, df=df, df2=df2, cnt=cnt,
                win_off=win_off, keys=ims.ion_keys, dds=dds, sf_peak_df=sf_peak_df)


def test_api_table_rows_are_ions_with_hits(c3):
    df, f = c3["df"], c3["formulas"]
    has = np.add.reduceat(c3["cnt"], c3["win_off"][:-1]) > 0
    has &= np.diff(c3["win_off"]) > 0
    exp = pd.MultiIndex.from_arrays([f.ion_sf[has], np.asarray(f.adducts, dtype=object)[f.ion_adduct_code[has]]],
                                    names=["sf_id", "adduct"])
    assert list(df.columns) == ["chaos", "spatial", "spectral", "msm"]
    assert df.index.names == ["sf_id", "adduct"]
    assert df.index.equals(exp), "table rows != ions with >= 1 non-empty window (in (sf_id, adduct) order)"
    assert np.isfinite(df.to_numpy()).all()
    np.testing.assert_array_equal(df.msm.to_numpy(), (df.chaos * df.spatial * df.spectral).to_numpy())
    # a second search (steady state: reused alignment, warm workspaces) gives the same rows and metrics to 1e-12:
    # duplicate pixels are summed by f64 atomics in arrival order (the reference's unstable sort_values leaves the
    # order of a pixel's duplicates unspecified too), so the last bit may differ between runs
    pd.testing.assert_frame_equal(df, c3["df2"], check_exact=False, rtol=0, atol=1e-12)
    a, b = df.to_numpy(), c3["df2"].to_numpy()
    print(f"steady-state rerun: {int((a == b).sum()):,} of {a.size:,} values bit-identical, "
          f"max |diff| {np.abs(a - b).max(initial=0.0):.3e}")


@pytest.mark.timeout(900)
def test_api_table_sample_matches_oracle(c3):
    ions, df = c3["ions"], c3["df"]
    rng = np.random.default_rng(2024)
    pick = rng.choice(ions.n_ions, size=4096, replace=False)
    pick = np.unique(np.concatenate([pick, planted_ions(ions)[:512]]))
    first = ions.peak_mz[ions.win_off[:-1]][pick]
    assert first.min() < 250 and first.max() > 850, "sample must span the m/z range"
    rows, wins, sizes, npts, wall = oracle_rows(ions, pick, c3["peaks"], c3["dims"], PPM, NLEVELS)
    # the windows of the layout (ion-major in (sf_id, adduct) order = the ion table's order) have the oracle's sizes
    np.testing.assert_array_equal(sizes, c3["cnt"][wins])
    scored = {r[0] for r in rows}
    in_table = set(np.nonzero(pd.MultiIndex.from_arrays([ions.sf_ids, ions.adducts]).isin(df.index))[0].tolist())
    assert scored == {int(i) for i in pick if int(i) in in_table}
    tab = df.to_numpy()
    pos = {k: j for j, k in enumerate(df.index)}

    def lookup(i):
        return tab[pos[(int(ions.sf_ids[i]), ions.adducts[i])]]
    n_pos = assert_rows_match(rows, lookup)
    assert n_pos >= 10, "the sample must contain ions with real signal"
    print(f"config 3 API table: {len(rows)} sampled ions within 1e-5 of the oracle ({n_pos} with msm > 0), "
          f"oracle wall {wall:.1f}s, {npts:,} window points")


@pytest.mark.timeout(900)
def test_eight_way_shards_reassemble_single_gpu_table(c3):
    import torch
    from sm_distributed_amd import distributed as D
    world = 8
    rows = []
    plans = [D.plan_shards(c3["formulas"], c3["peaks"], PPM, world, r) for r in range(world)]
    assert sum(len(p.ion_idx) for p in plans) == c3["formulas"].n_ions
    for p in plans:
        rr, _ = D._device_rows(p, c3["peaks"], c3["conf"])
        rows.append(rr)
    torch.cuda.synchronize()
    df = D.rows_to_frame(torch.cat(rows), plans[0].global_keys)
    ref = c3["df"]
    assert df.index.equals(ref.index), "sharded table rows differ from the single-GPU table"
    a, b = df.to_numpy(), ref.to_numpy()
    assert np.abs(a - b).max(initial=0.0) <= 1e-12
    print(f"8-way reassembly: {len(df):,} rows, {int((a == b).sum()):,} of {a.size:,} values bit-identical, "
          f"max |diff| {np.abs(a - b).max(initial=0.0):.3e}")


def _forced_table(c3, mode, conf):
    from sm_distributed_amd import _lib
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    from sm_distributed_amd.formula_img_validator import sf_image_metrics
    L = _lib.lib()
    L.smg_debug_force_dense(mode)
    try:
        ims = compute_sf_images(None, c3["dds"], c3["sf_peak_df"], PPM)
        return sf_image_metrics(ims, None, c3["formulas"], c3["dds"], conf)
    finally:
        L.smg_debug_force_dense(0)


@pytest.mark.timeout(900)
def test_full_table_on_every_kernel(c3):
    ref = c3["df"]
    for mode in (1, 2):
        df = _forced_table(c3, mode, c3["conf"])
        assert df.index.equals(ref.index), f"forced mode {mode}: rows differ"
        d = np.abs(df.to_numpy() - ref.to_numpy())
        assert d.max(initial=0.0) <= 1e-9, (mode, float(d.max()))
        print(f"forced dense mode {mode}: {len(df):,} rows, max |diff| vs the LDS passes {d.max(initial=0.0):.2e}")
    # with the hot-spot clip (q99): the LDS passes, the wide pass and the pixel-indexed kernel agree on every row
    clip = {"image_generation": dict(c3["conf"]["image_generation"], do_preprocessing=True)}
    t0 = _forced_table(c3, 0, clip)
    assert t0.index.equals(ref.index)
    assert not np.allclose(t0.to_numpy(), ref.to_numpy()), "the clip must change some metric"
    for mode in (1, 2):
        df = _forced_table(c3, mode, clip)
        assert df.index.equals(t0.index), f"clip, forced mode {mode}: rows differ"
        d = np.abs(df.to_numpy() - t0.to_numpy())
        assert d.max(initial=0.0) <= 1e-9, (mode, float(d.max()))
        print(f"clip q99, forced dense mode {mode}: max |diff| vs the LDS passes {d.max(initial=0.0):.2e}")


@pytest.mark.timeout(900)
def test_full_table_fdr_matches_oracle(c3):
    from oracle import msm_oracle as O
    from sm_distributed_amd.fdr import FDR
    from sm_distributed_amd.formula_img_validator import sf_image_metrics_est_fdr
    ions, f, df = c3["ions"], c3["formulas"], c3["df"]
    fdr = FDR(0, 0, ions.decoy_sample_size, list(ions.target_adducts))
    sf, ta, da = ions.td
    fdr.td_df = pd.DataFrame({"sf_id": sf, "ta": ta, "da": da})
    got = sf_image_metrics_est_fdr(df, f, fdr)
    sf_msm = f.get_sf_adduct_sorted_df().join(df.msm).fillna(0)
    assert len(sf_msm) == ions.n_ions and (sf_msm.msm == 0).sum() > 1000, "the table must carry zero-msm ties"
    ofdr = O.estimate_fdr(sf_msm, fdr.td_df, list(ions.target_adducts), ions.decoy_sample_size)
    exp = df.join(ofdr, how="inner")[["chaos", "spatial", "spectral", "msm", "fdr"]]
    got, exp = got.sort_index(), exp.sort_index()
    assert got.index.equals(exp.index)
    np.testing.assert_array_equal(got.fdr.to_numpy(), exp.fdr.to_numpy())
    ann = got.index[got.fdr <= 0.1]
    assert ann.equals(exp.index[exp.fdr <= 0.1])
    print(f"full-table FDR: {len(got):,} target rows, {len(ann):,} annotations at FDR 0.1, "
          f"{int((sf_msm.msm == 0).sum()):,} zero-msm ions")
