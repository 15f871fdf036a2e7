"""Device path vs CPU oracle on seeded inputs (GPU only).

Bars (BASELINE.json north_star): window membership bit-exact, summed intensities within 1e-6 relative,
chaos / spatial / spectral / msm within 1e-5 absolute, identical set of scored ions.
"""
import numpy as np
import pytest

from tests.parity_cases import CASES, make_case, oracle_run, sf_peak_df

pytestmark = pytest.mark.gpu

METRIC_ATOL = 1e-5


def _device_run(ds, ions, ppm, nlevels=30, **kw):
    import torch
    from sm_distributed_amd import engine as E
    pm, dims = ds.pixel_map_dims()
    peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
    m, lo, hi = E.run_hot_path(peaks, dions, ppm, nlevels, **kw)
    torch.cuda.synchronize()
    return peaks, m.to_numpy(), lo.cpu().numpy(), hi.cpu().numpy()


_cache = {}


def _run_case(name):
    if name not in _cache:
        ds, ions, ppm, kw = make_case(name)
        imgs, df = oracle_run(ds, ions, ppm, **kw)
        peaks, m, lo, hi = _device_run(ds, ions, ppm, **kw)
        _cache[name] = (ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi)
    return _cache[name]


@pytest.mark.parametrize("name", CASES)
def test_metrics_match_oracle(name):
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case(name)
    has = (m["flags"] & 1) != 0
    dev_keys = set(zip(ions.sf_ids[has].tolist(), ions.adducts[has].tolist()))
    assert dev_keys == set(df.index.tolist()), "scored ion sets differ"
    idx = {k: i for i, k in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))}
    rows = np.array([idx[k] for k in df.index.tolist()], dtype=np.int64)
    for col in ("chaos", "spatial", "spectral", "msm"):
        ref = df[col].to_numpy()
        got = m[col][rows]
        err = np.abs(ref - got)
        assert err.max(initial=0.0) <= METRIC_ATOL, (col, float(err.max()), int(np.argmax(err)))
    # sanity: the case must exercise real signal, not only zeros
    assert (df.msm != 0).sum() > 0 or name in ("boundary", "nlevels1", "row", "column")


@pytest.mark.parametrize("name", ["basic", "dups", "boundary", "large_image"])
def test_window_membership_bit_exact(name):
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case(name)
    from oracle import msm_oracle as O
    mz_sorted = np.sort(ds.mz)
    olo, ohi = O.window_ranges(mz_sorted, ions.peak_mz, ppm)
    np.testing.assert_array_equal(lo, olo)
    np.testing.assert_array_equal(hi, ohi)
    np.testing.assert_array_equal(peaks.mz_sorted.cpu().numpy(), mz_sorted)


@pytest.mark.parametrize("name", ["basic", "dups", "zeros_rect"])
def test_images_match_oracle(name):
    """Per (ion, peak): device image = sorted hits[lo:hi] summed per pixel == oracle coo.toarray()."""
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case(name)
    hits = peaks.hits_sorted.cpu().numpy().view(np.uint64)
    pix = (hits & np.uint64(0x7FFFFFFF)).astype(np.int64)
    val = (hits >> np.uint64(32)).astype(np.uint32).view(np.float32).astype(np.float64)
    nrows, ncols = peaks.nrows, peaks.ncols
    checked = 0
    for i, key in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist())):
        a, b = ions.win_off[i], ions.win_off[i + 1]
        ref = imgs.get(key)
        for k in range(b - a):
            w = a + k
            dense = np.zeros(nrows * ncols)
            np.add.at(dense, pix[lo[w]:hi[w]], val[lo[w]:hi[w]])
            ref_img = ref[k] if (ref is not None and k < len(ref)) else None
            if ref_img is None:
                assert hi[w] == lo[w]
                continue
            r = ref_img.toarray().ravel()
            np.testing.assert_allclose(dense, r, rtol=1e-6, atol=0)
            coo = ref_img.tocoo()
            assert sorted((coo.row * ncols + coo.col).tolist()) == sorted(pix[lo[w]:hi[w]].tolist())
            checked += 1
    assert checked > 0


def test_dense_path_used_when_needed():
    _, _, _, _, _, _, _, m, _, _ = _run_case("big_window")
    assert ((m["flags"] & 8) != 0).any()      # big-ion LDS pass
    _, _, _, _, _, _, _, m, _, _ = _run_case("huge_window")
    assert ((m["flags"] & 2) != 0).any()      # dense global-scratch pass
    # images above 2^18 pixels whose presence bitmap fits the LDS: the rank-indexed wide pass, not the two-level
    # LDS passes (it outruns them there); the two-level passes are checked with smg_debug_force_two_level below
    for name in ("large_image", "large_blobs"):
        _, _, _, _, _, _, _, m, _, _ = _run_case(name)
        has = (m["flags"] & 1) != 0
        assert has.any() and ((m["flags"][has] & (0x20 | 0x10 | 2)) == (0x20 | 2)).all(), name


def test_forced_two_level_large_blobs_reaches_big_pass():
    """With the two-level passes forced, large_blobs exercises the two-level big-ion pass and the olist rebuilt
    from the two-level set (principal windows of 1707..2560 points), and still matches the oracle."""
    from sm_distributed_amd import _lib
    L = _lib.lib()
    L.smg_debug_force_two_level(1)
    try:
        ds, ions, ppm, kw = make_case("large_blobs")
        imgs, df = oracle_run(ds, ions, ppm, **kw)
        peaks, m, lo, hi = _device_run(ds, ions, ppm, **kw)
    finally:
        L.smg_debug_force_two_level(0)
    has = (m["flags"] & 1) != 0
    assert ((m["flags"][has] & 0x10) != 0).sum() >= 8
    assert ((m["flags"][has] & (0x10 | 8)) == (0x10 | 8)).any()   # two-level big-ion pass
    n0 = hi[ions.win_off[:-1]] - lo[ions.win_off[:-1]]
    assert (has & (n0 > 1706) & (n0 <= 2560)).any()              # olist rebuilt from the two-level set
    idx = {k: i for i, k in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))}
    rows = np.array([idx[k] for k in df.index.tolist()], dtype=np.int64)
    for col in ("chaos", "spatial", "spectral", "msm"):
        assert np.abs(df[col].to_numpy() - m[col][rows]).max(initial=0.0) <= METRIC_ATOL, col


# cases the sparse main pass (ion_sparse_kernel) scores: packed f32 hits, no hot-spot clip, <= 2^18 pixels
SPARSE_CASES = ["basic", "zeros_rect", "dups", "row", "column", "row_border1", "conn8_border1", "nlevels", "nlevels1",
                "boundary", "long_tail", "kmix", "wide_range", "nlevels100", "bands"]


@pytest.mark.parametrize("name", SPARSE_CASES)
def test_sparse_main_pass_scores_the_lds_ions(name):
    """The default main pass is the sparse one: every ion the main pass scored carries SMG_ION_SPARSE (and ion_pipe
    flags never appear together with it)."""
    m = _run_case(name)[7]
    has = (m["flags"] & 1) != 0
    main = has & ((m["flags"] & (2 | 8)) == 0)
    assert main.any() or name == "boundary"
    assert ((m["flags"][main] & 0x40) != 0).all(), name
    assert not (((m["flags"] & 0x40) != 0) & ((m["flags"] & (2 | 8 | 0x10)) != 0)).any()


def test_bands_case_reaches_the_hash_kruskal_and_two_bands():
    """bands: 1000-column image (two chaos bands) whose planted ions have > 64 chaos candidates on the sparse pass."""
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case("bands")
    sparse = ((m["flags"] & 0x41) == 0x41)
    assert sparse.sum() >= 8
    assert (df.chaos > 0).sum() >= 4  # real structure, not only isolated noise
    # the image is screened in more than one band: above 2^16 pixels the screen reads band bitmaps of
    # SpGeo.band_rows rows (smg_sparse.hip sparse_geo: the bitmap space below the survivor lists, 19,136 B, less
    # two buckets of 2^bs pixels and 128 bits, over ncols, minus 6)
    nrows, ncols = peaks.nrows, peaks.ncols
    npx = nrows * ncols
    assert npx > 1 << 16  # (images up to 2^16 pixels screen from the filter itself)
    bs = max((npx - 1).bit_length() - 10, 0)
    band_rows = (19136 * 8 - 2 * (1 << bs) - 128) // ncols - 6
    assert 8 <= band_rows < nrows, (band_rows, nrows)
    # ... and some sparse-pass ion has more than 64 chaos candidates (the block's hash Kruskal, not wave 0's): a
    # candidate is a pixel of erode_box(dilate_cross(principal presence)) (eL >= 1), border 0
    from scipy import ndimage
    from oracle.msm_oracle import BOX, CROSS
    hits = peaks.hits_sorted.cpu().numpy().view(np.uint64)
    pix = (hits & np.uint64(0x7FFFFFFF)).astype(np.int64)
    most = 0
    for i in np.nonzero(sparse)[0]:
        w = ions.win_off[i]
        pres = np.zeros(npx, bool)
        pres[pix[lo[w]:hi[w]]] = True
        bw = ndimage.binary_dilation(pres.reshape(nrows, ncols), structure=CROSS, border_value=0)
        bw = ndimage.binary_erosion(bw, structure=BOX, border_value=0)
        most = max(most, int(bw.sum()))
    assert most > 64, most


@pytest.mark.parametrize("name", SPARSE_CASES)
def test_legacy_main_pass_matches_oracle(name):
    """ion_pipe_kernel<512> (smg_debug_main_kernel(0)) stays correct: every sparse-pass case again through it."""
    from sm_distributed_amd import _lib
    ds, ions, ppm, kw, imgs, df, _, _, _, _ = _run_case(name)
    L = _lib.lib()
    L.smg_debug_main_kernel(0)
    try:
        _, m, _, _ = _device_run(ds, ions, ppm, **kw)
    finally:
        L.smg_debug_main_kernel(1)
    has = (m["flags"] & 1) != 0
    assert not ((m["flags"] & 0x40) != 0).any()
    idx = {k: i for i, k in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))}
    assert set(zip(ions.sf_ids[has].tolist(), ions.adducts[has].tolist())) == set(df.index.tolist())
    rows = np.array([idx[k] for k in df.index.tolist()], dtype=np.int64)
    for col in ("chaos", "spatial", "spectral", "msm"):
        err = np.abs(df[col].to_numpy() - m[col][rows])
        assert err.max(initial=0.0) <= METRIC_ATOL, (col, float(err.max()), int(np.argmax(err)))


# every LDS-path case again with the two-level pixel set forced (smg_debug_force_two_level)
TWO_LEVEL_CASES = ["basic", "zeros_rect", "dups", "row", "column", "row_border1", "conn8_border1", "nlevels",
                   "big_window", "boundary", "long_tail", "dups_heavy", "kmix", "clip99", "clip_q50_conn8",
                   "clip_dups_heavy", "clip_ties"]


@pytest.mark.parametrize("name", TWO_LEVEL_CASES)
def test_forced_two_level_matches_oracle(name):
    from sm_distributed_amd import _lib
    ds, ions, ppm, kw, imgs, df, _, _, _, _ = _run_case(name)
    L = _lib.lib()
    L.smg_debug_force_two_level(1)
    try:
        _, m, _, _ = _device_run(ds, ions, ppm, **kw)
    finally:
        L.smg_debug_force_two_level(0)
    has = (m["flags"] & 1) != 0
    lds = has & ((m["flags"] & 2) == 0)
    assert ((m["flags"][lds] & 0x10) != 0).all()
    assert lds.any() or name in ("dups_heavy", "clip_dups_heavy")  # duplicate lists / tables overflow the LDS passes
    idx = {k: i for i, k in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))}
    assert set(zip(ions.sf_ids[has].tolist(), ions.adducts[has].tolist())) == set(df.index.tolist())
    rows = np.array([idx[k] for k in df.index.tolist()], dtype=np.int64)
    for col in ("chaos", "spatial", "spectral", "msm"):
        err = np.abs(df[col].to_numpy() - m[col][rows])
        assert err.max(initial=0.0) <= METRIC_ATOL, (col, float(err.max()), int(np.argmax(err)))


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mode,impl", [(1, 1), (1, 0), (2, 1)])
def test_forced_dense_matches_oracle(name, mode, impl):
    """Every case again with every ion on the dense path (smg_debug_force_dense): mode 1 = the rank-indexed wide
    pass where the image fits it (with the clip too; its rejects on the pixel-indexed kernel) -- impl 1 its join
    variant (ion_wide_join_kernel, packed hits without the clip; the default), impl 0 ion_wide_kernel everywhere
    (smg_debug_wide_impl) --, mode 2 = the pixel-indexed kernel alone (sparse scatter into the slot's pixel-sized
    images, owner lists, candidate-only chaos)."""
    from sm_distributed_amd import _lib
    ds, ions, ppm, kw, imgs, df, _, _, _, _ = _run_case(name)
    L = _lib.lib()
    L.smg_debug_force_dense(mode)
    L.smg_debug_wide_impl(impl)
    try:
        _, m, _, _ = _device_run(ds, ions, ppm, **kw)
        _, m2, _, _ = _device_run(ds, ions, ppm, **kw)  # a second launch: slots start clean every launch
    finally:
        L.smg_debug_force_dense(0)
        L.smg_debug_wide_impl(1)
    has = (m["flags"] & 1) != 0
    assert ((m["flags"][has] & 2) != 0).all()
    wide = (m["flags"] & 0x20) != 0
    if mode == 2 or name == "xl_image":
        assert not wide.any()
    elif kw.get("do_preprocessing"):  # the wide pass clips; a table overflow would send an ion to the pixel kernel
        assert has.any() and wide[has].sum() >= 0.9 * has.sum()
    elif name == "wide_overflow":  # every ion's tail duplicates overflow the wide pass's table
        assert has.any() and not wide[has].any()
    else:
        assert wide[has].all()
    idx = {k: i for i, k in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))}
    assert set(zip(ions.sf_ids[has].tolist(), ions.adducts[has].tolist())) == set(df.index.tolist())
    rows = np.array([idx[k] for k in df.index.tolist()], dtype=np.int64)
    for col in ("chaos", "spatial", "spectral", "msm"):
        err = np.abs(df[col].to_numpy() - m[col][rows])
        assert err.max(initial=0.0) <= METRIC_ATOL, (col, float(err.max()), int(np.argmax(err)))
        assert np.abs(m2[col][rows] - m[col][rows]).max(initial=0.0) <= 1e-9


def test_sort_is_a_permutation():
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case("basic")
    # the duplicate-candidate flag (bit 31) is set by the sort's first pass: compare the hits without it
    a = np.sort(peaks.hits.cpu().numpy() & ~np.int64(0x80000000))
    b = np.sort(peaks.hits_sorted.cpu().numpy() & ~np.int64(0x80000000))
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("name", ["dups", "basic"])
def test_duplicate_flags_cover_every_window_duplicate(name):
    """Every pair of points sharing a pixel inside one window carries the duplicate-candidate flag."""
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case(name)
    hits = peaks.hits_sorted.cpu().numpy().view(np.uint64)
    pix = (hits & np.uint64(0x7FFFFFFF)).astype(np.int64)
    flag = ((hits >> np.uint64(31)) & np.uint64(1)).astype(bool)
    n_dup = 0
    for w in range(len(lo)):
        p = pix[lo[w]:hi[w]]
        if p.size < 2:
            continue
        _, inv, cnt = np.unique(p, return_inverse=True, return_counts=True)
        d = cnt[inv] > 1
        n_dup += int(d.sum())
        assert flag[lo[w]:hi[w]][d].all()
    assert n_dup > 0 or name == "basic"
    if name == "basic":
        assert flag.mean() < 0.2  # flags stay a small minority on ordinary data


def test_wide_pass_reached_without_forcing():
    """Windows beyond the big-ion pass go to the rank-indexed wide pass; its table overflow to the pixel kernel."""
    _, _, _, _, _, _, _, m, _, _ = _run_case("huge_window")
    dense = ((m["flags"] & 1) != 0) & ((m["flags"] & 2) != 0)
    assert dense.any() and ((m["flags"][dense] & 0x20) != 0).all()
    _, _, _, _, _, _, _, m, _, _ = _run_case("wide_overflow")
    has = (m["flags"] & 1) != 0
    assert has.any() and ((m["flags"][has] & 2) != 0).all() and not ((m["flags"][has] & 0x20) != 0).any()


def test_clip_runs_on_the_fast_paths():
    """The hot-spot clip (do_preprocessing) runs where the unclipped search would: the LDS passes (CLIP
    instantiations: each image clipped before its sums) on images up to 2^18 pixels, the rank-indexed wide pass on
    larger ones -- not only on the pixel-indexed kernel.  (clip_dups_heavy's flagged tail pixels overflow the LDS
    passes' duplicate table: those ions go on to the dense path, which the parity tests check.)"""
    for name in ("clip99", "clip_q50_conn8"):
        m = _run_case(name)[7]
        has = (m["flags"] & 1) != 0
        lds = has & ((m["flags"] & 2) == 0)
        assert has.any() and lds.sum() >= 0.5 * has.sum(), name
    m = _run_case("clip_large")[7]
    has = (m["flags"] & 1) != 0
    assert has.any() and ((m["flags"][has] & (0x20 | 2)) == (0x20 | 2)).all()


def test_lds_pipeline_paths_exercised():
    """The new cases reach the code they are meant for: multi-chunk tails on the main pass, duplicate-list
    overflow handed to the big-ion / dense passes, K = 1 and K > 8 ions."""
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case("long_tail")
    has = (m["flags"] & 1) != 0
    main = has & ((m["flags"] & (2 | 8)) == 0)
    tail = np.array([hi[ions.win_off[i] + 1:ions.win_off[i + 1]].sum() - lo[ions.win_off[i] + 1:ions.win_off[i + 1]].sum()
                     for i in range(ions.n_ions)])
    # > 4 register chunks (ion_sparse_kernel: 256 threads x 2 points; ion_pipe_kernel<512>: 512 x 2)
    sparse = (m["flags"] & 0x40) != 0
    assert (main & np.where(sparse, tail > 4 * 512, tail > 4 * 1024)).sum() >= 10
    _, _, _, _, _, _, _, m, _, _ = _run_case("dups_heavy")
    assert ((m["flags"] & (2 | 8)) != 0).any()
    ds, ions, ppm, kw, imgs, df, peaks, m, lo, hi = _run_case("kmix")
    K = np.diff(ions.win_off)
    has = (m["flags"] & 1) != 0
    assert (has & (K == 1)).any() and (has & (K > 8)).any()
    assert ((m["flags"][has & (K > 8)] & 2) != 0).all()


# ---- edge inputs: empty dataset, empty ion list, a 1x1 image, every point of a window on one pixel ----------
def _edge_case(name):
    from sm_distributed_amd import synthetic as syn
    from tests.parity_cases import subset_ions
    ions = syn.make_ion_table(6, seed=141, decoy_seed=142)
    if name == "no_points":
        ds = syn.make_dataset_np(4, 5, 0.0, seed=143)
        return ds, ions, 20.0
    if name == "no_ions":
        return syn.make_dataset_np(8, 8, 50, seed=144), subset_ions(ions, np.zeros(0, np.int64)), 20.0
    if name == "one_pixel":
        return syn.make_dataset_np(1, 1, 4000, seed=145, ions=ions, plant_fraction=1.0, plant_seed=146), ions, 30.0
    if name == "one_hot_pixel":  # a 6x6 image whose points all sit in spectrum 7 (heavy same-pixel duplicates)
        ds = syn.make_dataset_np(6, 6, 0.0, seed=147)
        rng = np.random.default_rng(148)
        mz = np.sort(np.concatenate([ions.peak_mz * (1 + rng.normal(0, 2e-6, ions.peak_mz.size)) for _ in range(8)])
                     ).astype(np.float32)
        off = np.zeros(37, np.int64)
        off[8:] = mz.size
        ints = rng.lognormal(6.0, 1.0, mz.size).astype(np.float32)
        return syn.SpectraSet(sp_off=off, mz=mz, ints=ints, coords=ds.coords), ions, 20.0
    raise KeyError(name)


@pytest.mark.parametrize("name", ["no_points", "no_ions", "one_pixel", "one_hot_pixel"])
@pytest.mark.parametrize("dense", [False, True])
def test_edge_inputs_match_oracle(name, dense):
    from sm_distributed_amd import _lib
    ds, ions, ppm = _edge_case(name)
    _, df = oracle_run(ds, ions, ppm)
    L = _lib.lib()
    L.smg_debug_force_dense(1 if dense else 0)
    try:
        _, m, lo, hi = _device_run(ds, ions, ppm)
    finally:
        L.smg_debug_force_dense(0)
    has = (m["flags"] & 1) != 0 if ions.n_ions else np.zeros(0, bool)
    assert set(zip(ions.sf_ids[has].tolist(), ions.adducts[has].tolist())) == set(df.index.tolist())
    if len(df):
        idx = {k: i for i, k in enumerate(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))}
        rows = np.array([idx[k] for k in df.index.tolist()], dtype=np.int64)
        for col in ("chaos", "spatial", "spectral", "msm"):
            err = np.abs(df[col].to_numpy() - m[col][rows])
            assert err.max(initial=0.0) <= METRIC_ATOL, (col, float(err.max()))
    if name == "one_hot_pixel":
        assert len(df) > 0
