"""The hand-written m/z sort (csrc/smg_sort.hip) and its fused duplicate-candidate flags (GPU only).

The reference sorts each segment's peaks by m/z (formula_imager_segm.py:73-74); only the set of points per
window matters downstream, but the sort here is stable, so its output is one exact array:
* smg_sort_points == the points permuted by a stable argsort of the m/z values (torch.sort(stable=True)), at
  sizes around the 8192-point tile, with heavy ties, over 1 to 4 radix passes and with 64-bit tile offsets
  (more than 2^30 points);
* the same arrays as rocPRIM's onesweep sort (smg_debug_sort_impl(0)) on a synthetic dataset, and as the
  hand-written sort's round-3 form, whose tiles find their offsets by decoupled look-back in ticket order
  (smg_debug_sort_impl(2)) instead of the reduce-then-scan offsets;
* smg_sort_points_flag == smg_flag_duplicates followed by smg_sort_points, bit for bit, on synthetic datasets and
  on the parity cases; datasets it does not cover (a spectrum not m/z-sorted, a shared pixel) take the two calls.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _peaks(mz, hits, sp_off=None, dims=(1, 1)):
    from sm_distributed_amd import engine as E
    return E.DevicePeaks(mz=mz, hits=hits, nrows=int(dims[0]), ncols=int(dims[1]), sp_off=sp_off)


def _expect(mz, hits):
    import torch
    order = torch.sort(mz, stable=True).indices
    return mz[order], hits[order]


def _random_points(n, seed, ties=False, lo=100.0, hi=1000.0):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    mz = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) * (hi - lo) + lo
    if ties:  # a few hundred distinct values: long runs of equal keys, stability visible
        mz = torch.round(mz * 0.3) / 0.3
    mz = mz.to(torch.float32)
    hits = torch.randint(0, 1 << 62, (n,), generator=g, device="cuda", dtype=torch.int64)
    return mz, hits


@pytest.mark.parametrize("n", [1, 2, 63, 8191, 8192, 8193, 100_003, 3_000_000])
@pytest.mark.parametrize("ties", [False, True])
def test_sort_matches_stable_argsort(n, ties):
    import torch
    mz, hits = _random_points(n, seed=n + int(ties), ties=ties)
    p = _peaks(mz, hits).sort()
    torch.cuda.synchronize()
    ek, ev = _expect(mz, hits)
    assert torch.equal(p.mz_sorted, ek)
    assert torch.equal(p.hits_sorted, ev)


@pytest.mark.parametrize("lo,hi,bits", [(100.0, 100.9, None), (1.0e-3, 1.0e6, None), (100.0, 1000.0, 31)])
def test_sort_any_number_of_passes(lo, hi, bits):
    """key_bits from 20 (3 passes of <= 9 bits... down to 1-2 passes for a narrow range) up to 31 (4 x 8)."""
    import torch
    mz, hits = _random_points(200_000, seed=7, lo=lo, hi=hi)
    p = _peaks(mz, hits)
    if bits is not None:
        p.sort_key_bits = bits
    p.sort()
    torch.cuda.synchronize()
    ek, ev = _expect(mz, hits)
    assert torch.equal(p.mz_sorted, ek) and torch.equal(p.hits_sorted, ev)


def test_sort_more_than_2p30_points_wide_lookback():
    """n >= 2^30 takes 64-bit tile offsets (reduce-then-scan counts and chunk totals)."""
    import torch
    n = (1 << 30) + 12345
    mz, hits = _random_points(n, seed=11, ties=True)
    try:
        p = _peaks(mz, hits).sort()
        torch.cuda.synchronize()
        ek, ev = _expect(mz, hits)
        assert torch.equal(p.mz_sorted, ek)
        assert torch.equal(p.hits_sorted, ev)
    finally:
        from sm_distributed_amd import engine as E
        for k in list(E._ws_cache):
            E._ws_cache.pop(k)
        p = mz = hits = ek = ev = None
        torch.cuda.empty_cache()


def _synthetic(nrows, ncols, lam, seed):
    from sm_distributed_amd import engine as E
    from sm_distributed_amd import synthetic as syn
    ions = syn.make_ion_table(200, seed=seed + 1, decoy_seed=seed + 2)
    mz, hits, dims, info = syn.make_dataset_torch(nrows, ncols, lam, seed=seed, device="cuda", ions=ions)
    return E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])


def test_native_sort_identical_to_rocprim():
    import torch
    from sm_distributed_amd._lib import lib
    p = _synthetic(200, 200, 800.0, seed=5)
    p.flag_duplicates(2.0)
    p.sort()
    a = (p.mz_sorted.clone(), p.hits_sorted.clone())
    try:
        assert lib().smg_debug_sort_impl(0) == 0
        p.sort()
        torch.cuda.synchronize()
    finally:
        lib().smg_debug_sort_impl(1)
    assert torch.equal(a[0], p.mz_sorted) and torch.equal(a[1], p.hits_sorted)


@pytest.mark.parametrize("n", [8193, 1_000_003])
def test_reduce_then_scan_identical_to_lookback(n):
    import torch
    from sm_distributed_amd._lib import lib
    mz, hits = _random_points(n, seed=n, ties=True)
    p = _peaks(mz, hits).sort()
    torch.cuda.synchronize()
    a = (p.mz_sorted.clone(), p.hits_sorted.clone())
    try:
        assert lib().smg_debug_sort_impl(2) == 0
        p.sort()
        torch.cuda.synchronize()
    finally:
        lib().smg_debug_sort_impl(1)
    assert torch.equal(a[0], p.mz_sorted) and torch.equal(a[1], p.hits_sorted)


@pytest.mark.parametrize("ppm", [2.0, 50.0])
def test_fused_flags_identical_to_flag_pass(ppm):
    import torch
    p = _synthetic(150, 170, 1500.0, seed=9)
    assert p.force is None and p.spectra_sorted()
    p.flag_and_sort(ppm)
    torch.cuda.synchronize()
    fused = p.hits_sorted.clone()
    p.flag_duplicates(ppm)
    p.sort()
    torch.cuda.synchronize()
    assert torch.equal(fused, p.hits_sorted)
    flagged = int(((fused >> 31) & 1).sum().item())
    assert 0 < flagged < fused.numel()  # the case has both kinds of points


@pytest.mark.parametrize("name", ["basic", "dups", "boundary", "conn8_border1", "large_image"])
def test_fused_flags_on_parity_cases(name):
    """The parity datasets through DevicePeaks.from_arrays (the drop-in path): flag_and_sort == the two calls,
    whichever way the dataset routes it (shared pixels / unsorted spectra take the separate flag pass)."""
    import torch
    from sm_distributed_amd import engine as E
    from tests.parity_cases import make_case
    ds, ions, ppm, kw = make_case(name)
    pm, dims = ds.pixel_map_dims()
    p = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    p.flag_and_sort(ppm)
    torch.cuda.synchronize()
    fused = p.hits_sorted.clone()
    q = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    q.flag_duplicates(ppm)
    q.sort()
    torch.cuda.synchronize()
    assert torch.equal(fused, q.hits_sorted)
    assert torch.equal(p.mz_sorted, q.mz_sorted)


def test_unsorted_spectrum_takes_flag_pass():
    """A spectrum that is not m/z-sorted flags all its points (smg_flag_duplicates): flag_and_sort must route such
    a dataset through the flag pass."""
    import torch
    from sm_distributed_amd import engine as E
    rng = np.random.default_rng(3)
    sp_off = np.array([0, 50, 120, 200], dtype=np.int64)
    mz = np.sort(rng.uniform(100, 200, 200)).astype(np.float32)
    mz[50:120] = mz[50:120][::-1].copy()  # spectrum 1 in descending order
    ints = rng.uniform(1, 10, 200).astype(np.float32)
    p = E.DevicePeaks.from_arrays(sp_off, mz, ints, np.arange(3, dtype=np.int32), (1, 3))
    assert not p.spectra_sorted()
    p.flag_and_sort(2.0)
    torch.cuda.synchronize()
    h = p.hits_sorted.cpu().numpy()
    pix = h & 0x7FFFFFFF
    assert ((h[pix == 1] >> 31) & 1).all()


@pytest.mark.parametrize("sizes", ["ragged", "long"])
def test_fused_flags_ragged_spectra(sizes):
    """Spectrum starts marked per tile from sp_off: empty spectra, one-point spectra, many spectra per 8192-point
    tile, and spectra longer than a tile; flags identical to the flag pass."""
    import torch
    from sm_distributed_amd import engine as E
    rng = np.random.default_rng(17)
    if sizes == "ragged":
        cnt = rng.choice([0, 0, 1, 2, 3, 7, 40, 300], size=60_000)
    else:
        cnt = rng.integers(5_000, 30_000, size=40)
    sp_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    n = int(sp_off[-1])
    mz = rng.uniform(100.0, 100.4 if sizes == "ragged" else 1000.0, n)  # both flagged and unflagged points
    for s in range(len(cnt)):
        mz[sp_off[s]:sp_off[s + 1]].sort()
    ints = rng.uniform(1, 10, n).astype(np.float32)
    pm = np.arange(len(cnt), dtype=np.int32)
    dims = (1, len(cnt))
    p = E.DevicePeaks.from_arrays(sp_off, mz.astype(np.float32), ints, pm, dims)
    assert p.force is None and p.spectra_sorted()
    p.flag_and_sort(50.0)
    torch.cuda.synchronize()
    fused = p.hits_sorted.clone()
    p.flag_duplicates(50.0)
    p.sort()
    torch.cuda.synchronize()
    assert torch.equal(fused, p.hits_sorted)
    flagged = int(((fused >> 31) & 1).sum().item())
    assert 0 < flagged < n


@pytest.mark.parametrize("n", [1, 63, 64, 65, 131072 * 3 + 77, 5_000_000])
def test_prefix_sums_match_exact_sums(n):
    """smg_hit_prefix_sums (chunked double-double scan): every block prefix (sum v, sum v^2 of unflagged points)
    equals the exactly rounded sum over the points before it (math.fsum) to ~1e-15 relative, whatever the
    chunk boundaries and a dynamic range of 1e-3..1e9."""
    import math

    import torch
    from sm_distributed_amd import _lib
    from sm_distributed_amd import engine as E
    rng = np.random.default_rng(n)
    v = (10.0 ** rng.uniform(-3, 9, n)).astype(np.float32)
    flag = rng.random(n) < 0.1
    hits = (v.view(np.uint32).astype(np.uint64) << np.uint64(32)) | (flag.astype(np.uint64) << np.uint64(31))
    d_hits = torch.from_numpy(hits.view(np.int64)).cuda()
    cum = E.hit_prefix_sums(_lib.SMG_HITS_PACKED_F32, d_hits, None, n).cpu().numpy()
    nb = (n + 63) // 64
    assert cum.shape == (nb + 1, 4)
    vd = v.astype(np.float64)
    check = sorted({0, 1, nb // 2, nb - 1, nb} | {b for b in (2048, 2049, 4096) if b <= nb})
    for b in check:
        x = math.fsum(vd[:64 * b])
        y = math.fsum((vd[:64 * b] ** 2)[~flag[:64 * b]])
        gx, gy = cum[b, 0] + cum[b, 1], cum[b, 2] + cum[b, 3]
        assert abs(gx - x) <= 1e-14 * max(abs(x), 1e-300), (b, gx, x)
        assert abs(gy - y) <= 1e-14 * max(abs(y), 1e-300), (b, gy, y)


def test_flag_ppm_tracks_the_sorted_copy():
    """The fused flag + sort flags only the sorted copy: a later plain sort() of the (unflagged) dataset-order hits
    must not claim that ppm's flags (flag_ppm None), so an image set made at that ppm re-flags before use; a flag
    pass then sort() carries the ppm again (engine.py flag_and_sort)."""
    import torch
    from sm_distributed_amd import synthetic as syn
    from sm_distributed_amd import engine as E
    mz, hits, dims, info = syn.make_dataset_torch(16, 16, 200.0, seed=3, device="cuda")
    p = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    p.flag_and_sort(5.0)
    assert p.flag_ppm == 5.0 and p.hits_flag_ppm is None
    fused = p.hits_sorted.clone()
    p.sort()
    assert p.flag_ppm is None
    p.flag_duplicates(5.0)
    assert p.hits_flag_ppm == 5.0
    p.sort()
    assert p.flag_ppm == 5.0
    torch.cuda.synchronize()
    assert torch.equal(p.hits_sorted, fused)  # the two ways give the same flags
