"""Maximum-size dataset on the device (GPU only): more than 2^32 resident points (config-5 scale, 1000x1000 px,
Poisson(4400) centroids ~= 4.4e9 points, ~160 GB of HBM at peak), so every point index on the path (sort,
window search, prefix sums, descriptors, dense slots) must be 64-bit clean.

The oracle cannot image 4.4e9 points, so parity is checked through size-independent properties plus a sample:
* the sort is a permutation: the wrapping int64 sums of the hit words (flag bit masked) and of the key bit patterns are equal
  before and after it (modular addition is order-independent), and the sorted keys never decrease, including
  across the 2^32 index boundary;
* a sample of ions (principal m/z in a narrow band) is imaged and scored by the oracle (oracle/cpu_baseline.py,
  i.e. formula_imager_segm.py:66-92 + formula_img_validator.py:72-84 on the band's m/z segment): window sizes
  identical, metrics within 1e-5 absolute.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

METRIC_ATOL = 1e-5


def _wrapsum(t, mask=None):
    import torch
    s = torch.zeros((), dtype=torch.int64, device=t.device)
    blk = 1 << 30
    for a in range(0, t.numel(), blk):
        x = t[a:a + blk].to(torch.int64)
        s += (x if mask is None else x & mask).sum()
    return int(s.item())


def test_more_than_2p32_points_sample_matches_oracle():
    import torch
    from oracle import cpu_baseline as CB
    from sm_distributed_amd import engine as E
    from sm_distributed_amd import synthetic as syn

    ppm, nlevels = 2.0, 30
    ions = syn.make_ion_table(300, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(1000, 1000, 4400.0, seed=42, device="cuda", ions=ions)
    n = info["n_points"]
    assert n > (1 << 32)
    try:
        peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
        dions = E.DeviceIons.from_arrays(ions.win_off, ions.peak_mz, ions.peak_int)
        m, lo, hi = E.run_hot_path(peaks, dions, ppm, nlevels)
        torch.cuda.synchronize()
        # the sort permutes (key, hit) pairs
        # (without the duplicate-candidate flag, which the sort's first pass sets)
        noflag = ~(1 << 31)
        assert _wrapsum(peaks.hits, noflag) == _wrapsum(peaks.hits_sorted, noflag)
        assert _wrapsum(peaks.mz.view(torch.int32)) == _wrapsum(peaks.mz_sorted.view(torch.int32))
        blk = 1 << 30
        for a in range(0, n - 1, blk):
            s = peaks.mz_sorted[a:min(n, a + blk + 1)]
            assert bool((s[1:] >= s[:-1]).all())
        lo_h, hi_h = lo.cpu().numpy(), hi.cpu().numpy()
        got = m.to_numpy()
        assert (hi_h <= n).all() and (lo_h <= hi_h).all()
        assert int(hi_h.max()) > (1 << 32)  # some windows lie beyond the 32-bit index range

        # sample: ions whose principal m/z lies in [700, 702)
        first = ions.peak_mz[ions.win_off[:-1]]
        pick = np.nonzero((first >= 700.0) & (first < 702.0))[0][:10]
        assert pick.size >= 4
        lo_b = min(ions.peak_mz[ions.win_off[i]] for i in pick) * (1 - 2 * ppm * 1e-6) - 1e-3
        hi_b = max(ions.peak_mz[ions.win_off[i + 1] - 1] for i in pick) * (1 + 2 * ppm * 1e-6) + 1e-3
        pm, ph = [], []
        for a in range(0, n, blk):  # the resident (unsorted) dataset, flag bits masked off below
            mm, hh = peaks.mz[a:a + blk], peaks.hits[a:a + blk]
            sel = (mm >= lo_b) & (mm <= hi_b)
            pm.append(mm[sel].cpu().numpy())
            ph.append(hh[sel].cpu().numpy())
    finally:
        for k in [k for k in E._ws_cache]:
            E._ws_cache.pop(k)
        del mz, hits
        peaks = dions = m = lo = hi = None
        torch.cuda.empty_cache()
    b_mz = np.concatenate(pm)
    b_hits = np.concatenate(ph).view(np.uint64)
    b_pix = (b_hits & np.uint64(0x7FFFFFFF)).astype(np.int64)
    b_int = (b_hits >> np.uint64(32)).astype(np.uint32).view(np.float32)
    CB._init(b_pix, b_mz, b_int, dims, ppm, nlevels)
    tasks = [(int(i), ions.peak_mz[ions.win_off[i]:ions.win_off[i + 1]].copy(),
              ions.peak_int[ions.win_off[i]:ions.win_off[i + 1]].copy()) for i in pick]
    rows, _ = CB._work(tasks)
    assert len(rows) == pick.size
    from oracle import msm_oracle as O
    seg = np.sort(b_mz).astype(np.float64)
    for ion_id, c, s, p in rows:
        a, b = ions.win_off[ion_id], ions.win_off[ion_id + 1]
        assert got["flags"][ion_id] & 1
        np.testing.assert_allclose(got["chaos"][ion_id], c, atol=METRIC_ATOL, rtol=0)
        np.testing.assert_allclose(got["spatial"][ion_id], s, atol=METRIC_ATOL, rtol=0)
        np.testing.assert_allclose(got["spectral"][ion_id], p, atol=METRIC_ATOL, rtol=0)
        # window sizes: the oracle's searchsorted over the segment
        lower, upper = O.window_bounds(ions.peak_mz[a:b], ppm)
        cnt = np.searchsorted(seg, upper, "right") - np.searchsorted(seg, lower, "left")
        np.testing.assert_array_equal(hi_h[a:b] - lo_h[a:b], cnt)
