"""The multi-GPU path's device pieces on one GPU (GPU only): the m/z slice of the resident peaks
(smg_slice_mz_count / _copy, flags fused into the copy) and the per-rank scorer of distributed.score_sharded.
The world-size > 1 collectives run in tests/test_distributed_gloo.py (CPU ranks); here every rank's shard is
scored in turn on the one GPU and the union must equal the single-GPU table, and a world-size-1 RCCL group
runs score_sharded end to end."""
import socket

import numpy as np
import pandas as pd
import pytest

from tests.parity_cases import make_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["dups", "basic", "zeros_rect"])
def test_slice_equals_masked_flagged_points(name):
    import torch
    from sm_distributed_amd import engine as E
    ds, ions, ppm, kw = make_case(name)
    pm, dims = ds.pixel_map_dims()
    full = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    full.flag_duplicates(ppm)
    mz = full.mz.cpu().numpy()
    hits = full.hits.cpu().numpy()
    sp = np.repeat(np.arange(ds.n_spectra), np.diff(ds.sp_off))
    rng = np.random.default_rng(5)
    for lo, hi in [(mz.min(), mz.max()), (300.0, 301.5), tuple(np.sort(rng.uniform(100, 1000, 2))), (2000.0, 3000.0)]:
        sl = full.slice_mz(float(lo), float(hi), ppm)
        sel = (mz.astype(np.float64) >= lo) & (mz.astype(np.float64) <= hi)
        np.testing.assert_array_equal(sl.mz.cpu().numpy(), mz[sel])
        np.testing.assert_array_equal(sl.hits.cpu().numpy(), hits[sel])  # same duplicate flags as the full pass
        off = sl.sp_off.cpu().numpy()
        np.testing.assert_array_equal(np.diff(off), np.bincount(sp[sel], minlength=ds.n_spectra))
        assert sl.flag_duplicates(ppm).flags_preset_ppm == ppm  # no second flag pass
    torch.cuda.synchronize()


def _api_table(peaks, formulas, ppm):
    from sm_distributed_amd.dataset import ResidentDataset
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    from sm_distributed_amd.formula_img_validator import sf_image_metrics
    dds = ResidentDataset(peaks)
    conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    ims = compute_sf_images(None, dds, formulas.get_sf_peak_df(), ppm)
    return sf_image_metrics(ims, None, formulas, dds, conf)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_every_rank_shard_on_one_gpu_equals_single_gpu_table(world):
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    from sm_distributed_amd.formulas import FormulasSegm
    from tests.parity_cases import oracle_run
    ds, ions, ppm, kw = make_case("dups")
    pm, dims = ds.pixel_map_dims()
    peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    formulas = FormulasSegm.from_ion_table(ions, ppm)
    conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    rows = []
    for r in range(world):
        plan = D.plan_shards(formulas, peaks, ppm, world, r)
        rr, _ = D._device_rows(plan, peaks, conf)
        rows.append(rr.cpu())
    import torch
    df = D.rows_to_frame(torch.cat(rows), D.plan_shards(formulas, peaks, ppm, world, 0).global_keys)
    ref = _api_table(peaks, formulas, ppm)
    assert list(df.index) == list(ref.index)
    for c in ("chaos", "spatial", "spectral", "msm"):
        np.testing.assert_allclose(df[c].values, ref[c].values, rtol=0, atol=1e-12)
    _, exp = oracle_run(ds, ions, ppm)
    exp = exp.sort_index()
    assert list(df.index) == list(exp.index)
    for c in ("chaos", "spatial", "spectral", "msm"):
        assert np.abs(df[c].values - exp[c].values).max() <= 1e-5


def test_assembly_cache_follows_the_gathered_rows():
    """rows_to_frame's steady-state path (distributed.py: the row placement of the previous table, checked on the
    device and copied back with the columns) gives the single-GPU table for a repeated table, for the same rows
    in another block order (same shape, other placement: the check must reject the cached one) and back."""
    import torch
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    from sm_distributed_amd.formulas import FormulasSegm
    ds, ions, ppm, kw = make_case("dups")
    pm, dims = ds.pixel_map_dims()
    peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    formulas = FormulasSegm.from_ion_table(ions, ppm)
    conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    world = 3
    rows = [D._device_rows(D.plan_shards(formulas, peaks, ppm, world, r), peaks, conf)[0] for r in range(world)]
    gk = D.plan_shards(formulas, peaks, ppm, world, 0).global_keys
    ref = _api_table(peaks, formulas, ppm)
    a = torch.cat(rows)
    b = torch.cat(rows[::-1])
    assert a.is_cuda and not torch.equal(a[:, 0], b[:, 0])
    for t in (a, a, b, b, a):
        df = D.rows_to_frame(t, gk)
        assert list(df.index) == list(ref.index)
        for c in ("chaos", "spatial", "spectral", "msm"):
            np.testing.assert_allclose(df[c].values, ref[c].values, rtol=0, atol=1e-12)


def test_score_sharded_world1_rccl():
    import torch.distributed as dist
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    from sm_distributed_amd.formulas import FormulasSegm
    ds, ions, ppm, kw = make_case("basic")
    pm, dims = ds.pixel_map_dims()
    peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    formulas = FormulasSegm.from_ion_table(ions, ppm)
    conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        plan = D.plan_shards(formulas, peaks, ppm, 1, 0)
        df, ims = D.score_sharded(plan, peaks, conf)
        ref = _api_table(peaks, formulas, ppm)
        pd.testing.assert_frame_equal(df, ref, check_exact=False, rtol=0, atol=1e-12)
        assert sorted(k for k, _ in ims.collect()) == sorted(ref.index.tolist())
    finally:
        dist.destroy_process_group()


def test_shards_with_an_unsorted_spectrum_equal_single_gpu_table():
    """A dataset with spectra that are not m/z-sorted (accepted by the reference; every point of such a spectrum is
    a duplicate candidate): the rank slices take the masked-copy path and the shards still give the single-GPU
    table (slice_mz used to raise)."""
    import torch
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    from sm_distributed_amd.formulas import FormulasSegm
    ds, ions, ppm, kw = make_case("dups")
    mz = ds.mz.copy()
    for s in (3, 17, 40):  # reverse three spectra
        a, b = ds.sp_off[s], ds.sp_off[s + 1]
        mz[a:b] = mz[a:b][::-1].copy()
        ds.ints[a:b] = ds.ints[a:b][::-1].copy()
    ds.mz = mz
    pm, dims = ds.pixel_map_dims()
    peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims)
    assert not peaks.spectra_sorted()
    formulas = FormulasSegm.from_ion_table(ions, ppm)
    conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
    rows = []
    for r in range(3):
        plan = D.plan_shards(formulas, peaks, ppm, 3, r)
        rr, _ = D._device_rows(plan, peaks, conf)
        rows.append(rr.cpu())
    df = D.rows_to_frame(torch.cat(rows), D.plan_shards(formulas, peaks, ppm, 3, 0).global_keys)
    ref = _api_table(peaks, formulas, ppm)
    assert list(df.index) == list(ref.index)
    for c in ("chaos", "spatial", "spectral", "msm"):
        np.testing.assert_allclose(df[c].values, ref[c].values, rtol=0, atol=1e-12)


def _nccl_rank(rank, world, port, out_q):
    import os
    import torch
    import torch.distributed as dist
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    from sm_distributed_amd.formulas import FormulasSegm
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            device_id=dev)
    try:
        ds, ions, ppm, kw = make_case("basic")
        pm, dims = ds.pixel_map_dims()
        peaks = E.DevicePeaks.from_arrays(ds.sp_off, ds.mz, ds.ints, pm, dims, device=dev)
        formulas = FormulasSegm.from_ion_table(ions, ppm)
        conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
        plan = D.plan_shards(formulas, peaks, ppm, world, rank)
        df, _ = D.score_sharded(plan, peaks, conf)
        if rank == 0:
            ref = _api_table(peaks, formulas, ppm)
            same = df.index.equals(ref.index) and np.allclose(df.to_numpy(), ref.to_numpy(), rtol=0, atol=1e-12)
            out_q.put(("ok" if same else "mismatch", os.getpid()))
    except Exception as e:  # pragma: no cover - reported to the parent
        out_q.put(("error %r" % (e,), rank))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_score_sharded_world2_rccl():
    """score_sharded over a world-size-2 RCCL group, one process per GPU (skipped on a one-GPU box): the
    gathered table equals the single-GPU table."""
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (the driver's multi-GPU node); gloo world-size 2/3 runs cover the collectives on CPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_nccl_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5)[0] == "ok"
