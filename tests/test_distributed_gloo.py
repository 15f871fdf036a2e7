"""The multi-GPU product path on CPU ranks: world_size-2 (and 3) gloo process groups run
``distributed.plan_shards`` / ``score_sharded`` / ``search`` -- the same code the GPU ranks run over RCCL --
with the per-rank scorer replaced by the oracle (there is no device path on CPU).  The oracle scorer images
each rank's ions from the points of the rank's m/z slice only, so the test also proves the slice bounds hold
every window.  Rank 0 must rebuild exactly the single-process table, and ``search`` must give the
single-process annotations (msm_basic_search.py:13-31)."""
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    from sm_distributed_amd.formulas import FormulasSegm
    from tests.parity_cases import make_case
    ds, ions, ppm, kw = make_case("basic")
    return ds, ions, ppm, FormulasSegm.from_ion_table(ions, ppm)


def _oracle_scorer(ds):
    """score_local for CPU ranks: the oracle on the rank's m/z slice, rows in the device scorer's format."""
    from oracle import msm_oracle as O
    from tests.parity_cases import sf_peak_ints

    def score(plan, peaks, ds_config):
        pm, dims = ds.pixel_map_dims()
        sp = np.repeat(np.arange(ds.n_spectra), np.diff(ds.sp_off))
        m64 = ds.mz.astype(np.float64)
        sel = (m64 >= plan.mz_lo) & (m64 <= plan.mz_hi)  # the rank's slice (smg_slice_mz semantics)
        spectra = [(int(s), ds.mz[sel & (sp == s)], ds.ints[sel & (sp == s)].astype(np.float64))
                   for s in range(ds.n_spectra)]
        shard = plan.formulas
        imgs = O.compute_sf_images(spectra, pm, dims, shard.get_sf_peak_df(), plan.ppm)
        ints = shard.get_sf_peak_ints()
        rows = np.full((len(plan.ion_idx), 5), -1.0)
        keys = list(zip(shard.ion_sf.tolist(), np.asarray(shard.adducts, dtype=object)[shard.ion_adduct_code].tolist()))
        for i, key in enumerate(keys):
            if key in imgs:
                c, s, p = O.compute_img_metrics(imgs[key], ints[key], dims[0], dims[1],
                                                ds_config["image_generation"]["nlevels"])
                rows[i] = (plan.ion_idx[i], c, s, p, c * s * p)
        return torch.from_numpy(rows), None
    return score


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sm_distributed_amd import distributed as D
        from sm_distributed_amd.fdr import FDR
        ds, ions, ppm, formulas = _case()
        conf = {"image_generation": {"ppm": ppm, "nlevels": 30, "q": 99, "do_preprocessing": False}}
        plan = D.plan_shards(formulas, torch.from_numpy(ds.mz), ppm, world, rank)
        scorer = _oracle_scorer(ds)
        df, _ = D.score_sharded(plan, None, conf, score_local=scorer)
        fdr = FDR(0, 0, ions.decoy_sample_size, list(ions.target_adducts))
        sf, ta, da = ions.td
        fdr.td_df = pd.DataFrame({"sf_id": sf, "ta": ta, "da": da})
        res, _ = D.search(plan, None, formulas, fdr, conf, score_local=scorer)
        if rank == 0:
            pd.to_pickle({"table": df, "search": res, "counts": plan.counts}, out_path)
        else:
            assert df is None and res is None
    finally:
        dist.destroy_process_group()


def test_shard_bounds_balanced():
    from sm_distributed_amd import distributed as D
    costs = np.random.default_rng(0).uniform(1, 10, 1000)
    b = D.shard_bounds(costs, 8)
    assert b[0][0] == 0 and b[-1][1] == 1000
    assert all(b[i][1] == b[i + 1][0] for i in range(7))
    sums = [costs[x:y].sum() for x, y in b]
    assert max(sums) / min(sums) < 1.1


def test_shard_bounds_rank0_head():
    """shard_bounds with work of rank 0 besides its shard (head): rank 0's shard + head equals every other
    rank's shard."""
    from sm_distributed_amd import distributed as D
    costs = np.full(8000, 1.0)
    head = 500.0
    b = D.shard_bounds(costs, 8, head)
    sums = [costs[x:y].sum() for x, y in b]
    assert b[0][0] == 0 and b[-1][1] == 8000 and all(b[i][1] == b[i + 1][0] for i in range(7))
    loads = [sums[0] + head] + sums[1:]
    assert max(loads) - min(loads) <= 1.0, loads
    assert D.shard_bounds(costs, 8, 0.0) == D.shard_bounds(costs, 8)


def test_plan_shards_partitions_ions_and_slices_cover_windows():
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import synthetic as syn
    from sm_distributed_amd.formulas import FormulasSegm
    ions = syn.make_ion_table(2000, seed=5, decoy_seed=6)
    formulas = FormulasSegm.from_ion_table(ions)
    mz = torch.from_numpy(np.random.default_rng(1).uniform(100, 1000, 200000).astype(np.float32))
    for world in (2, 4, 8):
        plans = [D.plan_shards(formulas, mz, 2.0, world, r) for r in range(world)]
        allidx = np.concatenate([p.ion_idx for p in plans])
        assert np.array_equal(np.sort(allidx), np.arange(formulas.n_ions))
        for p in plans:
            pm = p.formulas.peak_mz
            assert (pm - pm * 2e-6 >= p.mz_lo).all() and (pm + pm * 2e-6 <= p.mz_hi).all()
        cost = plans[0].est_cost
        assert max(cost) / min(cost) < 1.05, cost
        # contiguous in principal m/z: slices overlap only by the isotope tails (< 6 Da)
        lo = sorted((p.mz_lo, p.mz_hi) for p in plans)
        assert all(lo[i + 1][0] > lo[i][0] for i in range(world - 1))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_search_matches_single_process(tmp_path, world):
    from oracle import msm_oracle as O
    from tests.parity_cases import oracle_run
    out = str(tmp_path / "rank0.pkl")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = pd.read_pickle(out)
    ds, ions, ppm, formulas = _case()
    _, exp = oracle_run(ds, ions, ppm)
    table = got["table"]
    assert list(table.index) == sorted(exp.index.tolist())  # (sf_id, adduct) order, as the single-GPU table
    exp = exp.sort_index()
    for c in ("chaos", "spatial", "spectral", "msm"):
        np.testing.assert_array_equal(table[c].values, exp[c].values)
    assert min(got["counts"]) > 0
    # search: FDR + filter on rank 0 == the single-process pipeline
    sf, ta, da = ions.td
    td = pd.DataFrame({"sf_id": sf, "ta": ta, "da": da})
    msm = formulas.get_sf_adduct_sorted_df().join(exp.msm).fillna(0)
    ofdr = O.estimate_fdr(msm, td, list(ions.target_adducts), ions.decoy_sample_size)
    e = exp.join(ofdr, how="inner")[["chaos", "spatial", "spectral", "msm", "fdr"]]
    e = e[(e.chaos > 0) | (e.spatial > 0) | (e.spectral > 0)].sort_index()
    r = got["search"].sort_index()
    assert list(r.index) == list(e.index)
    np.testing.assert_array_equal(r.fdr.values, e.fdr.values)


def test_rebalance_recuts_from_measured_times():
    """distributed.rebalance (bench.py's one re-cut after the warm-up): a rank measured slower than its estimate
    gives up ions to its neighbours, every ion stays in exactly one shard, the cut is the same on every rank, and
    times proportional to the estimates keep the cut."""
    from sm_distributed_amd import distributed as D
    ds, ions, ppm, f = _case()
    mz = torch.from_numpy(ds.mz.astype(np.float32))
    world = 3
    plans = [D.plan_shards(f, mz, ppm, world, r) for r in range(world)]
    est = plans[0].est_cost
    same = [D.rebalance(p, f, mz, est) for p in plans]
    assert [p.counts for p in same] == [plans[0].counts] * world
    slow = [2.0 * est[0], est[1], est[2]]
    new = [D.rebalance(p, f, mz, slow) for p in plans]
    assert all(p.counts == new[0].counts for p in new) and sum(new[0].counts) == f.n_ions
    assert new[0].counts[0] < plans[0].counts[0]
    got = np.sort(np.concatenate([p.ion_idx for p in new]))
    np.testing.assert_array_equal(got, np.arange(f.n_ions))
    with pytest.raises(ValueError):
        D.rebalance(plans[0], f, mz, [1.0, 0.0, 1.0])


def test_rebalance_head_cuts_rank0_smaller():
    """rebalance(head_seconds=...): rank 0's assembly of the gathered table is work the other ranks do not wait for
    in back-to-back searches, so its shard is cut smaller by it (shard_bounds' head); every ion stays in exactly
    one shard, the cut is the same on every rank, a negative head is refused."""
    from sm_distributed_amd import distributed as D
    ds, ions, ppm, f = _case()
    mz = torch.from_numpy(ds.mz.astype(np.float32))
    world = 3
    plans = [D.plan_shards(f, mz, ppm, world, r) for r in range(world)]
    est = plans[0].est_cost
    head = 0.3 * est[0]
    new = [D.rebalance(p, f, mz, est, head_seconds=head) for p in plans]
    assert all(p.counts == new[0].counts for p in new) and sum(new[0].counts) == f.n_ions
    assert new[0].counts[0] < plans[0].counts[0]
    got = np.sort(np.concatenate([p.ion_idx for p in new]))
    np.testing.assert_array_equal(got, np.arange(f.n_ions))
    # rank 0's estimated cost plus the head is about every other rank's
    e = new[0].est_cost
    assert abs((e[0] + head) - e[1]) < 0.1 * e[1] and abs(e[1] - e[2]) < 0.1 * e[1]
    with pytest.raises(ValueError):
        D.rebalance(plans[0], f, mz, est, head_seconds=-1.0)


def test_rebalance_rounds_converge_on_measured_times():
    """Repeated rebalance (bench.py's re-cuts until the ranks agree within 3 %): with a hidden per-ion cost that the
    model gets wrong by a smooth factor (x3 across the m/z range) plus a fixed per-rank cost, each round scales the
    costs of the previous cut (plan.costs) and the spread of the simulated rank times shrinks below 3 % within three
    rounds, every ion in exactly one shard on every rank."""
    from sm_distributed_amd import distributed as D
    ds, ions, ppm, f = _case()
    mz = torch.from_numpy(ds.mz.astype(np.float32))
    world = 4
    order, model = D._principal_costs(f, mz, ppm, 8192)
    true = model * np.linspace(1.0, 3.0, len(model))  # principal order

    def times_of(p):
        return [float(true[a:b].sum()) + 0.05 * float(true.sum()) / world for a, b in p.bounds]

    plans = [D.plan_shards(f, mz, ppm, world, r) for r in range(world)]
    spreads = []
    for _ in range(4):
        t = times_of(plans[0])
        spreads.append(max(t) / min(t) - 1.0)
        if spreads[-1] <= 0.03:
            break
        plans = [D.rebalance(p, f, mz, t) for p in plans]
        assert all(p.counts == plans[0].counts for p in plans) and sum(plans[0].counts) == f.n_ions
    assert spreads[0] > 0.1 and spreads[-1] <= 0.03, spreads
    got = np.sort(np.concatenate([p.ion_idx for p in plans]))
    np.testing.assert_array_equal(got, np.arange(f.n_ions))
