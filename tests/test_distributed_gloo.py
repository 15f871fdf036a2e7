"""N>1 path on CPU: world_size-2 gloo ranks shard the ions, score their shard, all-gather the fixed-size
metric rows; rank 0 must rebuild exactly the single-process table.  (On the GPU the same code runs over
RCCL with the device scorer; here the oracle stands in for the scorer.)"""
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


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import msm_oracle as O
        from sm_distributed_amd import distributed as D
        from sm_distributed_amd.engine import IonMetrics
        from tests.parity_cases import make_case, sf_peak_df, sf_peak_ints, subset_ions
        ds, ions, ppm, kw = make_case("basic")
        costs = D.ion_costs(ions.win_off, ions.peak_mz)
        a, b = D.shard_bounds(costs, world)[rank]
        shard = subset_ions(ions, np.arange(a, b))
        pm, dims = ds.pixel_map_dims()
        imgs = O.compute_sf_images(ds.spectra(), pm, dims, sf_peak_df(shard), ppm)
        ints = sf_peak_ints(shard)
        n = shard.n_ions
        vals = np.zeros((n, 5))
        for i, key in enumerate(zip(shard.sf_ids.tolist(), shard.adducts.tolist())):
            if key in imgs:
                c, s, p = O.compute_img_metrics(imgs[key], ints[key], dims[0], dims[1], 30)
                vals[i] = (c, s, p, c * s * p, 1)
        t = lambda j: torch.tensor(vals[:, j])
        m = IonMetrics(t(0), t(1), t(2), t(3), torch.tensor(vals[:, 4].astype(np.int32)))
        counts = D.exchange_counts(n, "cpu")
        rows = D.pack_rows(m, max(counts), device="cpu")
        table = D.gather_rows(rows, counts)
        if rank == 0:
            keys = list(zip(ions.sf_ids.tolist(), ions.adducts.tolist()))
            D.rows_to_frame(table, keys).to_pickle(out_path)
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


def test_two_rank_gather_matches_single_process(tmp_path):
    from oracle import msm_oracle as O
    from tests.parity_cases import make_case, oracle_run
    out = str(tmp_path / "rank0.pkl")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = pd.read_pickle(out)
    ds, ions, ppm, kw = make_case("basic")
    _, exp = oracle_run(ds, ions, ppm)
    got = got.sort_index()
    exp = exp.sort_index()
    assert got.index.equals(exp.index)
    for c in ("chaos", "spatial", "spectral", "msm"):
        np.testing.assert_allclose(got[c].values, exp[c].values, atol=1e-12)
