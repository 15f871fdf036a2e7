"""Multi-GPU layer: ion sharding + one collective for the per-ion metric rows.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Ions are independent, so the
formula list is sharded with the peak list replicated on every rank; the only exchange is a single
all-gather of fixed-size metric rows (chaos, spatial, spectral, msm, flags as f64 = 40 B/row), after
which rank 0 builds the reference DataFrame and runs FDR.  Images stay on the rank that scored them.

Sharding balances an estimated per-ion cost: the number of window points grows linearly with m/z for a
uniform-density dataset, and the reference's own workload model is exactly a product of histograms
(formula_imager_segm.py:9-14 _estimate_mz_workload); ``ion_costs`` uses the dataset's m/z histogram when
given, else sum of window m/z.  Contiguous shards in ion-table order keep each rank's windows spread over
the whole m/z range (ions are ordered by formula, not by mass).
"""
from __future__ import annotations

import numpy as np


def ion_costs(win_off, peak_mz, mz_hist=None, mz_edges=None):
    """Estimated points read per ion: sum over its windows of (histogram density at m/z) * window width."""
    win_off = np.asarray(win_off)
    peak_mz = np.asarray(peak_mz, dtype=np.float64)
    if mz_hist is not None:
        idx = np.clip(np.searchsorted(mz_edges, peak_mz) - 1, 0, len(mz_hist) - 1)
        dens = np.asarray(mz_hist, dtype=np.float64)[idx] / np.diff(mz_edges)[idx]
        w = dens * peak_mz
    else:
        w = peak_mz
    w = np.where(np.isfinite(w), w, 0.0)
    cs = np.concatenate([[0.0], np.cumsum(w)])
    return cs[win_off[1:]] - cs[win_off[:-1]] + 1.0  # +1: per-ion fixed cost


def shard_bounds(costs, world):
    """Contiguous [a, b) ion ranges with ~equal summed cost (greedy cut on the cost prefix sum)."""
    costs = np.asarray(costs, dtype=np.float64)
    n = len(costs)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    pref = np.concatenate([[0.0], np.cumsum(costs)])
    total = pref[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(pref, total * r / world)))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.array(cuts))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


ROW_FIELDS = ("chaos", "spatial", "spectral", "msm", "flags")


def pack_rows(metrics, n_max, device=None):
    """[n_max, 5] f64 row block of one rank (zero padded)."""
    import torch
    n = metrics.chaos.numel()
    dev = device if device is not None else metrics.chaos.device
    out = torch.zeros(n_max, len(ROW_FIELDS), dtype=torch.float64, device=dev)
    for j, f in enumerate(ROW_FIELDS):
        out[:n, j] = getattr(metrics, f).to(dev, dtype=torch.float64)
    return out


def gather_rows(rows, counts, group=None):
    """All-gather every rank's [n_max, 5] block; returns the concatenated [sum(counts), 5] table (every rank)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n_max = rows.shape[0]
    recv = torch.empty(world * n_max, rows.shape[1], dtype=rows.dtype, device=rows.device)
    dist.all_gather_into_tensor(recv, rows, group=group)
    parts = [recv[r * n_max: r * n_max + counts[r]] for r in range(world)]
    return torch.cat(parts, 0)


def exchange_counts(n_local, device, group=None):
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.tensor([n_local], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return [int(x.item()) for x in out]


def rows_to_frame(table, keys):
    """Rank-0 assembly: rows (global ion order) -> reference DataFrame for ions with images."""
    import pandas as pd
    t = table.cpu().numpy() if hasattr(table, "cpu") else np.asarray(table)
    has = (t[:, 4].astype(np.int64) & 1) != 0
    idx = np.nonzero(has)[0]
    df = pd.DataFrame({"sf_id": [keys[i][0] for i in idx], "adduct": [keys[i][1] for i in idx],
                       "chaos": t[idx, 0], "spatial": t[idx, 1], "spectral": t[idx, 2]},
                      columns=["sf_id", "adduct", "chaos", "spatial", "spectral"]).set_index(["sf_id", "adduct"])
    df["msm"] = df.chaos * df.spatial * df.spectral
    return df
