"""Ion-image generation: drop-in for sm/engine/msm_basic/formula_imager_segm.py.

``compute_sf_images(sc, ds, sf_peak_df, ppm)`` (reference :142-161) returns an ``IonImageSet``: the images
stay in HBM as (window -> [lo, hi) run of the m/z-sorted hit array) and are materialised as scipy COO
matrices only when a caller iterates them.  Semantics (complete-window):

* window = points with ``mz - mz*ppm*1e-6 <= mz_point <= mz + mz*ppm*1e-6`` (f64 bounds, :79-82);
* an (ion, peak_i) image exists iff its window holds >= 1 point, zero intensities included (:85-86);
* an ion appears iff >= 1 of its images exists; its list has length max(peak_i with image)+1 with
  ``None`` gaps (:95-109); duplicate pixels are summed by ``toarray()``.

The reference's m/z segmentation and chunking (:9-49, :68-69) only partition this same computation
over Spark workers; on one GPU the whole sorted peak list is resident, so neither exists here.

Host work is O(columns), never O(ions) in Python: the ion layout of ``sf_peak_df`` (ion identity, windows per
ion, window m/z in ion-major order, processing orders) is built on the device from three uploaded columns
(``device_layout``), on a side stream while the resident peaks are flagged and sorted on the main stream.
"""
from __future__ import annotations

import ctypes
import os
import threading
import warnings

import numpy as np
import pandas as pd
from scipy.sparse import coo_matrix

from .rdd import LocalRDD


class IonKeys:
    """(sf_id, adduct) of every ion of a layout, encoded ``key = sf_code * n_adducts + adduct_code`` and
    sorted, so ion order = (sf_id, adduct) order, the order of the reference's sf_df (formulas_segm.py:43-44).

    ``sf_code`` is the sf_id itself for integer ids (``sf_levels`` None), else its position in the sorted
    ``sf_levels``; ``adducts`` are the sorted adduct strings."""

    def __init__(self, keys: np.ndarray, adducts, sf_levels=None, keys_dev=None, codes=None, codes_dev=None):
        self.keys = keys
        self.keys_dev = keys_dev  # the same keys in HBM (device_layout keeps them)
        self.adducts = list(adducts)
        self.sf_levels = sf_levels
        self.n_cat = max(len(self.adducts), 1)
        self._tuples = None
        self._codes = codes       # (sf level values, sf code, adduct code) per ion, for multi_index
        self._codes_dev = {}      # device -> (int32 sf codes, int16 adduct codes) tensors
        if codes_dev is not None:
            self._codes_dev[str(codes_dev[0].device)] = codes_dev

    def __len__(self):
        return len(self.keys)

    @property
    def sf_code(self):
        return self.keys // self.n_cat

    @property
    def adduct_code(self):
        return (self.keys % self.n_cat).astype(np.int64)

    def sf_values(self, idx=None):
        c = self.sf_code if idx is None else self.keys[idx] // self.n_cat
        return c if self.sf_levels is None else np.asarray(self.sf_levels)[c]

    def tuples(self):
        if self._tuples is None:
            ad = np.asarray(self.adducts, dtype=object)[self.adduct_code]
            self._tuples = list(zip(self.sf_values().tolist(), ad.tolist()))
        return self._tuples

    def encode_codes(self, sf, adduct_codes, adducts):
        """encode() for adducts given as codes into the string list ``adducts`` (no per-row string hashing)."""
        cmap = pd.Index(self.adducts, dtype=object).get_indexer(pd.Index(list(adducts), dtype=object))
        code = cmap[np.asarray(adduct_codes, dtype=np.int64)] if len(cmap) else np.zeros(len(sf), np.int64)
        sf = np.asarray(sf)
        if self.sf_levels is None:
            sfc = sf.astype(np.int64) if sf.dtype.kind in "iu" else np.full(len(sf), -1, np.int64)
            ok = code >= 0
        else:
            sfc = pd.Index(self.sf_levels).get_indexer(pd.Index(sf)).astype(np.int64)
            ok = (code >= 0) & (sfc >= 0)
        return np.where(ok, sfc * self.n_cat + code, -1), ok

    def encode(self, sf, adducts):
        """Keys of (sf_id, adduct) pairs in this encoding; -1 for pairs that cannot be in it."""
        code = pd.Index(self.adducts, dtype=object).get_indexer(pd.Index(np.asarray(adducts, dtype=object)))
        sf = np.asarray(sf)
        if self.sf_levels is None:
            sfc = sf.astype(np.int64) if sf.dtype.kind in "iu" else np.full(len(sf), -1, np.int64)
            ok = code >= 0
        else:
            sfc = pd.Index(self.sf_levels).get_indexer(pd.Index(sf)).astype(np.int64)
            ok = (code >= 0) & (sfc >= 0)
        return np.where(ok, sfc * self.n_cat + code, -1), ok

    def level_codes(self):
        """(sf level values, int32 sf codes, int16 adduct codes) of every ion: the MultiIndex levels/codes."""
        if self._codes is None:
            sfc = self.keys // self.n_cat
            adc = (self.keys - sfc * self.n_cat).astype(np.int16)
            if self.sf_levels is None:
                new = np.ones(len(sfc), bool)
                new[1:] = sfc[1:] != sfc[:-1]  # keys sorted -> sf codes nondecreasing
                self._codes = (sfc[new], (np.cumsum(new) - 1).astype(np.int32), adc)
            else:
                self._codes = (np.asarray(self.sf_levels), sfc.astype(np.int32), adc)
        return self._codes

    def codes_dev(self, device):
        """level_codes()' sf and adduct codes as device tensors (cached per device)."""
        import torch
        cache = self._codes_dev
        key = str(device)
        if key not in cache:
            _, sfc, adc = self.level_codes()
            cache[key] = (torch.from_numpy(sfc).to(device), torch.from_numpy(adc).to(device))
        return cache[key]

    def multi_index_from_codes(self, sf_codes, ad_codes):
        """pd.MultiIndex [sf_id, adduct] from already gathered codes (the levels are those of the whole layout)."""
        sf_lv = self.level_codes()[0]
        return pd.MultiIndex(levels=[pd.Index(sf_lv), pd.Index(self.adducts, dtype=object)],
                             codes=[sf_codes, ad_codes], names=["sf_id", "adduct"], verify_integrity=False)

    def multi_index(self, idx):
        """pd.MultiIndex [sf_id, adduct] of the ions ``idx`` (ascending positions), built from codes (two
        gathers; the levels are those of the whole layout)."""
        sf_lv, sf_codes, ad_codes = self.level_codes()
        return pd.MultiIndex(levels=[pd.Index(sf_lv), pd.Index(self.adducts, dtype=object)],
                             codes=[sf_codes[idx], ad_codes[idx]], names=["sf_id", "adduct"],
                             verify_integrity=False)


def _adduct_codes(col):
    """(integer codes -- int8/16/32 straight from a Categorical, no copy --, sorted category strings) of an
    adduct column; a non-Categorical column is factorized (slow path: hashes every string)."""
    if isinstance(col.dtype, pd.CategoricalDtype):
        cats = [str(c) for c in col.cat.categories]
        codes = col.cat.codes.to_numpy()
        order = np.argsort(np.array(cats, dtype=object), kind="stable")
        if not (order == np.arange(len(cats))).all():
            rank = np.empty(len(cats), np.int64)
            rank[order] = np.arange(len(cats))
            codes = np.where(codes >= 0, rank[np.maximum(codes, 0)], -1)
            cats = [cats[i] for i in order]
    else:
        codes, uniq = pd.factorize(col.to_numpy(dtype=object), sort=True)
        cats = [str(u) for u in uniq]
    return codes, cats


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def device_layout(sf_peak_df: pd.DataFrame, device, stream=None):
    """Ion-major window table of FormulasSegm.get_sf_peak_df rows (sf_id, adduct, peak_i, mz), on the device.

    An ion gets max(peak_i)+1 windows (formula_imager_segm.py:95-109: list length max(peak_i)+1); windows
    without a row are padding (m/z -1: no point can match).  Returns (IonKeys, DeviceIons, K per ion)."""
    import torch

    from .engine import DeviceIons
    # the four columns go to the device as they are (no host-side arithmetic: zero-copy views of int64 / f64 /
    # Categorical-code columns), and the ion key is formed there
    sf = sf_peak_df["sf_id"].to_numpy()
    codes, cats = _adduct_codes(sf_peak_df["adduct"])
    n_cat = max(len(cats), 1)
    sf_levels = None
    if sf.dtype.kind not in "iu":
        sf, sf_levels = pd.factorize(sf, sort=True)
    peak_i = sf_peak_df["peak_i"].to_numpy()
    mz = sf_peak_df["mz"].to_numpy()
    if peak_i.dtype.kind not in "iu" or mz.dtype != np.float64:
        peak_i, mz = peak_i.astype(np.int64), mz.astype(np.float64)
    n_rows = len(sf)
    def t(a):  # host column -> device (read-only views, e.g. Categorical codes, are only read by the copy)
        a = np.ascontiguousarray(a)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            return torch.from_numpy(a).to(device)
    with torch.cuda.stream(stream) if stream is not None else _nullctx():
        if n_rows == 0:
            z = torch.zeros(1, dtype=torch.int64, device=device)
            e = torch.zeros(0, dtype=torch.int64, device=device)
            ions = DeviceIons(win_off=z, peak_mz=torch.zeros(0, dtype=torch.float64, device=device), theor=None,
                              win_order=e, ion_order=e, n_ions=0, n_windows=0, max_k=0)
            return IonKeys(np.zeros(0, np.int64), cats, sf_levels), ions, e
        sf_d, code_d, pk_d, mz_d = t(sf).long(), t(codes).long(), t(peak_i).long(), t(mz)
        key_d = sf_d * n_cat + code_d
        # one synchronisation for the key range and the checks: sf range, missing adducts, negative peak_i
        # and two facts that make later steps cheaper: rows in m/z order, one peak_i = 0 row per ion
        mz_sorted_rows = (mz_d[1:] >= mz_d[:-1]).all() if n_rows > 1 else torch.ones((), dtype=torch.bool,
                                                                                      device=device)
        kmin, kmax_key, sf_max, code_min, pk_min, rows_sorted, n_pk0, mz_pos = (int(v) for v in torch.stack(
            [key_d.min(), key_d.max(), sf_d.abs().max(), code_d.min(), pk_d.min(), mz_sorted_rows.long(),
             (pk_d == 0).sum(), (mz_d > 0).all().long()]).cpu().tolist())
        if sf_max >= (1 << 62) // n_cat:
            raise ValueError("sf_id out of range")
        if code_min < 0:
            raise ValueError("sf_peak_df has missing adducts")
        if pk_min < 0:
            raise ValueError("negative peak_i in sf_peak_df")
        span = kmax_key - kmin + 1
        if kmin >= 0 and span <= 8 * n_rows + (1 << 22):
            # dense key range (integer sf ids): ion index = rank of the key among the present ones, from a
            # presence table and its prefix sum -- no sort of the rows
            present = torch.zeros(span, dtype=torch.int32, device=device)
            present[key_d - kmin] = 1
            rank = torch.cumsum(present, 0, dtype=torch.int64)
            inv = rank[key_d - kmin] - 1
            uniq = torch.nonzero(present).flatten() + kmin  # synchronises (output size)
        else:
            uniq, inv = torch.unique(key_d, sorted=True, return_inverse=True)  # synchronises (output size)
        n_ions = uniq.numel()
        K = torch.zeros(n_ions, dtype=torch.int64, device=device)
        K.scatter_reduce_(0, inv, pk_d + 1, reduce="amax", include_self=True)
        win_off = torch.zeros(n_ions + 1, dtype=torch.int64, device=device)
        torch.cumsum(K, 0, out=win_off[1:])
        n_win, kmax = (int(v) for v in torch.stack([win_off[-1], K.max()]).cpu().tolist())
        slot = win_off[inv] + pk_d
        peak_mz = torch.full((n_win,), -1.0, dtype=torch.float64, device=device)
        peak_mz.scatter_(0, slot, mz_d)
        if n_win == n_rows and mz_pos:
            # as many rows as windows: a duplicate (sf_id, adduct, peak_i) row would leave a window unfilled
            win_order = slot  # rows come in m/z order (get_sf_peak_df sorts by mz): the search's locality order
            dup_rows = (peak_mz.min() < 0).to(torch.int64)
        else:
            # rows per window (atomic adds; torch.bincount runs a slow histogram kernel on ROCm)
            per_slot = torch.zeros(n_win, dtype=torch.int32, device=device)
            per_slot.index_add_(0, slot, torch.ones(1, dtype=torch.int32, device=device).expand(n_rows))
            win_order = torch.cat([slot, torch.nonzero(per_slot == 0).flatten()])
            dup_rows = ((per_slot.max() if n_win else torch.zeros((), dtype=torch.int32, device=device)) > 1
                        ).to(torch.int64)
        if rows_sorted and n_pk0 == n_ions:
            # ions in principal m/z order = the peak_i = 0 rows in row order (a stable compaction, no sort)
            is0 = pk_d == 0
            pos = torch.cumsum(is0.to(torch.int64), 0) - 1
            buf = torch.empty(n_ions + 1, dtype=torch.int64, device=device)
            buf.scatter_(0, torch.where(is0, pos, torch.full_like(pos, n_ions)), inv)
            ion_order = buf[:n_ions]
        else:
            first = peak_mz[win_off[:-1]]
            first = torch.where(first < 0, torch.full_like(first, float("inf")), first)
            ion_order = torch.sort(first, stable=True).indices
        # MultiIndex codes of every ion, formed on the device (keys sorted: sf codes nondecreasing); the host
        # forms the same codes from the keys when it needs them (IonKeys.level_codes)
        sfc = torch.div(uniq, n_cat, rounding_mode="floor")
        adc = (uniq - sfc * n_cat).to(torch.int16)
        if sf_levels is None:
            new = torch.ones(n_ions, dtype=torch.bool, device=device)
            new[1:] = sfc[1:] != sfc[:-1]
            codes_dev = (torch.cumsum(new.to(torch.int32), 0, dtype=torch.int32) - 1, adc)
        else:
            codes_dev = (sfc.to(torch.int32), adc)
        # the keys and the duplicate-row check in one copy
        tail = torch.cat([uniq, dup_rows.reshape(1)]).cpu().numpy()
        keys = tail[:-1]
        if int(tail[-1]):
            raise AssertionError("duplicate (sf_id, adduct, peak_i) rows in sf_peak_df")
        codes = None
    ions = DeviceIons(win_off=win_off, peak_mz=peak_mz, theor=None, win_order=win_order, ion_order=ion_order,
                      n_ions=n_ions, n_windows=n_win, max_k=kmax)
    return IonKeys(keys, cats, sf_levels, keys_dev=uniq, codes=codes, codes_dev=codes_dev), ions, K


# The ion layout of an sf_peak_df is a function of its four columns only, and a search per dataset runs over the same
# formula table (the reference keeps it in Postgres, formulas_segm.py:14-33): the last few layouts are kept, addressed
# by a hash of the columns' contents (not by object identity), so an edited or new table always gets its own layout.
_LAYOUT_CACHE = {}
_LAYOUT_KEEP = 4


def _layout_key(sf_peak_df, device):
    """xxh3-128 of the sf_id / peak_i / mz columns and the adduct column's categories + codes (None -- no caching --
    for a non-Categorical adduct column or non-integer sf ids: those take the slow path anyway).  ~1 ms per 1M rows,
    on the host while the device sorts."""
    import xxhash
    adduct = sf_peak_df["adduct"]
    sf = sf_peak_df["sf_id"].to_numpy()
    if not isinstance(adduct.dtype, pd.CategoricalDtype) or sf.dtype.kind not in "iu":
        return None
    h = xxhash.xxh3_128()
    for a in (sf, sf_peak_df["peak_i"].to_numpy(), sf_peak_df["mz"].to_numpy(), adduct.cat.codes.to_numpy()):
        a = np.ascontiguousarray(a)
        h.update(f"{a.dtype.str}{a.shape}".encode())
        h.update(a.view(np.uint8).reshape(-1) if a.size else b"")
    h.update("\x00".join(str(c) for c in adduct.cat.categories).encode())
    return (h.hexdigest(), str(device))


def cached_device_layout(sf_peak_df, device, stream=None):
    """device_layout(sf_peak_df, device, stream), reused while a table with the same contents comes again."""
    key = _layout_key(sf_peak_df, device)
    if key is not None and key in _LAYOUT_CACHE:
        return _LAYOUT_CACHE[key]
    out = device_layout(sf_peak_df, device, stream)
    if key is not None:
        while len(_LAYOUT_CACHE) >= _LAYOUT_KEEP:
            _LAYOUT_CACHE.pop(next(iter(_LAYOUT_CACHE)))
        _LAYOUT_CACHE[key] = out
    return out


METRIC_COLUMNS = ["chaos", "spatial", "spectral", "msm"]


def device_frame(ion_keys, cols, idx, cols_compact=False):
    """The reference metrics DataFrame (index [sf_id, adduct], columns chaos, spatial, spectral, msm) of the ions
    ``idx`` (device tensor, ascending positions of ``ion_keys``) from device metric columns ``cols`` [4, >n] (or
    [4, len(idx)] already in that order, ``cols_compact``): the rows and the index codes are gathered on the
    device and copied to pinned host memory, the codes first so that the MultiIndex is built while the columns
    copy; the DataFrame wraps the column-major block without a copy."""
    import torch
    sfc, adc = ion_keys.codes_dev(cols.device)
    parts = (sfc[idx], adc[idx], cols if cols_compact else cols[:, idx])
    if cols.device.type == "cuda":
        # the codes first: the MultiIndex is built on the host while the metric columns are still copying
        st = torch.cuda.current_stream(cols.device)
        host = [torch.empty(x.shape, dtype=x.dtype, pin_memory=True) for x in parts]
        host[0].copy_(parts[0], non_blocking=True)
        host[1].copy_(parts[1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(st)
        host[2].copy_(parts[2], non_blocking=True)
        ev.synchronize()
        mi = ion_keys.multi_index_from_codes(host[0].numpy(), host[1].numpy())
        st.synchronize()
    else:
        host = parts
        mi = ion_keys.multi_index_from_codes(host[0].numpy(), host[1].numpy())
    return pd.DataFrame(host[2].numpy().T, index=mi, columns=METRIC_COLUMNS, copy=False)


_STAGE = {}  # device -> [copy stream, free pinned uint8 buffers, lock]
_STAGE_LOCK = threading.Lock()


def _stage_buffers(device, n):
    """A pinned host buffer of >= n bytes taken from the device's pool of free staging buffers (allocated only when
    none is free: the per-step row mask never allocates pinned memory in steady state) and the device's copy stream.
    The buffer belongs to the caller until ``_release_stage_buffer``: a pending frame's mask is never overwritten,
    whatever the thread or the number of stages in flight."""
    import torch
    key = str(device)
    with _STAGE_LOCK:
        ent = _STAGE.get(key)
        if ent is None:
            ent = _STAGE[key] = [torch.cuda.Stream(device=device), [], threading.Lock()]
    with ent[2]:
        for i, b in enumerate(ent[1]):
            if b.numel() >= n:
                return ent[0], ent[1].pop(i)
    return ent[0], torch.empty(max(int(n), 1 << 20), dtype=torch.uint8, pin_memory=True)


def _release_stage_buffer(device, buf):
    ent = _STAGE.get(str(device))
    if ent is not None and buf is not None:
        with ent[2]:
            ent[1].append(buf)


class FrameIndex:
    """device_frame in two halves around a kernel launch.  ``stage(keep)`` (device bool[n_ion], queued before the
    launch) copies the row mask to a persistent pinned buffer on a copy stream of its own, which the compute stream
    waits for before the kernel (no copy runs beside it; the host does not synchronise) -- and takes the pinned block the
    DataFrame's columns will live in.  ``frame(cols)`` (after the launch) builds the MultiIndex on the host from
    the mask while the kernel still runs, then compacts the metric columns on the device (a scatter, no host
    synchronisation) and copies them to that block."""

    def __init__(self, ion_keys):
        self.ion_keys = ion_keys
        self.keep = None

    def stage(self, keep):
        import torch
        self.keep = keep
        if keep.device.type == "cuda" and _one_stream():
            n = keep.numel()
            main = torch.cuda.current_stream(keep.device)
            _, buf = _stage_buffers(keep.device, n)
            self._stage_buf = buf
            buf[:n].copy_(keep.view(torch.uint8), non_blocking=True)
            self.ev = torch.cuda.Event()
            self.ev.record(main)
            self.keep_host = buf[:n]
            self.cols_host = torch.empty(4 * n, dtype=torch.float64, pin_memory=True)
        elif keep.device.type == "cuda":
            n = keep.numel()
            main = torch.cuda.current_stream(keep.device)
            cs, buf = _stage_buffers(keep.device, n)
            self._stage_buf = buf
            cs.wait_stream(main)
            with torch.cuda.stream(cs):
                buf[:n].copy_(keep.view(torch.uint8), non_blocking=True)
                self.ev = torch.cuda.Event()
                self.ev.record(cs)
            keep.record_stream(cs)
            # the compute stream waits for the copy (no copy runs beside the persistent ion kernel).  The 10-ms
            # step quanta once blamed on such a copy are KFD queue evictions of the whole process (round 5:
            # evicted_ms grows by exactly those quanta, and a pending copy, barrier or kernel on a second queue
            # was measured not to stall a CU-filling kernel, scripts/queue_slice_probe.hip)
            main.wait_event(self.ev)
            self.keep_host = buf[:n]
            # the DataFrame's own pinned block (caching host allocator: reused once an earlier frame is freed),
            # taken before the kernel: a pinned allocation while a kernel runs remaps host memory and was seen to
            # stall the kernel (first calls of a process)
            self.cols_host = torch.empty(4 * n, dtype=torch.float64, pin_memory=True)
        else:
            self.ev = None

    def frame(self, cols):
        import torch
        keep = self.keep
        if self.ev is None:
            idx = torch.nonzero(keep).flatten().numpy()
            _, sfc, adc = self.ion_keys.level_codes()
            mi = self.ion_keys.multi_index_from_codes(sfc[idx], adc[idx])
            return pd.DataFrame(cols[:, idx].numpy().T, index=mi, columns=METRIC_COLUMNS, copy=False)
        self.ev.synchronize()  # the mask was copied before the kernel ran: ready while it runs
        idx = np.flatnonzero(self.keep_host.numpy())
        self.keep_host = None
        _release_stage_buffer(keep.device, self.__dict__.pop("_stage_buf", None))  # (the mask is read)
        m = len(idx)
        _, sfc, adc = self.ion_keys.level_codes()
        mi = self.ion_keys.multi_index_from_codes(sfc[idx], adc[idx])
        # rows of kept ions in table order, compacted on the device: row k of ion i goes to k*m + (rank of i among
        # the kept ions); the others to a dummy slot 4m
        n = keep.numel()
        pos = torch.cumsum(keep, 0) - 1
        dst = torch.arange(4, device=cols.device).unsqueeze(1) * m + pos.unsqueeze(0)
        dst = torch.where(keep.unsqueeze(0), dst, torch.full_like(dst, 4 * m))
        out = torch.empty(4 * m + 1, dtype=torch.float64, device=cols.device)
        out.scatter_(0, dst.flatten(), cols[:, :n].reshape(-1))
        host = self.cols_host[:4 * m]
        host.copy_(out[:4 * m], non_blocking=True)
        torch.cuda.current_stream(cols.device).synchronize()
        return pd.DataFrame(host.view(4, m).numpy().T, index=mi, columns=METRIC_COLUMNS, copy=False)


class ImageRows:
    """Columnar iso_image rows of an IonImageSet: per listed window (ion ``ion[j]``, peak ``peak[j]``) its
    ``counts[j]`` pixels above the threshold at ``pix/val[off[j]:off[j+1]]`` (ascending flattened index) and the
    image's ``vmin/vmax``; ``rows(job_id, db_id)`` yields the reference's tuples (search_results.py:93-95)."""

    def __init__(self, keys, ion, peak, counts, pix, val, vmin, vmax):
        self.keys, self.ion, self.peak, self.counts = keys, ion, peak, counts
        self.pix, self.val, self.vmin, self.vmax = pix, val, vmin, vmax
        self.off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)

    def rows(self, job_id, db_id):
        for j in np.nonzero(self.counts > 0)[0].tolist():
            sf_id, adduct = self.keys[int(self.ion[j])]
            a, b = self.off[j], self.off[j + 1]
            yield (job_id, db_id, sf_id, adduct, int(self.peak[j]), self.pix[a:b].tolist(), self.val[a:b].tolist(),
                   self.vmin[j], self.vmax[j])


class IonImageSet:
    """Device-resident ``RDD[((sf_id, adduct), [coo | None, ...])]``."""

    def __init__(self, peaks, ion_keys: IonKeys, ions_dev, K, lo, hi, dims, ppm=None):
        self.peaks = peaks              # DevicePeaks (sorted)
        self.ion_keys = ion_keys        # IonKeys: ion i = (sf_id, adduct), (sf_id, adduct) order
        self.ions_dev = ions_dev        # engine.DeviceIons: win_off, window m/z, ion_order (principal m/z)
        self.K = K                      # device int64[n_ion]: windows per ion (max(peak_i) + 1)
        self.lo = lo                    # device int64[n_win]
        self.hi = hi
        self.dims = dims
        self.ppm = ppm                  # the ppm of the duplicate flags and windows
        self.peaks_version = peaks.version if peaks is not None else 0
        self._has_dev = None
        self._has = None
        self._win_counts = None
        self._win_off = None
        self._sel = None                # optional ion subset (filter_by_keys)

    @property
    def n_ions(self):
        return len(self.ion_keys)

    @property
    def keys(self):
        """list[(sf_id, adduct)] in ion order (built on first use)."""
        return self.ion_keys.tuples()

    @property
    def win_off(self):
        if self._win_off is None:
            self._win_off = self.ions_dev.win_off.cpu().numpy()
        return self._win_off

    def ensure_current(self):
        """Restore the sorted peaks this set was built on if another compute_sf_images (another ppm) re-flagged
        and re-sorted them since: the duplicate-candidate flags must be those of this set's windows.  The sort is
        stable and keyed by m/z only, so re-flagging at this ppm and re-sorting gives back the same positions."""
        p = self.peaks
        if p is not None and (p.version != self.peaks_version or p.flag_ppm != self.ppm):
            p.flag_and_sort(self.ppm)
            p.prefix_sums()
            self.peaks_version = p.version
        return self

    # ---- bookkeeping -------------------------------------------------------------------------
    def has_images_device(self):
        """device bool[n_ion]: the ion has >= 1 window with >= 1 point (it appears in the RDD)."""
        import torch
        if self._has_dev is None:
            # windows of an ion are contiguous: count non-empty windows per ion by prefix differences (no sync)
            c = torch.zeros(self.lo.numel() + 1, dtype=torch.int64, device=self.lo.device)
            torch.cumsum(((self.hi - self.lo) > 0).to(torch.int64), 0, out=c[1:])
            off = self.ions_dev.win_off
            self._has_dev = (c[off[1:]] - c[off[:-1]]) > 0
        return self._has_dev

    def _counts(self):
        if self._has is None:
            self._win_counts = (self.hi - self.lo).cpu().numpy()
            self._has = self.has_images_device().cpu().numpy()
        return self._win_counts, self._has

    def ion_indices(self):
        _, has = self._counts()
        idx = np.nonzero(has)[0]
        if self._sel is not None:
            idx = idx[self._sel[idx]]
        return idx

    def filter_by_keys(self, index) -> "IonImageSet":
        """Keep ions whose key is in ``index`` without materialising anything (filter_sf_images)."""
        if isinstance(index, pd.MultiIndex) and index.nlevels == 2:
            k, ok = self.ion_keys.encode(index.get_level_values(0).to_numpy(), index.get_level_values(1))
            sel = np.isin(self.ion_keys.keys, k[ok])
        else:
            keep = set(index)
            sel = np.array([t in keep for t in self.keys], dtype=bool)
        out = IonImageSet(self.peaks, self.ion_keys, self.ions_dev, self.K, self.lo, self.hi, self.dims, self.ppm)
        out.peaks_version = self.peaks_version
        out._has_dev, out._has, out._win_counts, out._win_off = self._has_dev, self._has, self._win_counts, \
            self._win_off
        out._sel = sel if self._sel is None else (sel & self._sel)
        return out

    # ---- materialisation -----------------------------------------------------------------------
    def materialize(self, ion_idx):
        """[(key, [coo|None...])] for the given ions; gathers only their windows from HBM."""
        import torch
        cnt, _ = self._counts()
        self.ensure_current()
        nrows, ncols = self.dims
        win_off = self.win_off
        ion_idx = np.asarray(ion_idx, dtype=np.int64)
        if ion_idx.size == 0:
            return []
        Kp = win_off[ion_idx + 1] - win_off[ion_idx]
        w = np.repeat(win_off[ion_idx], Kp) + np.arange(Kp.sum()) - np.repeat(np.cumsum(Kp) - Kp, Kp)
        c = cnt[w]
        total = int(c.sum())
        out_hits = np.zeros(0, np.uint64)
        if total:
            dev = self.lo.device
            wt = torch.from_numpy(w).to(dev)
            ct = torch.from_numpy(c).to(dev)
            starts = self.lo[wt]
            base = torch.repeat_interleave(starts, ct)
            offs = torch.repeat_interleave(torch.cumsum(ct, 0) - ct, ct)
            idx = base + (torch.arange(total, device=dev) - offs)
            out_hits = self.peaks.hits_sorted[idx].cpu().numpy().view(np.uint64)
        pix = (out_hits & np.uint64(0x7FFFFFFF)).astype(np.int64)
        val = (out_hits >> np.uint64(32)).astype(np.uint32).view(np.float32).astype(np.float64)
        keys = self.keys
        res = []
        pos = 0
        wpos = 0
        for i, k in zip(ion_idx.tolist(), Kp.tolist()):
            imgs = []
            for _ in range(k):
                n = int(c[wpos])
                if n:
                    p = pix[pos:pos + n]
                    imgs.append(coo_matrix((val[pos:pos + n], (p // ncols, p % ncols)), shape=(nrows, ncols)))
                else:
                    imgs.append(None)
                pos += n
                wpos += 1
            last = max((j for j, m in enumerate(imgs) if m is not None), default=-1)
            res.append((keys[i], imgs[:last + 1]))
        return res

    def image_rows(self, threshold=0.001):
        """The iso_image rows of every listed ion (search_results.py:88-97) computed on the device
        (smg_iso_image_rows: duplicates summed, pixels > threshold, ascending flattened index, min / max over the
        whole image) -- nothing densified.  Returns the columnar ``ImageRows`` (host arrays)."""
        import torch

        from ._lib import check, lib
        from .engine import _p, _stream, workspace
        self.ensure_current()
        ion_idx = self.ion_indices()
        win_off = self.win_off
        Kp = win_off[ion_idx + 1] - win_off[ion_idx]
        w = (np.repeat(win_off[ion_idx], Kp) + np.arange(Kp.sum()) - np.repeat(np.cumsum(Kp) - Kp, Kp)).astype(np.int64)
        peak_i = w - np.repeat(win_off[ion_idx], Kp)
        ion_of = np.repeat(ion_idx, Kp)
        nrows, ncols = self.dims
        n = len(w)
        dev = self.lo.device
        cnt, _ = self._counts()
        total = int(cnt[w].sum()) if n else 0
        out_count = torch.zeros(n, dtype=torch.int64, device=dev)
        out_min = torch.zeros(n, dtype=torch.float64, device=dev)
        out_max = torch.zeros(n, dtype=torch.float64, device=dev)
        out_pix = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
        out_val = torch.empty(max(total, 1), dtype=torch.float64, device=dev)
        if n:
            wt = torch.from_numpy(w).to(dev)
            lo, hi = self.lo[wt].contiguous(), self.hi[wt].contiguous()
            sz = ctypes.c_size_t(0)
            check(lib().smg_iso_image_rows_workspace_size(n, total, ctypes.byref(sz)),
                  "smg_iso_image_rows_workspace_size")
            ws = workspace(sz.value, dev, "rows")
            check(lib().smg_iso_image_rows(_p(self.peaks.hits_sorted), _p(lo), _p(hi), n, total, int(nrows * ncols),
                                           float(threshold), _p(out_count), _p(out_min), _p(out_max), _p(out_pix),
                                           _p(out_val), _p(ws), ws.numel(), _stream(None)), "smg_iso_image_rows")
        counts = out_count.cpu().numpy()
        m = int(counts.sum())
        return ImageRows(keys=self.keys, ion=ion_of, peak=peak_i, counts=counts, pix=out_pix[:m].cpu().numpy(),
                         val=out_val[:m].cpu().numpy(), vmin=out_min.cpu().numpy(), vmax=out_max.cpu().numpy())

    def _items(self):
        return self.materialize(self.ion_indices())

    # ---- RDD surface ---------------------------------------------------------------------------
    def collect(self):
        return self._items()

    def take(self, n):
        return self.materialize(self.ion_indices()[:n])

    def count(self):
        return int(len(self.ion_indices()))

    def map(self, f):
        return LocalRDD(self._items()).map(f)

    def flatMap(self, f):
        return LocalRDD(self._items()).flatMap(f)

    def filter(self, f):
        return LocalRDD(self._items()).filter(f)

    def mapValues(self, f):
        return LocalRDD(self._items()).mapValues(f)

    def foreachPartition(self, f):
        f(iter(self._items()))

    def keys_with_images(self):
        keys = self.keys
        return [keys[i] for i in self.ion_indices()]

    def cache(self):
        return self

    def __iter__(self):
        return iter(self._items())


_SIDE = {}


def _one_stream():
    """SMG_ONE_STREAM=1: every queued operation of a search on the caller's stream (no side or copy stream)."""
    return os.environ.get("SMG_ONE_STREAM", "0") == "1"


def _side_stream(device):
    import torch
    if _one_stream():
        return torch.cuda.current_stream(device)
    key = str(device)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


def compute_sf_images(sc, ds, sf_peak_df, ppm):
    """formula_imager_segm.py:142-161.  ``sc`` is accepted for signature compatibility and ignored.

    Device order: the resident peaks are flagged and sorted on the current stream while the ion layout is
    uploaded and built on a side stream (or taken from the layout cache when the same table comes again:
    ``cached_device_layout``); the window search follows both on the side stream, beside the prefix sums on the
    current one (a latency-bound search beside a bandwidth-bound read); the current stream joins."""
    import torch

    from .dataset import spectra_from_duck
    from .engine import DevicePeaks, window_bounds
    if hasattr(ds, "device_peaks"):
        peaks = ds.device_peaks()
    else:
        off, mz, it = spectra_from_duck(ds)
        peaks = DevicePeaks.from_arrays(off, mz, it, np.asarray(ds.norm_img_pixel_inds), ds.get_dims())
    main = torch.cuda.current_stream(peaks.device)
    # SMG_LAYOUT_SIDE=0 (diagnostic): the ion layout's kernels queue behind the sort on the main stream (its host
    # work still overlaps the sort) instead of running beside it on the side stream
    side = _side_stream(peaks.device) if os.environ.get("SMG_LAYOUT_SIDE", "1") != "0" else main
    side.wait_stream(main)  # the side stream may reuse memory the main stream released
    peaks.flag_and_sort(ppm)
    keys, dions, K = cached_device_layout(sf_peak_df, peaks.device, side)
    # the window search on the side stream after the sort; lo / hi are allocated on the main stream (the side
    # stream waits for everything queued on it so far, so memory the main stream released is free)
    side.wait_stream(main)
    lo, hi = window_bounds(peaks, dions, ppm, stream=side)
    peaks.prefix_sums()
    main.wait_stream(side)
    for t in (dions.win_off, dions.peak_mz, dions.win_order, dions.ion_order, K, keys.keys_dev):
        if t is not None:
            t.record_stream(main)
    return IonImageSet(peaks, keys, dions, K, lo, hi, ds.get_dims(), ppm)
