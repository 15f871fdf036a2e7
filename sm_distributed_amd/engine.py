"""Device pipeline of the hot path: resident peak list -> m/z sort -> window search -> fused ion metrics.

This is the layer the reference-API mirror (formula_imager_segm / formula_img_validator) sits on.
Every call goes through libsmg.so (include/smg.h) on the current torch stream; torch is used only for
HBM allocation and streams.  There is no CPU fallback: on a machine without a GPU these functions raise.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("sm_distributed_amd device path needs a ROCm GPU (no CPU fallback)")
    torch.cuda.init()  # the HIP runtime is torch's: initialise it before the library's first call
    lib()  # fail loudly if libsmg.so is missing


_ws_cache: dict = {}


def workspace(nbytes: int, device, tag: str) -> torch.Tensor:
    """Grow-only per-(tag, device) workspace so hot calls do not allocate."""
    key = (tag, str(device))
    t = _ws_cache.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
        _ws_cache[key] = t
    return t


@dataclass
class DevicePeaks:
    """The dataset resident in HBM.

    ``mz``: float32[N]; ``hits``: int64[N] holding uint64 ``pixel | f32bits(intensity) << 32``; both in
    dataset (spectrum) order.  ``mz_sorted``/``hits_sorted`` are the m/z-sorted copies made by ``sort``.
    """
    mz: torch.Tensor
    hits: torch.Tensor
    nrows: int
    ncols: int
    sp_off: torch.Tensor | None = None     # int64[n_spectra+1] (dataset order), for duplicate flags
    force: torch.Tensor | None = None      # uint8[n_spectra]: spectra whose pixel is shared (non-injective map)
    mz_sorted: torch.Tensor | None = None
    hits_sorted: torch.Tensor | None = None
    flag_ppm: float | None = None          # the ppm of the flags hits_sorted carries (what the ion kernels read)
    hits_flag_ppm: float | None = None     # the ppm of the flags the dataset-order hits carry (None: unknown/stale)
    sort_key_bits: int | None = None
    cum: torch.Tensor | None = None  # 64-point block double-double prefix sums of the sorted hits
    cum_valid: bool = False          # cum describes the current hits_sorted
    version: int = 0                 # bumped by every flag pass / sort: an IonImageSet records the one it used
    flags_preset_ppm: float | None = None  # a slice's copy set the flags for this ppm (no flag pass needed)
    _sorted: bool | None = None      # spectra_sorted() result
    flag_state: torch.Tensor | None = None  # uint8 mirror of each hit's flag (the flag pass reads it, not the hits)

    @property
    def n_points(self) -> int:
        return int(self.mz.numel())

    @property
    def device(self):
        return self.mz.device

    @classmethod
    def from_arrays(cls, sp_off, mz, ints, pixel_map, dims, device="cuda", stream=None) -> "DevicePeaks":
        require_gpu()
        mz = np.ascontiguousarray(mz, dtype=np.float32)
        if mz.size and not (np.all(mz > 0) and np.all(np.isfinite(mz))):
            raise ValueError("m/z values must be positive and finite")
        d_off = torch.from_numpy(np.ascontiguousarray(sp_off, dtype=np.int64)).to(device)
        d_pix = torch.from_numpy(np.ascontiguousarray(pixel_map, dtype=np.int32)).to(device)
        d_ints = torch.from_numpy(np.ascontiguousarray(ints, dtype=np.float32)).to(device)
        d_mz = torch.from_numpy(mz).to(device)
        hits = torch.empty(mz.shape[0], dtype=torch.int64, device=device)
        check(lib().smg_pack_hits(_p(d_off), _p(d_pix), len(pixel_map), _p(d_ints), mz.shape[0], _p(hits),
                                  _stream(stream)), "smg_pack_hits")
        return cls(mz=d_mz, hits=hits, nrows=int(dims[0]), ncols=int(dims[1]), sp_off=d_off,
                   force=_force_flags(pixel_map, device))

    @classmethod
    def from_device(cls, mz: torch.Tensor, hits: torch.Tensor, dims, sp_off: torch.Tensor,
                    pixel_map=None) -> "DevicePeaks":
        force = _force_flags(pixel_map, mz.device) if pixel_map is not None else None
        return cls(mz=mz, hits=hits, nrows=int(dims[0]), ncols=int(dims[1]), sp_off=sp_off, force=force)

    def flag_duplicates(self, ppm: float, stream=None) -> "DevicePeaks":
        """Duplicate-candidate flags for this ppm (smg_flag_duplicates).  Every call recomputes them from the
        m/z values (12 B read per point), except on a slice whose copy already set them for this ppm."""
        if self.sp_off is None:
            raise ValueError("DevicePeaks needs sp_off (spectrum offsets) for duplicate flags")
        if self.flags_preset_ppm is not None and float(ppm) == self.flags_preset_ppm:
            self.hits_flag_ppm = float(ppm)
            return self
        self.flags_preset_ppm = None
        n_sp = int(self.sp_off.numel()) - 1
        if self.flag_state is None or self.flag_state.numel() != self.n_points:
            # 1 B per point: the flag pass then reads 5 B per point (m/z + state) instead of 12 B, and a hit only
            # where its flag changes
            with torch.cuda.stream(stream) if stream is not None else _nullctx():
                self.flag_state = ((self.hits >> 31) & 1).to(torch.uint8)
        check(lib().smg_flag_duplicates(_p(self.sp_off), n_sp, _p(self.mz), _p(self.hits), self.n_points,
                                        float(ppm), _p(self.force), _p(self.flag_state), _stream(stream)),
              "smg_flag_duplicates")
        self.hits_flag_ppm = float(ppm)
        self.version += 1
        return self

    def spectra_sorted(self) -> bool:
        """Every spectrum's m/z values are nondecreasing (checked once; the m/z array does not change)."""
        if self._sorted is None:
            n = self.n_points
            if n < 2:
                self._sorted = True
            else:
                starts = torch.zeros(n, dtype=torch.bool, device=self.device)
                so = self.sp_off[1:-1]
                starts[so[so < n]] = True
                bad = (self.mz[1:] < self.mz[:-1]) & ~starts[1:]
                self._sorted = not bool(bad.any().item())
        return self._sorted

    def slice_mz(self, lo: float, hi: float, ppm: float, stream=None) -> "DevicePeaks":
        """The points with lo <= mz <= hi (f64 comparison), in dataset order, as a new DevicePeaks whose
        duplicate-candidate flags for ``ppm`` are set by the copy (smg_slice_mz_count / _copy)."""
        if not self.spectra_sorted():
            return self._slice_mz_masked(lo, hi, ppm, stream)
        n_sp = int(self.sp_off.numel()) - 1
        sz = ctypes.c_size_t(0)
        check(lib().smg_slice_mz_workspace_size(n_sp, ctypes.byref(sz)), "smg_slice_mz_workspace_size")
        ws = workspace(sz.value, self.device, "slice")
        off = torch.empty(n_sp + 1, dtype=torch.int64, device=self.device)
        check(lib().smg_slice_mz_count(_p(self.sp_off), n_sp, _p(self.mz), float(lo), float(hi), _p(off), _p(ws),
                                       ws.numel(), _stream(stream)), "smg_slice_mz_count")
        n = int(off[-1].item())
        mz = torch.empty(n, dtype=torch.float32, device=self.device)
        hits = torch.empty(n, dtype=torch.int64, device=self.device)
        if n:
            check(lib().smg_slice_mz_copy(_p(self.sp_off), n_sp, _p(self.mz), _p(self.hits), _p(off), float(ppm),
                                          _p(self.force), _p(mz), _p(hits), _p(ws), _stream(stream)),
                  "smg_slice_mz_copy")
        out = DevicePeaks(mz=mz, hits=hits, nrows=self.nrows, ncols=self.ncols, sp_off=off, force=self.force)
        out.flags_preset_ppm = float(ppm)
        out._sorted = True
        # every value of the slice lies in [lo, hi]: positive f32 bit patterns are ordered like the values, so the
        # bits that vary among them are within those of f32(lo) rounded down and f32(hi) rounded up (no
        # aminmax + synchronisation per slice)
        if n and lo > 0.0:
            a = np.array([lo], np.float32)
            if float(a[0]) > lo:
                a = np.nextafter(a, np.float32(0))
            b = np.array([hi], np.float32)
            if float(b[0]) < hi:
                b = np.nextafter(b, np.float32(np.inf))
            out.sort_key_bits = max(1, (int(a.view(np.int32)[0]) ^ int(b.view(np.int32)[0])).bit_length())
        return out

    def _slice_mz_masked(self, lo: float, hi: float, ppm: float, stream=None) -> "DevicePeaks":
        """slice_mz for datasets with spectra that are not m/z-sorted (the reference accepts them; the flag pass
        flags every point of such a spectrum): a masked copy in dataset order (f64 comparison) and a full flag
        pass over the slice."""
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            m64 = self.mz.to(torch.float64)
            idx = torch.nonzero((m64 >= float(lo)) & (m64 <= float(hi))).flatten()
            del m64
            n_sp = int(self.sp_off.numel()) - 1
            sp = torch.searchsorted(self.sp_off[1:], idx, right=True)
            off = torch.zeros(n_sp + 1, dtype=torch.int64, device=self.device)
            off[1:] = torch.cumsum(torch.bincount(sp, minlength=n_sp)[:n_sp], 0)
            out = DevicePeaks(mz=self.mz[idx], hits=self.hits[idx], nrows=self.nrows, ncols=self.ncols, sp_off=off,
                              force=self.force)
        out.flag_duplicates(ppm, stream)
        out.flags_preset_ppm = float(ppm)
        out._sorted = False
        return out

    def sort(self, stream=None) -> "DevicePeaks":
        """Stable m/z sort of the points (smg_sort_points), flags as the hits carry them: the sorted copy's flags
        are then those of the last flag pass over the hits (flag_ppm None if the hits' flags are stale, e.g. after
        a fused flag_and_sort, which flags only the sorted copy)."""
        self._sort_into(lambda ws: lib().smg_sort_points(
            _p(self.mz), _p(self.hits), self.n_points, self.key_bits(), _p(self.mz_sorted), _p(self.hits_sorted),
            _p(ws), ws.numel(), _stream(stream)), "smg_sort_points", stream)
        self.flag_ppm = self.hits_flag_ppm
        return self

    def _sort_into(self, call, name, stream=None):
        n = self.n_points
        if self.mz_sorted is None or self.mz_sorted.numel() != n:
            self.mz_sorted = torch.empty_like(self.mz)
            self.hits_sorted = torch.empty_like(self.hits)
        self.cum_valid = False
        self.version += 1
        if n == 0:
            return
        sz = ctypes.c_size_t(0)
        check(lib().smg_sort_points_workspace_size(n, ctypes.byref(sz)), "smg_sort_points_workspace_size")
        ws = workspace(sz.value, self.device, "sort")
        check(call(ws), name)

    def flag_and_sort(self, ppm: float, stream=None) -> "DevicePeaks":
        """flag_duplicates(ppm) then sort(), with one pass less: the sort's first pass sets the flags from each
        point's spectrum neighbours (smg_sort_points_flag), the same flags as the flag pass when every spectrum is
        m/z-sorted and no pixel is shared.  Otherwise (and on a slice whose copy set the flags) the separate flag
        pass, then the sort."""
        preset = self.flags_preset_ppm is not None and float(ppm) == self.flags_preset_ppm
        if self.sp_off is None or self.force is not None or preset or not self.spectra_sorted():
            self.flag_duplicates(ppm, stream)
            return self.sort(stream)
        n_sp = int(self.sp_off.numel()) - 1
        self._sort_into(lambda ws: lib().smg_sort_points_flag(
            _p(self.sp_off), n_sp, _p(self.mz), _p(self.hits), self.n_points, self.key_bits(), float(ppm),
            _p(self.mz_sorted), _p(self.hits_sorted), _p(ws), ws.numel(), _stream(stream)), "smg_sort_points_flag",
            stream)
        self.flag_ppm = float(ppm)  # the sorted copy's flags; the dataset-order hits keep whatever they had
        return self

    def prefix_sums(self, stream=None) -> "DevicePeaks":
        """(sum v, sum v^2 of unflagged points) prefix sums over hits_sorted: window sums for the ion kernel."""
        self.cum = hit_prefix_sums(_lib.SMG_HITS_PACKED_F32, self.hits_sorted, None, self.n_points, self.cum,
                                   stream)
        self.cum_valid = True
        return self

    def sorted_cum(self, stream=None) -> torch.Tensor:
        """Prefix sums of the current sorted hits (recomputed after every sort)."""
        if not self.cum_valid:
            self.prefix_sums(stream)
        return self.cum

    def key_bits(self) -> int:
        """Low bits in which the dataset's f32 m/z bit patterns differ (the sort ignores the common prefix);
        computed once, the m/z array does not change."""
        if self.sort_key_bits is None:
            lo, hi = torch.aminmax(self.mz)
            a = int(lo.view(torch.int32).item())
            b = int(hi.view(torch.int32).item())
            self.sort_key_bits = max(1, (a ^ b).bit_length())
        return self.sort_key_bits


@dataclass
class DeviceIons:
    """Theoretical windows of a batch of ions, ion-major (FormulasSegm.get_sf_peak_df / get_sf_peak_ints).

    ``win_off``: int64[n_ion+1]; ``peak_mz``/``theor``: float64[n_win]; ``win_order``: windows sorted by
    m/z (the reference's sf_peak_df order); ``ion_order``: ions sorted by principal m/z.
    """
    win_off: torch.Tensor
    peak_mz: torch.Tensor
    theor: torch.Tensor
    win_order: torch.Tensor
    ion_order: torch.Tensor
    n_ions: int
    n_windows: int
    max_k: int

    @classmethod
    def from_arrays(cls, win_off, peak_mz, theor, device="cuda") -> "DeviceIons":
        win_off = np.ascontiguousarray(win_off, dtype=np.int64)
        peak_mz = np.ascontiguousarray(peak_mz, dtype=np.float64)
        theor = np.ascontiguousarray(theor, dtype=np.float64)
        n_ions = len(win_off) - 1
        K = np.diff(win_off)
        if n_ions and K.max(initial=0) > 32:
            raise ValueError("at most 32 theoretical peaks per ion are supported")
        win_order = np.argsort(peak_mz, kind="stable").astype(np.int64)
        first = np.full(n_ions, np.inf)
        nz = K > 0
        first[nz] = peak_mz[win_off[:-1][nz]]
        ion_order = np.argsort(first, kind="stable").astype(np.int64)
        t = lambda a: torch.from_numpy(a).to(device)
        return cls(win_off=t(win_off), peak_mz=t(peak_mz), theor=t(theor), win_order=t(win_order),
                   ion_order=t(ion_order), n_ions=n_ions, n_windows=int(win_off[-1]) if n_ions else 0,
                   max_k=int(K.max(initial=0)))


def window_bounds(peaks: DevicePeaks, ions: DeviceIons, ppm: float, stream=None):
    """searchsorted of formula_imager_segm.py:79-82 for every window -> (lo, hi) int64 device tensors."""
    assert peaks.mz_sorted is not None, "call peaks.sort() first"
    lo = torch.empty(ions.n_windows, dtype=torch.int64, device=peaks.device)
    hi = torch.empty_like(lo)
    check(lib().smg_window_bounds(_p(ions.peak_mz), _p(ions.win_order), ions.n_windows, float(ppm),
                                  _p(peaks.mz_sorted), peaks.n_points, _p(lo), _p(hi), _stream(stream)),
          "smg_window_bounds")
    return lo, hi


@dataclass
class IonMetrics:
    chaos: torch.Tensor
    spatial: torch.Tensor
    spectral: torch.Tensor
    msm: torch.Tensor
    flags: torch.Tensor

    def to_numpy(self):
        return {k: getattr(self, k).cpu().numpy() for k in ("chaos", "spatial", "spectral", "msm", "flags")}


def hit_prefix_sums(hit_format: int, hits: torch.Tensor, hit_vals, n_points: int, out=None, stream=None):
    device = hits.device
    nb = (n_points + 63) // 64 + 1
    if out is None or out.shape[0] != nb:
        out = torch.empty(nb, 4, dtype=torch.float64, device=device)  # double-double (sum, sum of squares)
    sz = ctypes.c_size_t(0)
    check(lib().smg_hit_prefix_sums_workspace_size(n_points, ctypes.byref(sz)), "smg_hit_prefix_sums_workspace_size")
    ws = workspace(sz.value, device, "scan")
    check(lib().smg_hit_prefix_sums(hit_format, _p(hits), _p(hit_vals), n_points, _p(out), _p(ws), ws.numel(),
                                    _stream(stream)), "smg_hit_prefix_sums")
    return out


def ion_metrics_raw(hit_format: int, hits: torch.Tensor, hit_vals, hit_cum, lo, hi, win_off, theor, ion_order,
                    n_ions: int, nrows: int, ncols: int, nlevels: int = 30, q: float = 99.0,
                    do_preprocessing: bool = False, connectivity: int = 4, erosion_border: int = 0,
                    out: IonMetrics | None = None, stream=None) -> IonMetrics:
    device = lo.device
    if out is None:
        f64 = lambda: torch.empty(n_ions, dtype=torch.float64, device=device)
        out = IonMetrics(f64(), f64(), f64(), f64(), torch.empty(n_ions, dtype=torch.int32, device=device))
    if n_ions == 0:
        return out
    if hits.numel() == 0:  # no data points: every window is empty, no ion is scored (formula_img_validator.py:115-118)
        for t in (out.chaos, out.spatial, out.spectral, out.msm, out.flags):
            t.zero_()
        return out
    sz = ctypes.c_size_t(0)
    check(lib().smg_ion_metrics_workspace_size(n_ions, nrows, ncols, ctypes.byref(sz)),
          "smg_ion_metrics_workspace_size")
    ws = workspace(sz.value, device, "metrics")
    if _lib.check_build():  # the diagnostic build checks every hit index against the resident count
        check(lib().smg_debug_check_points(int(hits.numel())), "smg_debug_check_points")
    check(lib().smg_ion_metrics(hit_format, _p(hits), _p(hit_vals), _p(hit_cum), _p(lo), _p(hi), _p(win_off),
                                _p(theor),
                                _p(ion_order), n_ions, nrows, ncols, nlevels, float(q), int(bool(do_preprocessing)),
                                connectivity, erosion_border, _p(out.chaos), _p(out.spatial), _p(out.spectral),
                                _p(out.msm), _p(out.flags), _p(ws), ws.numel(), _stream(stream)),
          "smg_ion_metrics")
    return out


def ion_metrics(peaks: DevicePeaks, ions: DeviceIons, lo, hi, nlevels=30, q=99.0, do_preprocessing=False,
                connectivity=4, erosion_border=0, out=None, stream=None) -> IonMetrics:
    """Fused imaging + MSM scoring of every ion (one launch for the LDS path, one for the dense path)."""
    return ion_metrics_raw(_lib.SMG_HITS_PACKED_F32, peaks.hits_sorted, None, peaks.sorted_cum(stream), lo, hi,
                           ions.win_off,
                           ions.theor,
                           ions.ion_order, ions.n_ions, peaks.nrows, peaks.ncols, nlevels, q, do_preprocessing,
                           connectivity, erosion_border, out, stream)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _force_flags(pixel_map, device):
    """uint8 per spectrum: 1 where the pixel is shared by several spectra (reference tolerates duplicate
    coordinates with a warning, imzml_txt_converter.py:95-100); None when the map is injective."""
    pm = np.asarray(pixel_map)
    uniq, inv, cnt = np.unique(pm, return_inverse=True, return_counts=True)
    shared = cnt[inv] > 1
    if not shared.any():
        return None
    return torch.from_numpy(shared.astype(np.uint8)).to(device)


def run_hot_path(peaks: DevicePeaks, ions: DeviceIons, ppm: float, nlevels: int = 30, **kw):
    """One full pass: duplicate flags -> sort -> window search -> fused metrics (all on the current stream)."""
    peaks.flag_and_sort(ppm)
    peaks.prefix_sums()
    lo, hi = window_bounds(peaks, ions, ppm)
    return ion_metrics(peaks, ions, lo, hi, nlevels=nlevels, **kw), lo, hi


def metrics_from_images(ion_images, nrows, ncols, nlevels=30, q=99.0, do_preprocessing=False, connectivity=4,
                        erosion_border=0, device="cuda"):
    """Score explicit sparse images (the generic ``compute(iso_images_sparse, sf_ints)`` path).

    ``ion_images``: iterable of ``(imgs, sf_ints)``; ``imgs`` is a list of scipy sparse matrices or None,
    padded to len(sf_ints) as formula_img_validator.py:73-75 does.  Values keep float64.
    Returns numpy arrays (chaos, spatial, spectral, msm, flags).
    """
    require_gpu()
    pix_l, val_l, lo_l, hi_l, th_l, off = [], [], [], [], [], [0]
    pos = 0
    for imgs, sf_ints in ion_images:
        imgs = list(imgs) + [None] * (len(sf_ints) - len(imgs))
        for img, t in zip(imgs, sf_ints):
            lo_l.append(pos)
            if img is not None:
                c = img.tocoo()
                p = (c.row.astype(np.int64) * ncols + c.col.astype(np.int64))
                # duplicate pixels of this image carry the duplicate-candidate flag (bit 31)
                _, inv, cnt = np.unique(p, return_inverse=True, return_counts=True)
                p = np.where(cnt[inv] > 1, p | 0x80000000, p)
                pix_l.append(p.astype(np.uint32))
                val_l.append(c.data.astype(np.float64))
                pos += p.shape[0]
            hi_l.append(pos)
            th_l.append(float(t))
        off.append(len(lo_l))
    n_ions = len(off) - 1
    if n_ions == 0:
        return {k: np.zeros(0) for k in ("chaos", "spatial", "spectral", "msm", "flags")}
    pix = np.concatenate(pix_l) if pix_l else np.zeros(1, np.uint32)
    val = np.concatenate(val_l) if val_l else np.zeros(1, np.float64)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(device)
    d_pix = t(pix.view(np.int32), np.int32)
    d_val = t(val, np.float64)
    cum = hit_prefix_sums(_lib.SMG_HITS_SPLIT_F64, d_pix, d_val, pos)
    res = ion_metrics_raw(_lib.SMG_HITS_SPLIT_F64, d_pix, d_val, cum, t(lo_l, np.int64), t(hi_l, np.int64),
                          t(off, np.int64), t(th_l, np.float64), None, n_ions, nrows, ncols, nlevels, q,
                          do_preprocessing, connectivity, erosion_border)
    torch.cuda.synchronize()
    return res.to_numpy()
