"""ctypes binding of libsmg.so (declared in include/smg.h).

The product path has no CPU fallback: if the shared library is missing or cannot be loaded,
``lib()`` raises ``SmgLibraryError`` and every device entry point fails loudly.
"""
from __future__ import annotations

import ctypes
import os

# SMG_LIB overrides the path (diagnostic builds of the same C-ABI, e.g. scripts/build_sparse_variant.sh)
LIB_PATH = os.environ.get("SMG_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsmg.so")

SMG_OK = 0
SMG_ION_HAS_HITS = 0x1
SMG_ION_DENSE = 0x2
SMG_ION_CHAOS_NAN = 0x4
SMG_ION_BIG = 0x8
SMG_ION_TWO_LEVEL = 0x10
SMG_ION_WIDE = 0x20
SMG_ION_SPARSE = 0x40
SMG_HITS_PACKED_F32 = 0
PIXEL_MASK = 0x7FFFFFFF   # bit 31 of the pixel field = duplicate-candidate flag
SMG_HITS_SPLIT_F64 = 1
# pass ids of smg_debug_pass_times
SMG_PASS_DESC, SMG_PASS_MAIN, SMG_PASS_BIG, SMG_PASS_WIDE, SMG_PASS_DENSE, SMG_PASS_FINALIZE = range(6)
PASS_NAMES = {0: "ion_desc8_kernel", 1: "ion_sparse_kernel (main LDS pass)",
              2: "ion_pipe_kernel<1024> (big-ion LDS pass)", 3: "ion_wide_join_kernel (wide pass; ion_wide_kernel with the clip)",
              4: "ion_dense_kernel (pixel-indexed pass)", 5: "ion_finalize_kernel (LDS passes' scores)"}

# every symbol include/smg.h declares, with its ctypes prototype
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_D = ctypes.c_double
_SZ = ctypes.c_size_t
PROTOTYPES = {
    "smg_version": (ctypes.c_char_p, []),
    "smg_last_error": (ctypes.c_char_p, []),
    "smg_pack_hits": (ctypes.c_int, [_P, _P, _I64, _P, _I64, _P, _P]),
    "smg_flag_duplicates": (ctypes.c_int, [_P, _I64, _P, _P, _I64, _D, _P, _P, _P]),
    "smg_sort_points_workspace_size": (ctypes.c_int, [_I64, ctypes.POINTER(_SZ)]),
    "smg_sort_points": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _P, _SZ, _P]),
    "smg_sort_points_flag": (ctypes.c_int, [_P, _I64, _P, _P, _I64, _I32, _D, _P, _P, _P, _SZ, _P]),
    "smg_window_bounds": (ctypes.c_int, [_P, _P, _I64, _D, _P, _I64, _P, _P, _P]),
    "smg_align_windows": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, _P, _P, _P, _P]),
    "smg_slice_mz_workspace_size": (ctypes.c_int, [_I64, ctypes.POINTER(_SZ)]),
    "smg_slice_mz_count": (ctypes.c_int, [_P, _I64, _P, _D, _D, _P, _P, _SZ, _P]),
    "smg_slice_mz_copy": (ctypes.c_int, [_P, _I64, _P, _P, _P, _D, _P, _P, _P, _P, _P]),
    "smg_ion_metrics_workspace_size": (ctypes.c_int, [_I64, _I32, _I32, ctypes.POINTER(_SZ)]),
    "smg_hit_prefix_sums_workspace_size": (ctypes.c_int, [_I64, ctypes.POINTER(_SZ)]),
    "smg_hit_prefix_sums": (ctypes.c_int, [_I32, _P, _P, _I64, _P, _P, _SZ, _P]),
    "smg_ion_metrics": (ctypes.c_int, [_I32, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I32, _I32, _I32, _D, _I32,
                                       _I32, _I32, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "smg_iso_image_rows_workspace_size": (ctypes.c_int, [_I64, _I64, ctypes.POINTER(_SZ)]),
    "smg_iso_image_rows": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _D, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "smg_sample_spectra": (ctypes.c_int, [_P, _P, _P, _I64, _P, _P, _I64, _P, _P, _P, _I64, _P, _P]),
    "smg_debug_stream_read": (ctypes.c_int, [_P, _I64, _P, _I32, _P]),
    "smg_debug_force_two_level": (ctypes.c_int, [_I32]),
    "smg_debug_force_dense": (ctypes.c_int, [_I32]),
    "smg_debug_sort_impl": (ctypes.c_int, [_I32]),
    "smg_debug_main_kernel": (ctypes.c_int, [_I32]),
    "smg_debug_wide_impl": (ctypes.c_int, [_I32]),
    "smg_debug_stamps": (ctypes.c_int, [_P, ctypes.c_int]),
    "smg_debug_sparse_stamps": (ctypes.c_int, [_P, ctypes.c_int]),
    "smg_debug_check_points": (ctypes.c_int, [_I64]),
    "smg_debug_check_read": (ctypes.c_int, [_P, _I32]),
    "smg_debug_time_main_pass": (ctypes.c_int, [_I32]),
    "smg_debug_main_pass_times": (ctypes.c_int, [_P, _I32, ctypes.POINTER(_I32)]),
    "smg_debug_pass_times": (ctypes.c_int, [_P, _P, _I32, ctypes.POINTER(_I32)]),
    "smg_isotope_centroids": (ctypes.c_int, [ctypes.c_char_p, _I32, _D, _I32, _I32, _I32, _P, _P,
                                             ctypes.POINTER(_I32)]),
    "smg_isotope_centroids_batch": (ctypes.c_int, [_P, _P, _I64, _I32, _D, _I32, _I32, _I32, _P, _P, _P, _I32]),
}


class SmgLibraryError(ImportError):
    pass


class SmgError(RuntimeError):
    pass


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SmgLibraryError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback for the device path)")
        try:
            handle = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the machine
            raise SmgLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int, what: str = "smg call"):
    if rc != SMG_OK:
        msg = lib().smg_last_error().decode(errors="replace")
        raise SmgError(f"{what} failed with status {rc}: {msg}")


def version() -> str:
    return lib().smg_version().decode()


CHECK_NAMES = ("positions_claimed", "descriptor_mismatches", "loads_outside_window", "double_hand_outs",
               "records_read_as_descriptors", "reject_list_overflows", "windows_out_of_range", "descriptors_checked")
_check_build = None


def check_build() -> bool:
    """True when the loaded library is the -DSMG_CHECK diagnostic build (libsmg_check.so)."""
    global _check_build
    if _check_build is None:
        buf = (ctypes.c_ulonglong * 8)()
        _check_build = lib().smg_debug_check_read(ctypes.cast(buf, ctypes.c_void_p), 0) == SMG_OK
    return _check_build


def check_counters() -> dict:
    """The check build's counters since the last read (smg_debug_check_read), by name; reset on read."""
    buf = (ctypes.c_ulonglong * 8)()
    check(lib().smg_debug_check_read(ctypes.cast(buf, ctypes.c_void_p), 8), "smg_debug_check_read")
    return dict(zip(CHECK_NAMES, (int(x) for x in buf)))
