"""libsmg.so loads on CPU and exports every symbol include/smg.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "smg.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(smg_[a-z0-9_]+)\s*\(", hdr)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("smg_version", "smg_last_error", "smg_pack_hits", "smg_sort_points", "smg_window_bounds",
              "smg_ion_metrics", "smg_ion_metrics_workspace_size", "smg_sample_spectra"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from sm_distributed_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libsmg.so is not built: run __graft_entry__.build()")
    h = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(h, s)]
    assert not missing, missing
    assert set(declared_symbols()) == set(_lib.PROTOTYPES)


def test_version_and_argument_errors_without_gpu():
    import sm_distributed_amd
    from sm_distributed_amd import _lib
    L = _lib.lib()
    assert b"gfx950" in L.smg_version()
    assert L.smg_version().decode().startswith(f"smg {sm_distributed_amd.__version__} ")  # one version
    assert L.smg_debug_main_kernel(2) == -1 and L.smg_debug_main_kernel(1) == 0
    assert L.smg_debug_wide_impl(2) == -1 and L.smg_debug_wide_impl(1) == 0
    sz = ctypes.c_size_t(0)
    assert L.smg_ion_metrics_workspace_size(10, 0, 5, ctypes.byref(sz)) == -1  # bad shape -> SMG_ERR_INVALID
    assert b"bad arguments" in L.smg_last_error()
    assert L.smg_ion_metrics_workspace_size(10, 500, 500, ctypes.byref(sz)) == 0 and sz.value > 0
    # invalid nlevels is rejected before any device work
    rc = L.smg_ion_metrics(0, None, None, None, None, None, None, None, None, 5, 10, 10, 0, 99.0, 0, 4, 0,
                           None, None, None, None, None, None, 0, None)
    assert rc == -1 and b"nlevels" in L.smg_last_error()


def test_device_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from sm_distributed_amd import engine
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        engine.require_gpu()
