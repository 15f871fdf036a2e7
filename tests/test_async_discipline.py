"""The inline-asm prefetch loads obey their discipline in the generated gfx950 ISA: no instruction touches a
register with a load in flight before its counted wait, on any control-flow path, and no such register is spilled
(scripts/check_async_regs.py).  CPU-only: compiles the kernels to assembly.

* ion_wide_kernel, ion_wide_join_kernel and the big-ion pass (ion_pipe_kernel<1024>) use compiler-tracked loads
  only: no asynchronous load at all.
* the main pass (ion_pipe_kernel<512>) keeps its asynchronous loads: zero violations.  Its two
  wave-0 loads (scheduling ticket, ion descriptor; tagged "smg:wave0") are waited by wave 0 only; paths that skip
  that wait through an exec-zero branch (the other waves, which issued no such load) are reported as guarded, and
  only for tagged loads -- an untagged load, or a tagged one whose wait is skipped on a path without an exec-zero
  branch, is a violation."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _check(asm, kern):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_async_regs.py"), asm, kern],
                       capture_output=True, text=True)
    last = r.stdout.strip().split("\n")[-1]
    parts = last.replace(",", "").split()
    n_loads, n_bad, n_guarded = int(parts[0]), int(parts[4]), int(parts[6])
    return n_loads, n_bad, n_guarded, r.stdout


@pytest.mark.timeout(600)
def test_async_load_registers_are_never_touched_in_flight(tmp_path):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "sm_distributed_amd", "csrc", "smg_metrics.hip")
    asm = str(tmp_path / "smg_metrics.s")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
                    "-S", src, "-o", asm], check=True, capture_output=True)
    for kern in ("_ZN3smg15ion_wide_kernelILi0E", "_ZN3smg20ion_wide_join_kernel", "_ZN3smg15ion_pipe_kernelILi0ELi1024"):
        n_loads, n_bad, n_guarded, out = _check(asm, kern)
        assert (n_loads, n_bad, n_guarded) == (0, 0, 0), out
    n_loads, n_bad, n_guarded, out = _check(asm, "_ZN3smg15ion_pipe_kernelILi0ELi512")
    assert n_loads > 0 and n_bad == 0, out
    # every guarded report is one of the tagged wave-0 loads, pinned exactly: the ticket atomic and the
    # descriptor load of each of the two 512-thread instantiations, once each -- a new guarded path fails here
    guarded = [l for l in out.split("\n") if l.startswith("GUARDED")]
    assert all("smg:wave0" in l for l in guarded), out
    assert n_guarded == 4, out
    per = {}
    for l in guarded:
        inst, op = l.split()[1], ("atomic" if "global_atomic" in l else "load")
        per[(inst, op)] = per.get((inst, op), 0) + 1
    assert len({k[0] for k in per}) == 2 and all(v == 1 for v in per.values()), out


@pytest.mark.timeout(600)
def test_sparse_main_pass_async_loads(tmp_path):
    """ion_sparse_kernel (smg_sparse.hip) keeps ion_pipe_kernel's asynchronous loads: zero violations, and no path
    that skips a wait (the principal waits dominate every use of those registers; the wave-0 loads are waited where
    every path from them passes)."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "sm_distributed_amd", "csrc", "smg_sparse.hip")
    asm = str(tmp_path / "smg_sparse.s")
    # the flags the library's build gives this file (Makefile SPARSE_FLAGS: its instruction scheduler)
    flags = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sm_distributed_amd", "csrc"), "print-sparse-flags"],
                           check=True, capture_output=True, text=True).stdout.split()
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
                    *flags, "-S", src, "-o", asm], check=True, capture_output=True)
    n_loads, n_bad, n_guarded, out = _check(asm, "_ZN3smg12_GLOBAL__N_117ion_sparse_kernel")
    assert n_loads > 0 and n_bad == 0 and n_guarded == 0, out


def _kernel(tmp_path, lines):
    s = tmp_path / "k.s"
    s.write_text("\n".join(["_ZN3smg4testE:"] + lines + ["s_endpgm", ".size _ZN3smg4testE"]))
    return str(s)


def test_checker_follows_commented_loop_labels(tmp_path):
    """A load whose register is overwritten behind a branch to a label carrying a loop comment is caught."""
    s = _kernel(tmp_path, [";;#ASMSTART", "global_load_dwordx2 v[4:5], v[8:9], off", ";;#ASMEND",
                           "s_branch .LBB0_7", "s_endpgm", ".LBB0_7:                               ;   in Loop: Header=BB0_3 Depth=1",
                           "v_mov_b32_e32 v4, 0"])
    n_loads, n_bad, _, out = _check(s, "_ZN3smg4testE")
    assert n_loads == 1 and n_bad == 1, out


def test_checker_execz_paths(tmp_path):
    """A use reached only by skipping the wait through s_cbranch_execz is guarded for a tagged wave-0 load and a
    violation for an untagged one; a tagged load used on a fall-through path before its wait is a violation."""
    body = ["s_cbranch_execz .LBB0_2", ";;#ASMSTART", "s_waitcnt vmcnt(0)", ";;#ASMEND", ".LBB0_2:",
            "v_mov_b32_e32 v4, 0"]
    for tag, bad, guarded in (("", 1, 0), (" ; smg:wave0", 0, 1)):
        s = _kernel(tmp_path, [";;#ASMSTART", "global_load_dwordx2 v[4:5], v[8:9], off" + tag, ";;#ASMEND"] + body)
        n_loads, n_bad, n_guarded, out = _check(s, "_ZN3smg4testE")
        assert (n_loads, n_bad, n_guarded) == (1, bad, guarded), out
    s = _kernel(tmp_path, [";;#ASMSTART", "global_load_dwordx2 v[4:5], v[8:9], off ; smg:wave0", ";;#ASMEND",
                           "v_mov_b32_e32 v5, 1"] + body)
    n_loads, n_bad, n_guarded, out = _check(s, "_ZN3smg4testE")
    assert (n_loads, n_bad) == (1, 1), out


def test_checker_execnz_fallthrough_is_exec_zero(tmp_path):
    """s_cbranch_execnz jumps to the wave-0 block that waits; its fall-through (exec zero) reaches the use: guarded
    for a tagged load, a violation for an untagged one."""
    body = ["s_cbranch_execnz .LBB0_3", ".LBB0_2:", "v_mov_b32_e32 v4, 0", "s_endpgm", ".LBB0_3:", ";;#ASMSTART",
            "s_waitcnt vmcnt(0)", ";;#ASMEND", "s_branch .LBB0_2"]
    for tag, bad, guarded in (("", 1, 0), (" ; smg:wave0", 0, 1)):
        s = _kernel(tmp_path, [";;#ASMSTART", "global_load_dwordx2 v[4:5], v[8:9], off" + tag, ";;#ASMEND"] + body)
        n_loads, n_bad, n_guarded, out = _check(s, "_ZN3smg4testE")
        assert (n_loads, n_bad, n_guarded) == (1, bad, guarded), out
