"""The inline-asm prefetch loads obey their discipline in the generated gfx950 ISA: no instruction touches a
register with a load in flight before its counted wait, on any control-flow path, and no such register is spilled
(scripts/check_async_regs.py).  CPU-only: compiles the kernels to assembly.

* ion_wave_kernel (main pass) and ion_wide_kernel use compiler-tracked loads only: no asynchronous load at all.
* ion_pipe_kernel (the legacy main pass and the big-ion pass) keeps its asynchronous loads.  The path check reports
  two per instantiation that follow a wave-0-only wait (the ticket and descriptor loads are issued by wave 0, the
  other waves skip the wait with an exec-zero branch): the static check cannot see that those paths carry no load.
  Their number is pinned, so a new one fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIPE_KNOWN = 4  # per pipe-kernel prefix (two template instantiations, two wave-0 paths each)


def _check(asm, kern):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_async_regs.py"), asm, kern],
                       capture_output=True, text=True)
    last = r.stdout.strip().split("\n")[-1]
    n_loads, n_bad = int(last.split()[0]), int(last.split(",")[1].split()[0])
    return n_loads, n_bad, r.stdout


@pytest.mark.timeout(600)
def test_async_load_registers_are_never_touched_in_flight(tmp_path):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    asm = {}
    for name in ("smg_metrics", "smg_wave"):
        src = os.path.join(ROOT, "sm_distributed_amd", "csrc", name + ".hip")
        asm[name] = str(tmp_path / (name + ".s"))
        extra = ["-fno-strict-aliasing"] if name == "smg_wave" else []  # as the Makefile builds it
        subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
                        *extra, "-S", src, "-o", asm[name]], check=True, capture_output=True)
    for name, kern in (("smg_wave", "_ZN3smg15ion_wave_kernel"), ("smg_metrics", "_ZN3smg15ion_wide_kernelILi0E")):
        n_loads, n_bad, out = _check(asm[name], kern)
        assert n_bad == 0 and n_loads == 0, out
    for kern in ("_ZN3smg15ion_pipe_kernelILi0ELi512", "_ZN3smg15ion_pipe_kernelILi0ELi1024"):
        n_loads, n_bad, out = _check(asm["smg_metrics"], kern)
        assert n_loads > 0 and n_bad <= PIPE_KNOWN, out


def test_checker_follows_commented_loop_labels(tmp_path):
    """A load whose register is overwritten behind a branch to a label carrying a loop comment is caught."""
    s = tmp_path / "k.s"
    s.write_text("\n".join([
        "_ZN3smg4testE:", ";;#ASMSTART", "global_load_dwordx2 v[4:5], v[8:9], off", ";;#ASMEND",
        "s_branch .LBB0_7", "s_endpgm", ".LBB0_7:                               ;   in Loop: Header=BB0_3 Depth=1",
        "v_mov_b32_e32 v4, 0", "s_endpgm", ".size _ZN3smg4testE"]))
    n_loads, n_bad, out = _check(str(s), "_ZN3smg4testE")
    assert n_loads == 1 and n_bad == 1, out
