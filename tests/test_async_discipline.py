"""The LDS and wide kernels' inline-asm prefetch loads obey their discipline in the generated gfx950 ISA: no
instruction touches a register with a load in flight before its counted wait, on any control-flow path, and
no such register is spilled (scripts/check_async_regs.py).  CPU-only: compiles the kernel to assembly."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_async_load_registers_are_never_touched_in_flight(tmp_path):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    for name, kerns in (("smg_metrics", ("_ZN3smg15ion_pipe_kernelILi0ELi512", "_ZN3smg15ion_pipe_kernelILi0ELi1024",
                                         "_ZN3smg15ion_wide_kernelILi0E")),
                        ("smg_wave", ("_ZN3smg15ion_wave_kernel",))):
        src = os.path.join(ROOT, "sm_distributed_amd", "csrc", name + ".hip")
        asm = str(tmp_path / (name + ".s"))
        extra = ["-fno-strict-aliasing"] if name == "smg_wave" else []  # as the Makefile builds it
        subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only",
                        *extra, "-S", src, "-o", asm], check=True, capture_output=True)
        for kern in kerns:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_async_regs.py"), asm, kern],
                               capture_output=True, text=True)
            assert r.returncode == 0, r.stdout
            assert "0 violations" in r.stdout and not r.stdout.startswith("0 async")
