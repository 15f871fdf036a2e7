"""Host-side diagnostics of KFD queue evictions (sm_distributed_amd/hostmem.py): CPU tests of the sysfs readers
and the memory-policy call (the step-time outlier analysis)."""
import os
import subprocess
import sys

from sm_distributed_amd import hostmem


def test_eviction_counter_without_a_gpu_reads_none():
    c = hostmem.EvictionCounter(None)
    assert c.path is None and c.read() is None
    # a gpu id no KFD node has: no process dir matches
    assert hostmem.EvictionCounter("no-such-gpu").read() is None


def test_kfd_gpu_id_of_an_absent_bus_is_none():
    assert hostmem.kfd_gpu_id(0x1FF) is None


def test_numa_balancing_switch_reads_as_int_or_none():
    v = hostmem.numa_balancing_enabled()
    assert v is None or isinstance(v, int)


def test_numa_optout_sets_a_local_policy_in_a_fresh_process():
    # in a child, so that this test process keeps its default policy; /proc/self/status shows the policy's effect
    # only through numa_maps, so the check is the syscall's success where the kernel has NUMA support
    code = ("import sys; sys.path.insert(0, %r); from sm_distributed_amd import hostmem; "
            "r = hostmem.numa_balancing_optout(); assert hostmem.numa_balancing_optout() is r; print(r)"
            % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() in ("True", "False")
