"""KFD's queue-eviction counter of this process, and an opt-out from one trigger of evictions.

KFD evicts all of a process's GPU queues -- every running kernel stops until they are restored -- when an MMU
notifier invalidates a userptr range of the process (host memory the GPU maps) or when TTM evicts one of its
buffers.  A userptr restore is scheduled one millisecond later, i.e. at the next scheduler tick (10 ms at
HZ = 100), so a 31-ms kernel takes 41, 51 or 61 ms: the step-time outliers of rounds 3-5
(profiles/round5/r5ol*: ``evicted_ms`` grows in 10-ms steps exactly when the main pass does, the short descriptor
pass never stretches, and the shader clock falls only while the GPU sits idle in the evictions).

``EvictionCounter`` reads /sys/class/kfd/kfd/proc/<pid>/stats_<gpu_id>/evicted_ms, so that bench.py can put each
step's eviction time in its line.  ``numa_balancing_optout()`` takes the process out of NUMA-balancing scans (a
trigger where the kernel has numa_balancing = 1; the pool's boxes have it off): the scanner skips a memory area
unless its policy -- the area's own, else the scanning thread's -- carries MPOL_F_MOF (mm/mempolicy.c,
vma_policy_mof), and an explicit MPOL_LOCAL task policy does not.  Threads inherit the policy at creation, so it
must run before the process starts its threads.
"""
from __future__ import annotations

import ctypes
import glob
import os

_MPOL_LOCAL = 4
_SYS_SET_MEMPOLICY = {"x86_64": 238, "aarch64": 237}
_KFD_PROC = "/sys/class/kfd/kfd/proc"
_KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
_done = None


def numa_balancing_optout() -> bool:
    """Set this thread's memory policy to MPOL_LOCAL (no MPOL_F_MOF: NUMA-balancing scans skip the process's
    memory).  Once per process.  True when the policy is set."""
    global _done
    if _done is not None:
        return _done
    _done = False
    nr = _SYS_SET_MEMPOLICY.get(os.uname().machine)
    if nr is None:
        return False
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        _done = libc.syscall(ctypes.c_long(nr), ctypes.c_int(_MPOL_LOCAL), ctypes.c_void_p(None),
                             ctypes.c_ulong(0)) == 0
    except (OSError, AttributeError):
        _done = False
    return _done


def numa_balancing_enabled():
    """The kernel's automatic NUMA balancing switch (/proc/sys/kernel/numa_balancing), None if unreadable."""
    try:
        with open("/proc/sys/kernel/numa_balancing") as fh:
            return int(fh.read().strip())
    except (OSError, ValueError):
        return None


def kfd_gpu_id(pci_bus: int):
    """KFD's gpu_id of the GPU on PCI bus ``pci_bus`` (topology node location_id = bus << 8 | device << 3 | fn)."""
    for d in glob.glob(os.path.join(_KFD_NODES, "*")):
        try:
            with open(os.path.join(d, "gpu_id")) as fh:
                gid = fh.read().strip()
            with open(os.path.join(d, "properties")) as fh:
                props = dict(ln.split() for ln in fh if len(ln.split()) == 2)
        except OSError:
            continue
        if gid != "0" and (int(props.get("location_id", "-1")) >> 8) & 0xFF == pci_bus:
            return gid
    return None


class EvictionCounter:
    """KFD's evicted_ms of this process on one GPU (/sys/class/kfd/kfd/proc/<pid>/stats_<gpu_id>/evicted_ms).
    The directory is named by the host's pid, which a container does not see, so it is found as the one process
    with queues on that GPU; ``read()`` is None when that is ambiguous or unreadable."""

    def __init__(self, gpu_id):
        self.path = None
        if gpu_id is None:
            return
        hits = []
        for d in glob.glob(os.path.join(_KFD_PROC, "*")):
            qs = glob.glob(os.path.join(d, "queues", "*", "gpuid"))
            try:
                on = any(open(q).read().strip() == gpu_id for q in qs)
            except OSError:
                continue
            if on:
                hits.append(os.path.join(d, f"stats_{gpu_id}", "evicted_ms"))
        if len(hits) == 1:
            self.path = hits[0]

    def read(self):
        if self.path is None:
            return None
        try:
            with open(self.path) as fh:
                return int(fh.read().strip())
        except (OSError, ValueError):
            return None
