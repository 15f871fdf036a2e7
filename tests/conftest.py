import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libsmg.so")


def pytest_sessionfinish(session, exitstatus):
    """With the -DSMG_CHECK diagnostic library loaded (SMG_LIB=.../libsmg_check.so), report its counters for the whole
    session (SMG_CHECK_OUT: also into that file) and fail the session if any check failed."""
    mod = sys.modules.get("sm_distributed_amd._lib")
    if mod is None or mod._lib is None or not mod.check_build():
        return
    try:
        c = mod.check_counters()
    except Exception as e:  # a device fault earlier in the session: report it, keep the test reports
        print(f"\nSMG_CHECK counters unreadable: {e}")
        session.exitstatus = 1
        return
    bad = {k: v for k, v in c.items() if k not in ("positions_claimed", "descriptors_checked") and v}
    line = f"SMG_CHECK counters over the session: {c}"
    print("\n" + line)
    out = os.environ.get("SMG_CHECK_OUT")
    if out:
        with open(out, "a") as fh:
            fh.write(line + "\n")
    if bad:
        session.exitstatus = 1
