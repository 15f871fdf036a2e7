"""Diagnostic: does a libsmg HIP call work when it is the first HIP call of the process (before torch's lazy
CUDA init)?  usage: diag_init_order.py [torch_first]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from sm_distributed_amd import _lib
if len(sys.argv) > 1:
    torch.cuda.init()
    print("torch initialised first", flush=True)
L = _lib.lib()
sz = ctypes.c_size_t(0)
rc = L.smg_hit_prefix_sums_workspace_size(1000, ctypes.byref(sz))
print("libsmg first call rc", rc, L.smg_last_error().decode(), flush=True)
x = torch.ones(4, device="cuda")
print("torch tensor ok", float(x.sum()), flush=True)
rc = L.smg_hit_prefix_sums_workspace_size(1000, ctypes.byref(sz))
print("libsmg second call rc", rc, L.smg_last_error().decode(), flush=True)
