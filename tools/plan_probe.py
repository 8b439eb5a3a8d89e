"""Print the device's CU count (torch and HIP) and the blocked-kernel plan the library picks for N = 24."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.ops import native
lib = native.require()
p = torch.cuda.get_device_properties(0)
print("torch:", p.name, "CUs", p.multi_processor_count, flush=True)
k, L = ctypes.c_int(0), ctypes.c_int(0)
W = lib.gadmm_chain_blocked_plan(24, 50, 0, ctypes.byref(k), ctypes.byref(L))
print("plan before any tensor:", W, k.value, L.value, flush=True)
x = torch.zeros(4, device="cuda")
W = lib.gadmm_chain_blocked_plan(24, 50, 0, ctypes.byref(k), ctypes.byref(L))
print("plan after a tensor:", W, k.value, L.value, flush=True)
