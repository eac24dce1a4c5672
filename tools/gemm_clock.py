#!/usr/bin/env python3
"""Profiling-only: the fused backward GEMM (K = N = 512, 2,097,152 rows) from the product library or
a knob variant (LIB=tools/_build/liblt_<name>.so), REPS launches, for `rocprofv3 --pmc
GRBM_GUI_ACTIVE`: the counter over the kernel's duration gives its average shader clock, to tell
whether an epilogue costs issue slots or clock (power)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import _native as N  # noqa: E402

lib = N.load()
if os.environ.get("LIB"):
    lib = ctypes.CDLL(os.path.join(REPO, os.environ["LIB"]))
    lib.vss_linear_tanh_backward_chunks.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
    lib.vss_linear_tanh_backward_chunks.restype = ctypes.c_int64
    lib.vss_linear_tanh_backward.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32] + \
        [ctypes.c_void_p] * 5
rows, k, n = int(os.environ.get("ROWS", 2097152)), 512, 512
g = torch.Generator(device="cuda").manual_seed(0)
gz = torch.randn(rows, k, device="cuda", generator=g) * 1e-3
w_t = (torch.randn(k, n, device="cuda", generator=g) / k ** 0.5).t().contiguous()
y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g))
out = torch.empty(rows, n, device="cuda")
part = torch.empty(lib.vss_linear_tanh_backward_chunks(rows, k, n), n, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(int(os.environ.get("REPS", 10))):
    lib.vss_linear_tanh_backward(st, rows, k, n, gz.data_ptr(), w_t.data_ptr(), y.data_ptr(), out.data_ptr(),
                                 part.data_ptr())
torch.cuda.synchronize()
print("done")
