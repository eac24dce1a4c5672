"""Workload for rocprofv3 PMC passes over the update's streaming helper kernels (profiling tool):
first_layer_kernel (vss_linear_tanh, 2,097,152 x 52 -> 256) and dtanh_small_k_kernel<4, true>
(vss_output_backward, 2 output columns over 256), five launches each."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd.update import linear_tanh, output_backward  # noqa: E402

rows = 2097152
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randn(rows, 52, device="cuda", generator=g)
w1 = torch.randn(256, 52, device="cuda", generator=g) / 8
b1 = torch.randn(256, device="cuda", generator=g)
go = torch.randn(rows, 2, device="cuda", generator=g)
wo = torch.randn(2, 256, device="cuda", generator=g)
for _ in range(5):
    y = linear_tanh(x, w1, b1)
    gz, db, dw = output_backward(go, wo, y)
torch.cuda.synchronize()
print("bytes/launch algorithmic: first_layer", rows * (52 + 256) * 4, "output_backward", rows * (4 + 2 * 256) * 4)
