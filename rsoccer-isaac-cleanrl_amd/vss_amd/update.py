"""PPO-update helper: the backward of a hidden tanh layer in one HIP pass
(csrc/vss_update.hip, include/vss.h `vss_tanh_grad_bias`).

    gz, db = tanh_grad_bias(gy, y)   # gz = gy * (1 - y^2), db = gz.sum(0)

replaces torch's tanh_backward + the bias-gradient reduction that autograd issues for
nn.Tanh -> nn.Linear (ppo_continuous_action_isaacgym.py:104-111).  On a ROCm device it runs the
HIP kernel (and raises if the library is missing); CPU tensors (the CPU test suite's PPO loop)
take the same formula in torch.
"""
from __future__ import annotations

import torch

from . import _native as N

_COLS = (64, 128, 256, 512, 1024)


def tanh_grad_bias(gy: torch.Tensor, y: torch.Tensor):
    if gy.shape != y.shape or gy.dim() != 2:
        raise ValueError(f"gy {tuple(gy.shape)} and y {tuple(y.shape)} must be the same (rows, cols)")
    if gy.device.type != "cuda":
        gz = gy * (1.0 - y * y)
        return gz, gz.sum(0)
    rows, cols = y.shape
    if cols not in _COLS or gy.dtype != torch.float32 or y.dtype != torch.float32:
        raise ValueError(f"vss_tanh_grad_bias: fp32 with cols in {_COLS}, got {gy.dtype}/{y.dtype} x {cols}")
    lib = N.load()
    if rows == 0:  # empty tensors have no storage to hand over
        return torch.empty_like(y), torch.zeros(cols, device=y.device, dtype=torch.float32)
    gy = gy.contiguous()
    y = y.contiguous()
    gz = torch.empty_like(y)
    partial = torch.empty((lib.vss_tanh_grad_chunks(rows, cols), cols), device=y.device, dtype=torch.float32)
    N.check(lib.vss_tanh_grad_bias(N.stream_of(y.device), rows, cols, gy.data_ptr(), y.data_ptr(), gz.data_ptr(),
                                   partial.data_ptr()), "vss_tanh_grad_bias")
    return gz, partial.sum(0)
