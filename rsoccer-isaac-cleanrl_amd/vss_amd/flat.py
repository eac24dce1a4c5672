"""The PPO update's parameters and gradients as flat fp32 buffers (ppo_continuous_action_isaacgym.py:166,
351-354 of the reference: loss.backward(), clip_grad_norm_, optim.Adam).

    flat = FlatGrads(agent, flat_params=True)   # every .grad (and parameter) a view of one buffer
    opt = FlatAdam(flat, lr, eps=1e-5)          # one launch per step, the clip folded in
    flat.zeroed_backward(loss)                  # zero + loss.backward(), MLP gradients written in place
    flat.all_reduce_mean(world)                 # the data-parallel exchange: ONE all-reduce
    flat.clip_norm_(max_norm); opt.step()

The update's MLP backward (vss_amd.mlp._TanhMLP) and the direct minibatch (vss_amd.minibatch) write their
gradients straight into the FlatGrads views (grad_dst) instead of handing them to autograd's accumulation.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from . import _native as N

DIRECT_GRADS = [False]  # set by FlatGrads.zeroed_backward() around the update's loss.backward()


def grad_dst(p: torch.Tensor):
    """The .grad of a FlatGrads-owned parameter, which _TanhMLP's backward writes directly inside
    FlatGrads.zeroed_backward(): the buffer was zeroed just before and each parameter receives exactly
    one gradient per backward, so writing it equals autograd's accumulation into zero -- without one add
    kernel per parameter.  None anywhere else (plain autograd: torch.autograd.grad, other callers)."""
    g = p.grad
    if DIRECT_GRADS[0] and getattr(p, "_vss_flat_grad", False) and g is not None and g.is_cuda \
            and g.dtype == torch.float32:
        return g
    return None


class FlatGrads:
    """All parameter gradients as views of ONE contiguous fp32 buffer, so the data-parallel
    exchange is a single all-reduce (4.3 MB for the SA agent) with no pack/unpack copies.  The MLPs'
    backward (_TanhMLP) writes their gradients straight into these views (grad_dst).  With
    flat_params the parameters themselves become views of one buffer as well (same order), which
    FlatAdam steps in one launch."""

    ALIGN = 64  # floats: every tensor starts 256-B aligned (the HIP entries take 16-B aligned buffers)

    def __init__(self, module: nn.Module, flat_params: bool = False):
        self.params = [p for p in module.parameters() if p.requires_grad]
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off = -(-(off + p.numel()) // self.ALIGN) * self.ALIGN
        dev = self.params[0].device
        # the gaps between tensors stay zero in both buffers (zero gradients leave them unchanged)
        self.flat = torch.zeros(off, device=dev, dtype=torch.float32)
        self.flat_p = torch.zeros(off, device=dev, dtype=torch.float32) if flat_params else None
        self.optimizer = None  # a FlatAdam stepping these buffers (clip_norm_ then defers to it)
        for p, o in zip(self.params, offs):
            p.grad = self.flat[o:o + p.numel()].view_as(p)
            p._vss_flat_grad = True
            if flat_params:
                if p.dtype != torch.float32:
                    raise ValueError("flat_params: fp32 parameters only")
                view = self.flat_p[o:o + p.numel()].view_as(p)
                view.copy_(p.detach())
                p.data = view

    def zero(self):
        self.flat.zero_()

    def zeroed_backward(self, loss: torch.Tensor):
        """zero() then loss.backward() (ppo…:351-352), the MLPs' gradients written in place (grad_dst)."""
        self.zero()
        DIRECT_GRADS[0] = True
        try:
            loss.backward()
        finally:
            DIRECT_GRADS[0] = False

    def all_reduce_mean(self, world: int):
        if world > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
            self.flat.mul_(1.0 / world)

    def clip_norm_(self, max_norm: float) -> torch.Tensor:
        """nn.utils.clip_grad_norm_(agent.parameters(), max_norm) (ppo…:353) on the flat buffer: the L2
        norm of all the gradients (one reduction instead of one per tensor and a norm of the norms), the
        same coefficient max_norm / (norm + 1e-6) clamped to 1, one in-place scale.  Returns the norm.
        With a FlatAdam attached the scale is applied inside its next step() (the norm's partial sums are
        taken here, vss_grad_sq_partials), and the returned tensor is FlatAdam.norm, which holds this norm
        only once that step() has run (before it: the previous step's); read it after optimizer.step()."""
        if self.optimizer is not None:
            return self.optimizer.defer_clip(max_norm)
        total = torch.linalg.vector_norm(self.flat)
        self.flat.mul_(torch.clamp(max_norm / (total + 1e-6), max=1.0))
        return total


class FlatAdam(torch.optim.Optimizer):
    """optim.Adam(agent.parameters(), lr, eps=1e-5) (ppo…:166, step at ppo…:354) over FlatGrads' flat
    parameter and gradient buffers: one launch (vss_adam_step_clipped) per step, which also applies the
    clip_grad_norm_ (ppo…:353) requested through FlatGrads.clip_norm_ just before -- instead of torch's
    norm chain and multi-tensor Adam (~8 launches, ~130 us per minibatch at the reference's 4,095 envs).
    Same update rule, in torch's fused-Adam arithmetic (tests/test_ppo.py); param_groups[0]["lr"] is read
    at every step, so --anneal-lr / --adaptative-lr act on it as on torch's Adam.  A clip to max_norm 0
    zeroes the gradients, as clip_grad_norm_'s does; a step without a clip request does not clip."""

    NO_CLIP = -1.0  # vss_adam_step_clipped's "no clip requested" (max_norm < 0)

    def __init__(self, flat: FlatGrads, lr: float, betas=(0.9, 0.999), eps: float = 1e-5):
        if flat.flat_p is None or not flat.flat.is_cuda:
            raise ValueError("FlatAdam: a FlatGrads with flat_params=True on a ROCm device")
        super().__init__(flat.params, dict(lr=lr, betas=betas, eps=eps))
        self.flat = flat
        flat.optimizer = self
        n = flat.flat.numel()
        self.exp_avg = torch.zeros_like(flat.flat_p)
        self.exp_avg_sq = torch.zeros_like(flat.flat_p)
        self.steps = 0
        self.nparts = int(N.load().vss_grad_sq_partials_count(n))
        self.partial = torch.zeros(self.nparts, device=flat.flat.device)
        self.norm = torch.zeros(1, device=flat.flat.device)
        self._max_norm = self.NO_CLIP

    def zero_grad(self, set_to_none: bool = True):
        """Zero the flat gradient buffer (the .grad tensors are views of it and stay in place)."""
        self.flat.zero()

    def defer_clip(self, max_norm: float) -> torch.Tensor:
        """Take the norm's partial sums of the current gradients now; the next step() applies the clip.
        Returns self.norm, written by that step()."""
        max_norm = float(max_norm)
        if not max_norm >= 0.0:
            raise ValueError(f"FlatAdam: max_norm must be >= 0, got {max_norm}")
        N.check(N.load().vss_grad_sq_partials(N.stream_of(self.flat.flat.device), self.flat.flat.numel(),
                                              self.flat.flat.data_ptr(), self.partial.data_ptr()),
                "vss_grad_sq_partials")
        self._max_norm = max_norm
        return self.norm

    @torch.no_grad()
    def step(self, closure=None):
        if closure is not None:
            raise ValueError("FlatAdam.step: no closure")
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        self.steps += 1
        f = self.flat
        if self._max_norm == self.NO_CLIP:
            # no clip: the norm is not needed, but the kernel reads the partials -- take them for this step
            N.check(N.load().vss_grad_sq_partials(N.stream_of(f.flat.device), f.flat.numel(), f.flat.data_ptr(),
                                                  self.partial.data_ptr()), "vss_grad_sq_partials")
        N.check(N.load().vss_adam_step_clipped(
            N.stream_of(f.flat.device), f.flat.numel(), self.nparts, self.partial.data_ptr(), self._max_norm,
            float(g["lr"]), float(b1), float(b2), float(g["eps"]), self.steps, f.flat.data_ptr(), f.flat_p.data_ptr(),
            self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self.norm.data_ptr()), "vss_adam_step_clipped")
        self._max_norm = self.NO_CLIP  # a clip applies to the step right after it only
