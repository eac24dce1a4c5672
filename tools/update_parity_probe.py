#!/usr/bin/env python3
"""Profiling-only: where the update's gradient error against fp64 comes from, per parameter, on the rollout rows of
tests/test_update_parity.py (MB minibatch rows, default 2,097,152): the direct minibatch with the fused loss and
without, the autograd path on the same x6 GEMMs (minibatch_losses + FlatGrads.zeroed_backward) and torch's plain
fp32 autograd, each as the relative error of every parameter's gradient against fp64 autograd of the reference's
expressions."""
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from vss_amd.minibatch import disable_graph_packet_capture  # noqa: E402

disable_graph_packet_capture()
import torch  # noqa: E402

import test_update_parity as T  # noqa: E402
from test_ppo import _args  # noqa: E402
from vss_amd import minibatch as MB  # noqa: E402
from vss_amd.flat import FlatGrads  # noqa: E402


def main():
    mb = int(os.environ.get("MB", "2097152"))
    agent0, *data = T.make_rollout_rows()
    x, act, lp, adv, ret, val = data
    inds = torch.randperm(x.shape[0], device="cuda", generator=torch.Generator(device="cuda").manual_seed(mb))[:mb]
    args = _args(norm_adv=True, **T.COEF)
    names = [n for n, _ in agent0.named_parameters()]
    res = {}
    for label, fused in (("direct_fused", True), ("direct_separate", False)):
        MB.FUSED_LOSS = fused
        agent = copy.deepcopy(agent0)
        flat = FlatGrads(agent)
        pad = MB.padding_rows(mb, "cuda")
        rows = MB.DirectRows(mb, mb + pad, 52, 2, "cuda")
        src = rows.gather(inds, x, act, lp, adv, ret, val, True)
        MB.direct_minibatch(agent, args, rows.obs, rows.act, rows.logp, rows.adv, *src, rows.ret, rows.val)
        res[label] = [p.grad.double().clone() for p in agent.parameters()]
        del rows, flat, agent
    agent = copy.deepcopy(agent0)
    flat = FlatGrads(agent)
    a = adv[inds]
    a = (a - a.mean()) / (a.std() + 1e-8)
    pad = MB.padding_rows(mb, "cuda")
    ip = torch.cat([inds, inds[:pad]]) if pad else inds
    loss, _ = MB.minibatch_losses(agent, args, x[ip], act[ip], lp[inds], a, ret[inds], val[inds])
    flat.zeroed_backward(loss)
    res["autograd_x6"] = [p.grad.double().clone() for p in agent.parameters()]
    del agent, flat, loss
    torch.cuda.empty_cache()
    _, res["torch_fp32"] = T._reference_grads(agent0, data, inds, torch.float32)
    _, g64 = T._reference_grads(agent0, data, inds, torch.float64)
    cat = lambda gs: torch.cat([t.reshape(-1) for t in gs])  # noqa: E731
    out = {"mb": mb, "overall": {k: T._rel(cat(v), cat(g64)) for k, v in res.items()}, "per_parameter": {}}
    for i, n in enumerate(names):
        out["per_parameter"][n] = {k: T._rel(v[i], g64[i]) for k, v in res.items()}
        out["per_parameter"][n]["norm_share"] = float(g64[i].norm() / cat(g64).norm())
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
