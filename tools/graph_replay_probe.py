#!/usr/bin/env python3
"""Debug-only: does a captured HIP graph give the same bits on every replay of the SAME inputs?

The update's captured minibatch (MinibatchGraph) went wrong from its 9th replay with ROCm's graph
packet capture on (DEBUG_CLR_GRAPH_PACKET_CAPTURE unset / 1; profiles/r03w_graph_probe2.log).  Here
nothing changes between replays (no optimizer step, same gathered rows), so every replay must equal
the first bit for bit; the first replay that does not, and which outputs differ, locate the defect.
Stages (STAGES, comma separated), each captured and replayed REPLAYS times:

  kernel    one call of each x6 entry point (forward 512->512, forward+output layer, backward,
            weight gradient) on static buffers
  mlp       the actor MLP's forward + backward (_TanhMLP, or torch's nn.Sequential for PATH=torch)
  minibatch MinibatchGraph's body (forward, losses, backward into FlatGrads)

PATH_MLP selects the update's MLP arithmetic: x6 (default product), fp32 (VSS_UPDATE_GEMM=fp32), split
(VSS_UPDATE_MLP=split: hipBLASLt + vss_tanh_grad_bias; needs tools/ab_switches_r04.patch applied), torch (plain nn.Sequential); LOSS selects the
minibatch loss: fused (vss_ppo_loss, default) or torch (the reference's expressions).  PATH_MLP=torch
LOSS=torch puts no kernel of this repository in the graph.  Set DEBUG_CLR_GRAPH_PACKET_CAPTURE on the
command line.  NOISE > 0 launches that many tiny eager kernels after each replay; stage ppo runs the
original failure's setting (ppo_update, 8 epochs x 2 minibatches, captured vs eager)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
PATH = os.environ.get("PATH_MLP", "x6")
if PATH == "fp32":
    os.environ["VSS_UPDATE_GEMM"] = "fp32"
if PATH == "split":  # retired from the product in round 5: apply tools/ab_switches_r04.patch first
    os.environ["VSS_UPDATE_MLP"] = "split"
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402
from vss_amd import minibatch as MBM, mlp as MLP  # noqa: E402
from envs._gym import Box  # noqa: E402
from vss_amd import update as U  # noqa: E402

if PATH == "torch":
    MLP.mlp_forward = lambda seq, x: seq(x)
# LOSS=torch: the minibatch loss as the reference's torch expressions and their autograd (~100 small
# kernels; what the update ran before vss_ppo_loss) instead of the fused HIP loss
LOSS = os.environ.get("LOSS", "fused")
if LOSS == "torch":
    from vss_amd.loss import reference_loss
    MBM.ppo_loss = reference_loss

R = int(os.environ.get("REPLAYS", 16))
MB = int(os.environ.get("MB", 2097152))


def agent():
    from collections import namedtuple
    Env = namedtuple("Env", ["single_observation_space", "single_action_space"])
    torch.manual_seed(42)
    return P.Agent(Env(Box(-np.inf, np.inf, (52,)), Box(-1.0, 1.0, (2,)))).cuda()


NOISE = int(os.environ.get("NOISE", 0))  # eager launches between replays (tiny kernels)


def replay_check(name, capture_fn, outputs_fn):
    """capture_fn() is run once eagerly (warm-up), then captured; the graph is replayed R times and
    every replay's outputs are compared bitwise with the first replay's (and with the eager run's).
    With NOISE > 0, that many tiny eager kernels are launched after each replay (what the PPO loop's
    gathers, normalisation, clipping and Adam step do between two minibatches)."""
    eager = [t.clone() for t in outputs_fn(capture_fn())]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        res = capture_fn()
    outs = outputs_fn(res)
    first, bad = None, []
    scratch = torch.zeros(64, device="cuda")
    for r in range(1, R + 1):
        g.replay()
        for _ in range(NOISE):
            scratch.add_(1.0)
        torch.cuda.synchronize()
        cur = [t.clone() for t in outs]
        if first is None:
            first = cur
            d_eager = max((a.float() - b.float()).abs().max().item() for a, b in zip(eager, cur))
            continue
        diffs = [i for i, (a, b) in enumerate(zip(first, cur)) if not torch.equal(a, b)]
        if diffs:
            bad.append((r, diffs, max((first[i].float() - cur[i].float()).abs().max().item() for i in diffs)))
    verdict = "STABLE" if not bad else f"DIFFERS from replay {bad[0][0]} (outputs {bad[0][1]}, max |diff| {bad[0][2]:.3e})"
    print(f"[{name}] {R} replays: {verdict}; replay 1 vs eager max |diff| {d_eager:.3e}", flush=True)
    if bad:
        print(f"[{name}]   differing replays: {[b[0] for b in bad]}", flush=True)
    del g
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return not bad


def stage_kernel():
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.tanh(torch.randn(MB, 512, device="cuda", generator=g))
    w = torch.randn(512, 512, device="cuda", generator=g) / 512 ** 0.5
    b = torch.randn(512, device="cuda", generator=g) * 0.1
    w4 = torch.randn(256, 512, device="cuda", generator=g) / 512 ** 0.5
    b4 = torch.randn(256, device="cuda", generator=g) * 0.1
    wo = torch.randn(2, 256, device="cuda", generator=g) * 0.01
    bo = torch.zeros(2, device="cuda")
    gz = torch.randn(MB, 512, device="cuda", generator=g) * 1e-3
    y = torch.empty(MB, 512, device="cuda")
    ok = replay_check("kernel linear_tanh_x6 512->512", lambda: U.linear_tanh_x6(x, w, b, out=y), lambda r: [r])
    ok &= replay_check("kernel linear_tanh_out_x6 512->256->2", lambda: U.linear_tanh_out_x6(x, w4, b4, wo, bo),
                       lambda r: list(r))
    ok &= replay_check("kernel linear_tanh_backward_x6 512<-512", lambda: U.linear_tanh_backward_x6(gz, w, x),
                       lambda r: list(r))
    ok &= replay_check("kernel weight_grad_x6 512x512", lambda: U.weight_grad_x6(gz, x), lambda r: [r])
    return ok


def stage_mlp():
    a = agent()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(MB, 52, device="cuda", generator=g)
    gout = torch.randn(MB, 2, device="cuda", generator=g) * 1e-3
    params = list(a.actor_mean.parameters())

    def body():
        for p in params:
            p.grad = None
        out = MLP.mlp_forward(a.actor_mean, x)
        grads = torch.autograd.grad(out, params, gout)
        return [out.detach()] + [t.detach() for t in grads]
    return replay_check(f"mlp actor fwd+bwd ({PATH})", body, lambda r: r)


def stage_minibatch():
    a = agent()
    flat = P.FlatGrads(a)
    args = P.parse_args([])
    g = torch.Generator(device="cuda").manual_seed(3)
    pad = P.padding_rows(MB, "cuda")
    mbg = MBM.MinibatchGraph(a, flat, args, MB, (52,), (2,), "cuda")
    mbg.obs.copy_(torch.randn(MB + pad, 52, device="cuda", generator=g))
    mbg.act.copy_(torch.randn(MB + pad, 2, device="cuda", generator=g) * 0.5)
    for t in (mbg.logp, mbg.adv, mbg.ret, mbg.val):
        t.copy_(torch.randn(MB, device="cuda", generator=g))
    mbg.logp -= 3.0
    return replay_check(f"minibatch body ({PATH})", mbg._body, lambda r: list(r) + [flat.flat])


def stage_ppo():
    """The original failure's setting (tools/graph_probe.py): ppo_update over 8 epochs x 2 minibatches
    with optimizer steps, captured vs eager, from the same initial weights."""
    args = P.parse_args([])
    args.update_epochs, args.num_minibatches = int(os.environ.get("EPOCHS", 8)), 2
    n = 2 * MB
    g = torch.Generator(device="cuda").manual_seed(3)
    obs = torch.randn(n, 52, device="cuda", generator=g)
    act = torch.randn(n, 2, device="cuda", generator=g) * 0.5
    logp, adv, ret, val = (torch.randn(n, device="cuda", generator=g) for _ in range(4))
    logp -= 3.0
    out = []
    for use_graph in (False, True):
        a = agent()
        flat = P.FlatGrads(a)
        opt = torch.optim.Adam(a.parameters(), lr=1e-3, eps=1e-5)
        graph = MBM.MinibatchGraph(a, flat, args, MB, (52,), (2,), "cuda") if use_graph else None
        st = P.ppo_update(a, opt, flat, args, obs, logp, act, adv, ret, val,
                          gen=torch.Generator(device="cuda").manual_seed(7), graph=graph)
        out.append((torch.cat([p.detach().reshape(-1) for p in a.parameters()]), st))
        del graph
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    d = (out[0][0] - out[1][0]).abs().max().item()
    s0 = {k: round(float(v), 6) for k, v in out[0][1].items()}
    s1 = {k: round(float(v), 6) for k, v in out[1][1].items()}
    print(f"[ppo_update {args.update_epochs} epochs x 2 minibatches ({PATH})] max |param diff| graph vs eager "
          f"{d:.3e}\n  eager {s0}\n  graph {s1}", flush=True)
    return d == 0.0


def main():
    print(f"DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '<unset>')} "
          f"PATH_MLP={PATH} LOSS={LOSS} MB={MB} REPLAYS={R} NOISE={NOISE} torch {torch.__version__} hip {torch.version.hip}", flush=True)
    ok = True
    for st in os.environ.get("STAGES", "kernel,mlp,minibatch").split(","):
        ok &= {"kernel": stage_kernel, "mlp": stage_mlp, "minibatch": stage_minibatch, "ppo": stage_ppo}[st]()
    print("ALL STABLE" if ok else "SOME STAGE DIFFERS", flush=True)


if __name__ == "__main__":
    main()
