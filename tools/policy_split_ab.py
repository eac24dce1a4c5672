#!/usr/bin/env python3
"""Profiling-only: the rollout policy at small batches, the product library (vss_policy_forward) against
tools/_build/libpol_old.so (the previous kernels, built from an earlier csrc/vss_policy.hip): the same
(seed, counter) and weights, outputs compared bit for bit (action, log-prob, entropy, value), then
timed with HIP events (median of 5 rounds of 20 launches)."""
import ctypes
import os
import statistics
import sys
from collections import namedtuple

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402

PACKET_CAPTURE_OFF = P.disable_graph_packet_capture()  # an entry point: before anything initialises the GPU
from envs._gym import Box  # noqa: E402
from vss_amd import _native as N  # noqa: E402
from vss_amd.policy import FusedPolicy  # noqa: E402


print(f"DEBUG_CLR_GRAPH_PACKET_CAPTURE off: {PACKET_CAPTURE_OFF}", flush=True)


def timeit(fn, iters=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    Env = namedtuple("Env", ["single_observation_space", "single_action_space"])
    old = ctypes.CDLL(os.path.join(REPO, "tools", "_build", "libpol_old.so"))
    new = N.load()
    old.vss_policy_forward.argtypes = new.vss_policy_forward.argtypes
    st = N.stream_of(torch.device("cuda"))
    for n_act in (2, 6):
        torch.manual_seed(n_act)
        agent = P.Agent(Env(Box(-np.inf, np.inf, (52,)), Box(-1.0, 1.0, (n_act,)))).cuda()
        with torch.no_grad():
            agent.actor_logstd.fill_(-0.5)
        fused = FusedPolicy(agent)
        for rows in (1, 37, 1000, 4095, 8192):
            obs = torch.randn(rows, 52, device="cuda")
            outs = {}
            for name, L in (("new", new), ("old", old)):
                o = [torch.empty(rows, n_act, device="cuda"), torch.empty(rows, device="cuda"),
                     torch.empty(rows, device="cuda"), torch.empty(rows, 1, device="cuda")]

                def run(L=L, o=o):
                    return L.vss_policy_forward(st, rows, n_act, obs.data_ptr(), fused._actor.data_ptr(),
                                                agent.actor_logstd.data_ptr(), fused._critic.data_ptr(), 7, 3, None,
                                                o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), o[3].data_ptr(), None)
                assert run() == 0
                torch.cuda.synchronize()
                outs[name] = ([t.clone() for t in o], run)
            same = all(torch.equal(a, b) for a, b in zip(outs["new"][0], outs["old"][0]))
            diff = max(float((a - b).abs().max()) for a, b in zip(outs["new"][0], outs["old"][0]))
            t = {name: statistics.median(timeit(outs[name][1]) for _ in range(5)) for name in ("new", "old")}
            print(f"n_act {n_act} rows {rows:5d}: outputs {'bit-exact' if same else f'DIFFER (max {diff:.3e})'}; "
                  f"new {t['new']:7.1f} us  old {t['old']:7.1f} us  ({t['old'] / t['new']:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
