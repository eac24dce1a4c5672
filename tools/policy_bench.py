#!/usr/bin/env python3
"""Time the rollout policy forward at 65,536 rows: torch Agent (hipBLASLt fp32) vs the fused
HIP kernel (vss_policy_forward).  Per rollout step the reference runs actor+critic on next_obs
and the critic on the terminal obs (ppo…:262,272) = 3.23 MFLOP per env-step."""
import json
import os
import sys
from collections import namedtuple

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402
from envs._gym import Box  # noqa: E402
from vss_amd.policy import FusedPolicy  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    rows = int(os.environ.get("ROWS", 65536))
    Env = namedtuple("Env", ["single_observation_space", "single_action_space"])
    torch.manual_seed(0)
    agent = P.Agent(Env(Box(-np.inf, np.inf, (52,)), Box(-1.0, 1.0, (2,)))).cuda()
    fused = FusedPolicy(agent)
    obs = torch.randn(rows, 52, device="cuda")
    tobs = torch.randn(rows, 52, device="cuda")

    def torch_step():
        with torch.no_grad():
            agent.get_action_and_value(obs)
            agent.get_value(tobs)

    def fused_step():
        fused.get_action_and_value(obs)
        fused.get_value(tobs)

    t_torch = timeit(torch_step)
    t_fused = timeit(fused_step)
    t_ac = timeit(lambda: fused.get_action_and_value(obs))
    flop_ac = 2 * rows * (52 * 256 + 256 * 512 + 512 * 512 + 512 * 256 + 256 * 2 + 52 * 256 + 256 * 512 + 512 * 512 + 512 * 256 + 256)
    # build variants placed in tools/_build/libpol_*.so (e.g. hipcc ... -DVPOL_CK=.. -DVPOL_OS=.. -shared)
    import ctypes
    import glob
    from vss_amd import _native as N
    var = {}
    for path in sorted(glob.glob(os.path.join(REPO, "tools", "_build", "libpol_*.so"))):
        L = ctypes.CDLL(path)
        L.vss_policy_forward.argtypes = N.load().vss_policy_forward.argtypes
        act = torch.empty(rows, 2, device="cuda")
        lp = torch.empty(rows, device="cuda")
        v = torch.empty(rows, 1, device="cuda")
        st = N.stream_of(torch.device("cuda"))

        def run(L=L):
            L.vss_policy_forward(st, rows, 2, obs.data_ptr(), fused._actor.data_ptr(),
                                 agent.actor_logstd.data_ptr(), fused._critic.data_ptr(), 1, 1, None,
                                 act.data_ptr(), lp.data_ptr(), None, v.data_ptr(), None)
        var[os.path.basename(path)] = timeit(run)
    # diagnostic: the same launch with the actor's weights streamed twice (as actor and as "critic"):
    # a 2.1 MB stream that fits one XCD's 4 MB L2, against the 4.3 MB actor + critic stream
    act = torch.empty(rows, 2, device="cuda")
    lp = torch.empty(rows, device="cuda")
    v = torch.empty(rows, 1, device="cuda")
    st = N.stream_of(torch.device("cuda"))
    L0 = N.load()
    var["actor_weights_twice (diagnostic, wrong values)"] = timeit(lambda: L0.vss_policy_forward(
        st, rows, 2, obs.data_ptr(), fused._actor.data_ptr(), agent.actor_logstd.data_ptr(), fused._actor.data_ptr(),
        1, 1, None, act.data_ptr(), lp.data_ptr(), None, v.data_ptr(), None))
    var["critic_only"] = timeit(lambda: fused.get_value(tobs))
    print(json.dumps({"variants_actor_critic_ms": var}))
    print(json.dumps({"rows": rows, "torch_ms_per_step": t_torch, "fused_ms_per_step": t_fused,
                      "speedup": t_torch / t_fused, "fused_actor_critic_ms": t_ac,
                      "fused_actor_critic_tflops": flop_ac / (t_ac * 1e-3) / 1e12, "peak_fp32_mfma_tflops": 157.3}))


if __name__ == "__main__":
    main()
