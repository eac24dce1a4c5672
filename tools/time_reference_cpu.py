#!/usr/bin/env python3
"""Time the REFERENCE's own VSS.step control flow on this container's CPU (build container only:
imports /root/reference through the stub harness of tests/golden/gen_golden.py; physics hook =
the oracle's C physics), beside the C oracle on the same workload.  Output: one JSON line used in
DESIGN.md §7 as the reference-vs-oracle calibration.  Never runs on the GPU box."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests", "golden"))
import gen_golden as G  # noqa: E402  (sets PYTORCH_JIT=0, installs stubs on demand)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def time_reference(n, steps, threads):
    torch.set_num_threads(threads)
    env = G.make_env(n, 400)
    gen = np.random.default_rng(1)
    acts = [torch.from_numpy(gen.uniform(-1, 1, (n, 2, 3, 2)).astype(np.float32)) for _ in range(8)]
    env.step(acts[0])
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(acts[k % 8])
    return n * steps / (time.perf_counter() - t0)


def time_oracle(n, steps):
    O = G.O
    h = O.HostEnv(n)
    prm = O.params()
    O.reset_dones(h, prm)
    io = O.make_io(n, O.MODE_FULL)
    gen = np.random.default_rng(1)
    acts = [gen.uniform(-1, 1, (n, 12)).astype(np.float32) for _ in range(8)]
    t0 = time.perf_counter()
    for k in range(steps):
        O.step(h, O.MODE_FULL, acts[k % 8], io, prm)
    return n * steps / (time.perf_counter() - t0)


def main():
    G.install_stubs()
    G.O.build()
    rec = G.Recorder()
    rec.install()
    res = {"host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": "),
           "nproc": os.cpu_count(), "rows": []}
    for n, steps in ((16, 1000), (4096, 50), (65536, 5)):
        for thr in (os.cpu_count(), 1):
            r = time_reference(n, steps, thr)
            rec.take()
            res["rows"].append({"fields": n, "steps": steps, "impl": "reference VSS.step (torch eager CPU) + oracle physics hook",
                                "threads": thr, "env_steps_per_s": r})
        res["rows"].append({"fields": n, "steps": steps, "impl": "oracle/vss_oracle.c", "threads": 1,
                            "env_steps_per_s": time_oracle(n, steps)})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
