"""BASELINE config 2 at its full shape: the HIP step kernel at 4,096 fields, random
actions U[-1, 1], seeds 1..8, free-running for 1,000 steps each against the CPU oracle, with the max
abs / rel error per output channel and the integer mismatch counts reported (needs a GPU).

Per step and seed every output of `VSS.step` (envs/vss.py:180-333 + Ext VecTask.step) is compared:
the 46 live state channels, progress / reset / rng counter / dof (pre_physics_step), the observation
and terminal observation per feature (52 channels, all 6 agents), the 4 reward channels, time-outs
and progress_f.  Bar (tolerance written here): floats BIT-EXACT (max abs error 0 and no value whose
bits differ) -- the kernel and the oracle evaluate the same float32 operation sequence with FMA
contraction off -- and integers exact.  The oracle runs the 8 seeds in 8 host threads (ctypes
releases the GIL) and writes into pinned buffers that are compared on the GPU.
"""
import json
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

import oracle as O
from test_gpu_parity import host_from, make_vss, oracle_params

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
N_FIELDS, STEPS, SEEDS = 4096, 1000, tuple(range(1, 9))
LIVE = [0, 1, 2, 3] + [c + k for c in (O.CH_RX, O.CH_RY, O.CH_RQZ, O.CH_RQW, O.CH_RVX, O.CH_RVY, O.CH_RW)
                       for k in range(6)]
FLOAT_TOL = 0.0  # bit-exact (see the module docstring)


class Seed:
    """One seed: the device env, the oracle env, pinned host outputs and the running error maxima."""

    def __init__(self, seed):
        self.seed = seed
        self.env = make_vss(N_FIELDS, seed=seed)
        self.h = host_from(self.env)
        self.prm = oracle_params(self.env)
        self.gen = np.random.default_rng(seed)
        n = N_FIELDS
        pin = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt).pin_memory()  # noqa: E731
        self.pinned = dict(obs=pin(n * 6, 52), terminal_obs=pin(n * 6, 52), rew=pin(n, 24), time_outs=pin(n, dt=torch.uint8),
                           progress_f=pin(n), state=pin(58, n), progress=pin(n, dt=torch.int64),
                           reset=pin(n, dt=torch.int64), dof=pin(n, 12), ctr=pin(n, dt=torch.int32))
        # the oracle writes straight into the pinned buffers
        self.io = {k: self.pinned[k].numpy() for k in ("obs", "terminal_obs", "rew", "time_outs", "progress_f")}
        self.io.update(reward_sum=None, dones_rep=None, ou_buf=None)
        z = lambda c: torch.zeros(c, dtype=torch.float64, device=DEV)  # noqa: E731
        self.err = dict(state=z(len(LIVE)), obs=z(52), terminal_obs=z(52), rew=z(4), dof=z(12), progress_f=z(1))
        self.ref = dict(state=z(len(LIVE)), obs=z(52), terminal_obs=z(52), rew=z(4), dof=z(12), progress_f=z(1))
        self.bitdiff = torch.zeros((), dtype=torch.int64, device=DEV)
        self.int_mismatch = {k: torch.zeros((), dtype=torch.int64, device=DEV)
                             for k in ("progress", "reset", "ctr", "time_outs")}
        self.resets = self.goals = self.timeouts = 0

    def oracle_step(self, a):
        O.step(self.h, O.MODE_FULL, a, self.io, self.prm)
        self.pinned["state"].numpy()[:] = self.h.state
        self.pinned["progress"].numpy()[:] = self.h.progress
        self.pinned["reset"].numpy()[:] = self.h.reset
        self.pinned["dof"].numpy()[:] = self.h.dof
        self.pinned["ctr"].numpy()[:] = self.h.ctr.view(np.int32)

    def compare(self, obs, tobs, rew, time_outs, progress_f):
        """Accumulate per-channel max |d| and max |want| on the GPU (no host sync)."""
        want = {k: v.to(DEV, non_blocking=True) for k, v in self.pinned.items()}
        env = self.env
        # (got, want, the dimension reduced over: fields / rows)
        pairs = dict(state=(env.state[LIVE], want["state"][LIVE], 1),
                     obs=(obs.reshape(-1, 52), want["obs"], 0),
                     terminal_obs=(tobs.reshape(-1, 52), want["terminal_obs"], 0),
                     rew=(rew.reshape(-1, 4), want["rew"].reshape(-1, 4), 0),
                     dof=(env.dof_velocity_buf.reshape(-1, 12), want["dof"], 0),
                     progress_f=(progress_f.reshape(-1, 1), want["progress_f"].reshape(-1, 1), 0))
        for k, (got, w, red) in pairs.items():
            d = (got.double() - w.double()).abs().amax(dim=red)
            self.err[k] = torch.maximum(self.err[k], d)
            self.ref[k] = torch.maximum(self.ref[k], w.double().abs().amax(dim=red))
            self.bitdiff += (got.contiguous().view(torch.int32) != w.contiguous().view(torch.int32)).sum()
        self.int_mismatch["progress"] += (env.progress_buf != want["progress"]).sum()
        self.int_mismatch["reset"] += (env.reset_buf != want["reset"]).sum()
        self.int_mismatch["ctr"] += (env.rng_counter.view(torch.int32) != want["ctr"]).sum()
        self.int_mismatch["time_outs"] += (time_outs.to(torch.uint8) != want["time_outs"]).sum()

    def report(self):
        rel = {k: (self.err[k] / self.ref[k].clamp_min(1e-30)).amax().item() for k in self.err}
        return dict(seed=self.seed, fields=N_FIELDS, steps=STEPS, resets=self.resets, goals=self.goals,
                    time_outs=self.timeouts,
                    max_abs={k: v.amax().item() for k, v in self.err.items()}, max_rel=rel,
                    max_abs_per_channel={k: v.tolist() for k, v in self.err.items()},
                    float_values_with_differing_bits=int(self.bitdiff.item()),
                    integer_mismatches={k: int(v.item()) for k, v in self.int_mismatch.items()})


def test_config2_4096_fields_1000_steps_seeds_1_to_8_bit_exact(capsys):
    seeds = [Seed(s) for s in SEEDS]
    pool = ThreadPoolExecutor(max_workers=len(seeds))
    for t in range(STEPS):
        acts = [s.gen.uniform(-1.0, 1.0, (N_FIELDS, 12)).astype(np.float32) for s in seeds]
        outs = []
        for s, a in zip(seeds, acts):
            outs.append(s.env.step(torch.from_numpy(a).to(DEV).view(N_FIELDS, 2, 3, 2)))
        list(pool.map(lambda sa: sa[0].oracle_step(sa[1]), zip(seeds, acts)))
        for s, (obs_dict, rew, reset, extras) in zip(seeds, outs):
            s.compare(obs_dict["obs"], extras["terminal_observation"], rew, extras["time_outs"],
                      extras["progress_buffer"])
            s.resets += int(s.h.reset.sum())
            s.goals += int((np.abs(s.io["rew"][:, 0]) > 0).sum())
            s.timeouts += int(s.io["time_outs"].sum())
        torch.cuda.synchronize()  # the pinned buffers are rewritten by the next step's oracle
    pool.shutdown()
    reports = [s.report() for s in seeds]
    with capsys.disabled():
        for r in reports:
            print(f"\nconfig2 seed {r['seed']}: {r['fields']} fields x {r['steps']} steps, resets {r['resets']}, "
                  f"goals {r['goals']}, time-outs {r['time_outs']} | max abs " +
                  " ".join(f"{k} {v:g}" for k, v in r["max_abs"].items()) +
                  f" | float values with differing bits {r['float_values_with_differing_bits']}"
                  f" | integer mismatches {r['integer_mismatches']}")
        print("CONFIG2_PARITY " + json.dumps(reports))
    for r in reports:
        assert all(v <= FLOAT_TOL for v in r["max_abs"].values()), r
        assert r["float_values_with_differing_bits"] == 0, r
        assert all(v == 0 for v in r["integer_mismatches"].values()), r
        assert r["resets"] > 0 and r["time_outs"] > 0
    assert sum(r["goals"] for r in reports) > 0
