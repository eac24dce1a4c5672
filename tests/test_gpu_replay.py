"""The HIP step kernels against the REFERENCE's golden fixtures, directly (needs a GPU).

`vss_step_replay` / `vss_reset_dones_replay` (include/vss.h) run the product kernel templates
with the reference's own recorded torch draws (reset sampling, envs/vss.py:267-333; OU noise,
envs/wrappers.py:5-19) in place of the Philox stream, so the fixtures made by the reference
(tests/golden/gen_golden.py) check the kernel itself, not only the oracle.  Teacher-forced step
by step, exactly like tests/test_oracle_golden.py checks the oracle:

  * G4 = BASELINE config 1: 16 fields x 1,000 steps of the raw VSS.step (FULL contract), with
    goals forced at the time-out edge;
  * G5: SingleAgent / CMA / DMA wrappers, 6 fields x 60 steps, with goals forced at both ends,
    mid-episode and at the time-out edge;
  * the construction-time reset (VSS.__init__ -> reset_dones over every field).

Bar: integers (progress, reset, dones, time-outs) bit-exact; floats bit-exact except values that
go through sin/cos (the reference's torch sin/cos/atan2 vs the kernel's polynomial / algebraic
forms), which agree within 2e-6; rewards within 1e-6 (the reference's torch reductions).
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle as O
import replay_draws as RD
from test_oracle_golden import TRIG_ATOL, assert_obs_equal, assert_wrapped_goals_pinned, load
from vss_amd import _native as N

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
QUAT = list(range(O.CH_RQZ, O.CH_RQZ + 12))


class DevEnv:
    """Device buffers in the include/vss.h layout, driven through the replay entries."""

    def __init__(self, n, mode):
        self.n, self.mode = n, mode
        self.state = torch.zeros((O.STATE_CHANNELS, n), device=DEV)
        self.state[O.CH_RQW:O.CH_RQW + 6] = 1.0
        self.progress = torch.zeros(n, dtype=torch.int64, device=DEV)
        self.reset = torch.ones(n, dtype=torch.int64, device=DEV)
        self.dof = torch.zeros((n, 12), device=DEV)
        self.ctr = torch.zeros(n, dtype=torch.int32, device=DEV)
        agents = {O.MODE_FULL: 6, O.MODE_SA: 1, O.MODE_CMA: 1, O.MODE_DMA: 3}[mode]
        R = 3 if mode == O.MODE_DMA else 1
        rew_w = 24 if mode == O.MODE_FULL else 4
        rows = n * R
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=DEV)  # noqa: E731
        self.io = dict(obs=z(n * agents, 52), terminal_obs=z(n * agents, 52), rew=z(rows, rew_w),
                       reward_sum=z(rows), time_outs=z(rows, dt=torch.uint8), progress_f=z(rows),
                       dones_rep=z(rows, dt=torch.int64) if mode == O.MODE_DMA else None,
                       ou_buf=z(n, 12) if mode != O.MODE_FULL else None)

    def c_state(self):
        p = N.ptr
        return N.VssState(p(self.state), p(self.progress), p(self.reset), p(self.dof), p(self.ctr))

    def set_live(self, live, live_state, progress, reset, dof=None):
        s = np.zeros((O.STATE_CHANNELS, self.n), np.float32)
        s[live] = live_state
        self.state.copy_(torch.from_numpy(s))
        self.progress.copy_(torch.from_numpy(np.asarray(progress, np.int64)))
        self.reset.copy_(torch.from_numpy(np.asarray(reset, np.int64)))
        if dof is not None:
            self.dof.copy_(torch.from_numpy(np.asarray(dof, np.float32)))

    @staticmethod
    def draws(rows, normals):
        u = torch.from_numpy(np.ascontiguousarray(rows, np.float32)).to(DEV)
        z = None if normals is None else torch.from_numpy(np.ascontiguousarray(normals, np.float32)).to(DEV)
        return N.VssReplayDraws(u.data_ptr(), u.shape[1], N.ptr(z)), (u, z)

    def step(self, actions, rows, normals, max_len):
        L = N.load()
        a = torch.from_numpy(np.ascontiguousarray(actions, np.float32)).to(DEV)
        io = self.io
        cio = N.VssStepIO(*(N.ptr(io[k]) if k != "actions" else a.data_ptr() for k in
                            ("actions", "ou_buf", "obs", "terminal_obs", "rew", "reward_sum", "dones_rep",
                             "time_outs", "progress_f")))
        prm = N.VssParams(10.0, 2.0, 3.0, 0.0, 1.0, int(max_len), 1)
        st = self.c_state()
        d, keep = self.draws(rows, normals)
        rc = L.vss_step_replay(N.stream_of(torch.device(DEV)), self.n, self.mode, ctypes.byref(prm),
                               ctypes.byref(st), ctypes.byref(cio), ctypes.byref(d))
        N.check(rc, "vss_step_replay")
        torch.cuda.synchronize()

    def reset_dones(self, rows, max_len):
        prm = N.VssParams(10.0, 2.0, 3.0, 0.0, 1.0, int(max_len), 1)
        st = self.c_state()
        d, keep = self.draws(rows, None)
        rc = N.load().vss_reset_dones_replay(N.stream_of(torch.device(DEV)), self.n, ctypes.byref(prm),
                                             ctypes.byref(st), ctypes.byref(d))
        N.check(rc, "vss_reset_dones_replay")
        torch.cuda.synchronize()

    def host(self, k):
        return self.io[k].cpu().numpy()


def assert_state(dev, live, want, msg):
    quat = np.isin(live, QUAT)
    got = dev.state.cpu().numpy()[live]
    np.testing.assert_array_equal(got[~quat], want[~quat], err_msg=msg)
    np.testing.assert_allclose(got[quat], want[quat], atol=TRIG_ATOL, rtol=0, err_msg=msg)


def step_draws(g, done_of_step):
    """Per step: (rows, rounds) of the reference's reset draws regrouped per field."""
    n = g["init_state"].shape[1]
    sizes = RD.split_steps(g["u_sizes"], g["u_ncalls"])
    flats = RD.split_steps(g["uniforms"], [int(s.sum()) for s in sizes])
    return [RD.to_rows(flats[t], np.nonzero(done_of_step[t])[0], n, sizes[t]) for t in range(len(flats))]


@pytest.mark.parametrize("name", ["g4_full_rollout.npz", "g5_wrapped_sa.npz"])
def test_construction_reset_replay_matches_reference(golden_dir, name):
    """VSS.__init__ -> reset_dones over all fields (envs/vss.py:72, 267-333) on the HIP reset kernel."""
    g = load(golden_dir, name)
    n = g["init_state"].shape[1]
    dev = DevEnv(n, O.MODE_FULL)
    rows, rounds = RD.to_rows(g["init_uniforms"], np.arange(n), n, g["init_u_sizes"])
    dev.reset_dones(rows, int(g["max_len"]))
    assert_state(dev, g["live_channels"], g["init_state"][g["live_channels"]], "construction reset")
    np.testing.assert_array_equal(dev.dof.cpu().numpy(), 0)


def test_full_step_replay_matches_reference_config1(golden_dir):
    """BASELINE config 1 (16 fields x 1,000 steps, random actions) through vss_step_replay (FULL):
    progress / reset / time-out ordering, rewards, terminal obs, reset sampling, dof zeroing
    (envs/vss.py:180-333, Ext VecTask.step) -- the reference's outputs vs the HIP kernel."""
    g = load(golden_dir, "g4_full_rollout.npz")
    live = g["live_channels"]
    T, n = g["reset"].shape
    assert (T, n) == (1000, 16)
    ml = int(g["max_len"])
    obs_at = {int(t): i for i, t in enumerate(g["obs_steps"])}
    forced = {int(t): i for i, t in enumerate(g["forced_steps"])}
    draws = step_draws(g, g["reset"])
    dev = DevEnv(n, O.MODE_FULL)
    resets = 0
    for t in range(T):
        if t == 0:
            dev.set_live(live, g["start_state"][live], np.zeros(n), np.ones(n), np.zeros((n, 12)))
        else:
            pre = g["forced_state"][forced[t]] if t in forced else g["state"][t - 1]
            dev.set_live(live, pre, g["progress"][t - 1], g["reset"][t - 1], g["dof"][t - 1])
        rows, rounds = draws[t]
        dev.step(g["actions"][t], rows, None, ml)
        msg = f"step {t}"
        np.testing.assert_array_equal(dev.reset.cpu().numpy(), g["reset"][t], err_msg=msg)
        np.testing.assert_array_equal(dev.progress.cpu().numpy(), g["progress"][t], err_msg=msg)
        np.testing.assert_array_equal(dev.host("time_outs"), g["time_outs"][t], err_msg=msg)
        np.testing.assert_array_equal(dev.host("progress_f"), g["progress_f"][t], err_msg=msg)
        np.testing.assert_array_equal(dev.dof.cpu().numpy(), g["dof"][t], err_msg=msg)
        np.testing.assert_allclose(dev.host("rew"), g["rew"][t], rtol=1e-6, atol=1e-6, err_msg=msg)
        assert_state(dev, live, g["state"][t], msg)
        if t in obs_at:
            assert_obs_equal(dev.host("obs"), g["obs"][obs_at[t]])
            assert_obs_equal(dev.host("terminal_obs"), g["terminal_obs"][obs_at[t]])
        resets += int(g["reset"][t].sum())
    assert resets == int(g["reset"].sum()) and resets > 30 and g["time_outs"].sum() > 0
    (t2, t1), (f2, f1) = g["edge_steps"], g["edge_fields"]
    assert g["time_outs"][t1, f1] == 1 and g["time_outs"][t2, f2] == 0 and (t2, t1) == (ml - 3, ml - 2)


@pytest.mark.parametrize("mode_name", ["sa", "cma", "dma"])
def test_wrapped_step_replay_matches_reference(golden_dir, mode_name):
    """SingleAgent / CMA / DMA (envs/wrappers.py:5-19, 89-180) through vss_step_replay: the
    reference's OU normals and reset draws fed to the fused wrapper kernels, teacher-forced."""
    g = load(golden_dir, f"g5_wrapped_{mode_name}.npz")
    mode = {"sa": O.MODE_SA, "cma": O.MODE_CMA, "dma": O.MODE_DMA}[mode_name]
    live = g["live_channels"]
    T = g["dones"].shape[0]
    n = g["state"].shape[2]
    R = 3 if mode == O.MODE_DMA else 1
    agents = 3 if mode == O.MODE_DMA else 1
    ml = int(g["max_len"])
    draws = step_draws(g, g["dones"][:, ::R])
    normals = RD.split_steps(g["normals"], g["n_z"])
    forced = {int(t): i for i, t in enumerate(g["forced_steps"])}
    dev = DevEnv(n, mode)
    for t in range(T):
        if t == 0:
            pre = g["forced_state"][forced[0]] if 0 in forced else g["init_state"][live]
            dev.set_live(live, pre, np.zeros(n), np.ones(n), np.zeros((n, 12)))
            ou = np.zeros((n, 12), np.float32)
        else:
            pre = g["forced_state"][forced[t]] if t in forced else g["state"][t - 1]
            dev.set_live(live, pre, g["progress_f"][t - 1][::R].astype(np.int64), g["dones"][t - 1][::R])
            ou = g["action_buf"][t - 1]
        dev.io["ou_buf"].copy_(torch.from_numpy(np.ascontiguousarray(ou, np.float32)))
        assert normals[t].size == 12 * n, "random_ou draws one (N, 2, 3, 2) normal tensor per step"
        dev.step(g["actions"][t], draws[t][0], normals[t].reshape(n, 12), ml)
        msg = f"step {t}"
        np.testing.assert_array_equal(dev.host("ou_buf"), g["action_buf"][t], err_msg=msg)
        if mode == O.MODE_DMA:
            np.testing.assert_array_equal(dev.host("dones_rep"), g["dones"][t], err_msg=msg)
        else:
            np.testing.assert_array_equal(dev.reset.cpu().numpy(), g["dones"][t], err_msg=msg)
        np.testing.assert_array_equal(dev.host("time_outs"), g["time_outs"][t], err_msg=msg)
        np.testing.assert_array_equal(dev.host("progress_f"), g["progress_f"][t], err_msg=msg)
        np.testing.assert_allclose(dev.host("rew"), g["rews"][t], rtol=1e-6, atol=1e-6, err_msg=msg)
        np.testing.assert_allclose(dev.host("reward_sum"), g["reward"][t], rtol=1e-6, atol=2e-6, err_msg=msg)
        assert_obs_equal(dev.host("obs"), g["obs"][t], agents=agents)
        assert_obs_equal(dev.host("terminal_obs"), g["terminal_obs"][t], agents=agents)
        assert_state(dev, live, g["state"][t], msg)
    assert_wrapped_goals_pinned(g, R)


def test_replay_entries_reject_bad_draws():
    """The parity entries validate their draw descriptors (VSS_E_ARG, no launch)."""
    L = N.load()
    dev = DevEnv(4, O.MODE_SA)
    prm = N.VssParams(10.0, 2.0, 3.0, 0.0, 1.0, 400, 1)
    st = dev.c_state()
    u = torch.zeros((4, 22), device=DEV)
    io = N.VssStepIO(*(N.ptr(dev.io[k]) if k != "actions" else dev.io["obs"].data_ptr() for k in
                       ("actions", "ou_buf", "obs", "terminal_obs", "rew", "reward_sum", "dones_rep",
                        "time_outs", "progress_f")))
    short = N.VssReplayDraws(u.data_ptr(), 21, u.data_ptr())
    no_normals = N.VssReplayDraws(u.data_ptr(), 22, None)
    s = N.stream_of(torch.device(DEV))
    assert L.vss_step_replay(s, 4, O.MODE_SA, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(io), ctypes.byref(short)) == 1
    assert L.vss_step_replay(s, 4, O.MODE_SA, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(io), ctypes.byref(no_normals)) == 1
    assert L.vss_step_replay(s, 4, O.MODE_SA, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(io), None) == 1
    assert L.vss_reset_dones_replay(s, 4, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(short)) == 1
    # a row holding more rejection rounds than the kernel's bound (64) is refused, not replayed short
    too_many = N.VssReplayDraws(u.data_ptr(), 14 * 65 + 8, u.data_ptr())
    assert L.vss_step_replay(s, 4, O.MODE_SA, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(io), ctypes.byref(too_many)) == 1
    assert L.vss_reset_dones_replay(s, 4, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(too_many)) == 1
