"""Pin the CPU oracle against golden vectors produced by the REFERENCE's own Python.

Fixtures: tests/golden/*.npz, made by tests/golden/gen_golden.py (imports /root/reference with
stub Isaac Gym modules; physics hook = this oracle's physics).  These tests run on CPU.
Tolerances: integer outputs (goal, dones, progress, time-outs, reset counts) bit-exact; float
outputs bit-exact except values that go through sin/cos (reference: torch atan2/sin/cos of the
quaternion; oracle: algebraic cos = w^2 - z^2, sin = 2wz, and polynomial half-angle sin/cos for
reset yaw), which must agree within 2e-6.
"""
import os

import numpy as np
import pytest

import oracle as O

TRIG_ATOL = 2e-6


def load(golden_dir, name):
    """All arrays of a fixture, decompressed once (an NpzFile re-reads a key on every access)."""
    with np.load(os.path.join(golden_dir, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def obs_trig_mask():
    """(312,) bool: obs features that are cos/sin(yaw) in the (2,3,52) layout."""
    m = np.zeros(52, bool)
    for k in range(3):
        m[4 + 9 * k + 4] = m[4 + 9 * k + 5] = True
    for k in range(3):
        m[31 + 7 * k + 4] = m[31 + 7 * k + 5] = True
    return np.tile(m, 6)


def assert_obs_equal(got, want, agents=6):
    got = got.reshape(-1, agents * 52)
    want = want.reshape(-1, agents * 52)
    trig = obs_trig_mask()[: agents * 52]
    np.testing.assert_array_equal(got[:, ~trig], want[:, ~trig])
    np.testing.assert_allclose(got[:, trig], want[:, trig], atol=TRIG_ATOL, rtol=0)


# --------------------------------------------------------------------------------- G1-G3
def test_compute_obs_matches_reference(golden_dir):
    g = load(golden_dir, "g1_g3_kernels.npz")
    s = g["obs_state"]
    n = s.shape[1]
    env = O.HostEnv(n)
    env.state[:] = s
    env.dof[:] = g["obs_actions"]
    obs = O.compute_obs(env, 6)
    assert_obs_equal(obs, g["obs"])
    # blue-team (DMA) and blue-robot-0 (SA) packings are prefixes of the full layout
    np.testing.assert_array_equal(O.compute_obs(env, 3), obs[:, :3])
    np.testing.assert_array_equal(O.compute_obs(env, 1), obs[:, :1])


def test_goal_and_dones_bit_exact(golden_dir):
    g = load(golden_dir, "g1_g3_kernels.npz")
    balls = np.ascontiguousarray(g["goal_ball"])
    m = len(balls)
    goal = np.zeros(m, np.int64)
    O.lib().oracle_goal_rew(m, O._p(balls), O._p(goal))
    want = g["goal"]  # (m, 2, 3): blue +g, yellow -g
    np.testing.assert_array_equal(want[:, 0, 0], goal)
    np.testing.assert_array_equal(want[:, 1, 2], -goal)
    prog = np.ascontiguousarray(g["goal_progress"])
    dones = np.zeros(m, np.int64)
    O.lib().oracle_vss_dones(m, O._p(balls), O._p(prog), 400, O._p(dones))
    np.testing.assert_array_equal(dones, g["dones"])
    assert dones.sum() > 0 and (dones == 0).sum() > 0


def test_grad_move_energy_match_reference(golden_dir):
    g = load(golden_dir, "g1_g3_kernels.npz")
    n = len(g["ball"])
    pb, b = np.ascontiguousarray(g["prev_ball"]), np.ascontiguousarray(g["ball"])
    grad = np.zeros(n, np.float32)
    O.lib().oracle_grad_rew(n, O._p(pb), O._p(b), O._p(grad))
    np.testing.assert_allclose(grad, g["grad"][:, 0, 0], rtol=0, atol=1e-6)
    np.testing.assert_allclose(-grad, g["grad"][:, 1, 1], rtol=0, atol=1e-6)
    move = np.zeros((n, 6), np.float32)
    pr, r = np.ascontiguousarray(g["prev_rob"]), np.ascontiguousarray(g["rob"])
    O.lib().oracle_move_rew(n, O._p(pr), O._p(r), O._p(pb), O._p(b), O._p(move))
    np.testing.assert_allclose(move, g["move"].reshape(n, 6), rtol=0, atol=1e-6)


# --------------------------------------------------------------------------------- G4
def _env_from_live(n, live_channels, live_state, progress, reset):
    env = O.HostEnv(n)
    env.state[:] = 0
    env.state[live_channels] = live_state
    env.progress[:] = progress
    env.reset[:] = reset
    return env


def test_construction_reset_matches_reference(golden_dir):
    """VSS.__init__ → reset_dones over all fields (envs/vss.py:72, 267-333), replayed draws."""
    g = load(golden_dir, "g4_full_rollout.npz")
    n = g["init_state"].shape[1]
    env = O.HostEnv(n)
    draws, keep = O.make_draws(g["init_uniforms"], np.zeros(0, np.float32))
    O.reset_dones(env, O.params(max_episode_length=int(g["max_len"])), draws)
    assert draws.uniform_pos == len(g["init_uniforms"]), "reference draw count not reproduced"
    want = g["init_state"]
    live = g["live_channels"]
    quat = np.isin(live, list(range(O.CH_RQZ, O.CH_RQZ + 12)))
    np.testing.assert_array_equal(env.state[live[~quat]], want[live[~quat]])
    np.testing.assert_allclose(env.state[live[quat]], want[live[quat]], atol=TRIG_ATOL, rtol=0)


def test_full_step_bookkeeping_matches_reference(golden_dir):
    """Teacher-forced replay of the reference's VSS.step over BASELINE config 1 (16 fields x
    1,000 steps, random actions) -- progress / reset / time-out ordering, rewards, terminal obs,
    reset sampling order, dof zeroing (envs/vss.py:180-333, Ext VecTask.step)."""
    g = load(golden_dir, "g4_full_rollout.npz")
    live = g["live_channels"]
    T, n = g["reset"].shape
    prm = O.params(max_episode_length=int(g["max_len"]))
    quat = np.isin(live, list(range(O.CH_RQZ, O.CH_RQZ + 12)))
    obs_at = {int(t): i for i, t in enumerate(g["obs_steps"])}
    u_off = np.concatenate([[0], np.cumsum(g["u_count"])])
    forced = {int(t): i for i, t in enumerate(g["forced_steps"])}
    for t in range(T):
        if t == 0:
            env = O.HostEnv(n)
            env.state[:] = g["start_state"]
            env.progress[:] = 0
            env.reset[:] = 1
        else:
            pre = g["forced_state"][forced[t]] if t in forced else g["state"][t - 1]
            env = _env_from_live(n, live, pre, g["progress"][t - 1], g["reset"][t - 1])
            env.dof[:] = g["dof"][t - 1]
        io = O.make_io(n, O.MODE_FULL)
        draws, keep = O.make_draws(g["uniforms"][u_off[t]:u_off[t + 1]], np.zeros(0, np.float32))
        O.step(env, O.MODE_FULL, g["actions"][t], io, prm, draws)
        assert draws.uniform_pos == g["u_count"][t], f"step {t}: draw count"
        np.testing.assert_array_equal(env.reset, g["reset"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(env.progress, g["progress"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(io["time_outs"], g["time_outs"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(io["progress_f"], g["progress_f"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(env.dof, g["dof"][t], err_msg=f"step {t}")
        np.testing.assert_allclose(io["rew"], g["rew"][t], rtol=1e-6, atol=1e-6, err_msg=f"step {t}")
        st = env.state[live]
        np.testing.assert_array_equal(st[~quat], g["state"][t][~quat], err_msg=f"step {t}")
        np.testing.assert_allclose(st[quat], g["state"][t][quat], atol=TRIG_ATOL, rtol=0, err_msg=f"step {t}")
        if t in obs_at:
            assert_obs_equal(io["obs"], g["obs"][obs_at[t]])
            assert_obs_equal(io["terminal_obs"], g["terminal_obs"][obs_at[t]])
    assert (T, n) == (1000, 16), "G4 is BASELINE config 1: 16 fields x 1,000 steps"
    assert g["time_outs"].sum() > 0 and (np.abs(g["rew"][:, :, 0]) > 0).sum() > 0
    # the time-out edge: a goal at progress max_len-1 is a time-out, at max_len-2 it is not
    ml = int(g["max_len"])
    (t2, t1), (f2, f1) = g["edge_steps"], g["edge_fields"]
    assert (t2, t1) == (ml - 3, ml - 2)
    assert g["reset"][t1, f1] == 1 and g["time_outs"][t1, f1] == 1 and g["progress"][t1, f1] == ml - 1
    assert g["reset"][t2, f2] == 1 and g["time_outs"][t2, f2] == 0 and g["progress"][t2, f2] == ml - 2


# --------------------------------------------------------------------------------- G5
@pytest.mark.parametrize("mode_name", ["sa", "cma", "dma"])
def test_wrapped_step_matches_reference(golden_dir, mode_name):
    """SingleAgent / CMA / DMA (envs/wrappers.py:5-19, 89-180), teacher-forced."""
    g = load(golden_dir, f"g5_wrapped_{mode_name}.npz")
    mode = {"sa": O.MODE_SA, "cma": O.MODE_CMA, "dma": O.MODE_DMA}[mode_name]
    live = g["live_channels"]
    T = g["dones"].shape[0]
    n = g["state"].shape[2]
    R = 3 if mode == O.MODE_DMA else 1
    agents = 3 if mode == O.MODE_DMA else 1
    prm = O.params(max_episode_length=int(g["max_len"]))
    quat = np.isin(live, list(range(O.CH_RQZ, O.CH_RQZ + 12)))
    u_off = np.concatenate([[0], np.cumsum(g["n_u"])])
    z_off = np.concatenate([[0], np.cumsum(g["n_z"])])
    forced = {int(t): i for i, t in enumerate(g["forced_steps"])}
    for t in range(T):
        if t == 0:
            pre = g["forced_state"][forced[0]] if 0 in forced else g["init_state"][live]
            env = _env_from_live(n, live, pre, np.zeros(n, np.int64), np.ones(n, np.int64))
            ou = np.zeros((n, 12), np.float32)
        else:
            pre = g["forced_state"][forced[t]] if t in forced else g["state"][t - 1]
            env = _env_from_live(n, live, pre, g["progress_f"][t - 1][::R].astype(np.int64), g["dones"][t - 1][::R])
            ou = g["action_buf"][t - 1].copy()
        io = O.make_io(n, mode)
        io["ou_buf"][:] = ou
        draws, keep = O.make_draws(g["uniforms"][u_off[t]:u_off[t + 1]], g["normals"][z_off[t]:z_off[t + 1]])
        O.step(env, mode, g["actions"][t], io, prm, draws)
        assert draws.uniform_pos == g["n_u"][t] and draws.normal_pos == g["n_z"][t]
        np.testing.assert_array_equal(io["ou_buf"], g["action_buf"][t], err_msg=f"step {t}")
        if mode == O.MODE_DMA:
            np.testing.assert_array_equal(io["dones_rep"], g["dones"][t])
        else:
            np.testing.assert_array_equal(env.reset, g["dones"][t])
        np.testing.assert_array_equal(io["time_outs"], g["time_outs"][t])
        np.testing.assert_array_equal(io["progress_f"], g["progress_f"][t])
        np.testing.assert_allclose(io["rew"], g["rews"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(io["reward_sum"], g["reward"][t], rtol=1e-6, atol=2e-6)
        assert_obs_equal(io["obs"], g["obs"][t], agents=1)
        assert_obs_equal(io["terminal_obs"], g["terminal_obs"][t], agents=1)
        st = env.state[live]
        np.testing.assert_array_equal(st[~quat], g["state"][t][~quat])
        np.testing.assert_allclose(st[quat], g["state"][t][quat], atol=TRIG_ATOL, rtol=0)
    assert_wrapped_goals_pinned(g, R)
    if mode == O.MODE_DMA:
        assert int(g["num_envs"]) == 3 * n  # DMA re-assigns num_environments (envs/wrappers.py:154)


def assert_wrapped_goals_pinned(g, R):
    """A G5 fixture exercises goal terminations (not only time-outs): goal-channel rewards of both
    signs, goal dones with time_outs = 0 (mid-episode: the OU buffer is zeroed mid-episode), and a
    goal at progress max_len - 1, where the reference's formula makes it a time-out
    (envs/vss.py:578-594, 634-655; Ext VecTask.step)."""
    goal = g["rews"][..., 0]
    done = g["dones"] != 0
    assert (goal > 0).sum() > 0 and (goal < 0).sum() > 0, "both teams must score"
    assert ((goal != 0) & done & (g["time_outs"] == 0)).sum() >= 4 * R, "goal dones with time_outs = 0"
    assert ((goal == 0) & done & (g["time_outs"] == 1)).sum() > 0, "plain time-outs"
    ml = int(g["max_len"])
    (t2, t1), (f2, f1) = g["edge_steps"], g["edge_fields"]
    assert (t2, t1) == (ml - 3, ml - 2)
    assert g["progress_f"][t1, f1 * R] == ml - 1 and g["time_outs"][t1, f1 * R] == 1 and goal[t1, f1 * R] != 0
    assert g["progress_f"][t2, f2 * R] == ml - 2 and g["time_outs"][t2, f2 * R] == 0 and goal[t2, f2 * R] != 0
    # a goal done mid-episode zeroes the done field's OU action buffer (envs/wrappers.py:105-107)
    mid = np.nonzero((goal[:, ::R] != 0) & (g["time_outs"][:, ::R] == 0))
    assert len(mid[0]) > 0 and np.all(g["action_buf"][mid[0], mid[1]] == 0)


def test_reset_placement_threshold_is_exact():
    """The HIP reset compares squared distances with 0x3ba0902d (csrc/vss_step.hip
    reset_field_split): the smallest float whose correctly rounded sqrt is >= 0.07f, so
    `d2 < T` is exactly the oracle's / reference's `sqrtf(d2) < 0.07` (envs/vss.py:293-298)."""
    c = np.float32(0.07)
    t = np.array([0x3ba0902d], dtype=np.uint32).view(np.float32)[0]
    below = np.nextafter(t, np.float32(0))
    assert np.sqrt(t) >= c and np.sqrt(below) < c
    # every float around the boundary (and a random sweep) classifies identically both ways
    around = (t.view(np.uint32) + np.arange(-4096, 4096, dtype=np.int64)).astype(np.uint32).view(np.float32)
    sweep = np.random.default_rng(0).uniform(0, 0.02, 200_000).astype(np.float32)
    for d2 in (around, sweep):
        assert np.array_equal(np.sqrt(d2) < c, d2 < t)


# --------------------------------------------------------------------------------- replay rows
def _reset_calls(g, steps_done):
    """(flat draws, env_ids, call sizes) of every reset_dones call a fixture recorded."""
    import replay_draws as RD
    n = g["init_state"].shape[1]
    sizes = RD.split_steps(g["u_sizes"], g["u_ncalls"])
    counts = [int(s.sum()) for s in sizes]
    yield g["init_uniforms"], np.arange(n), g["init_u_sizes"]
    for t, flat in enumerate(RD.split_steps(g["uniforms"], counts)):
        yield flat, np.nonzero(steps_done[t])[0], sizes[t]


@pytest.mark.parametrize("name", ["g4_full_rollout.npz", "g5_wrapped_sa.npz", "g5_wrapped_cma.npz", "g5_wrapped_dma.npz"])
def test_replay_rows_follow_reference_calls(golden_dir, name):
    """tests/replay_draws.py regroups the reference's batch-ordered reset draws into the per-field
    rows of vss_step_replay; the rejection rounds it derives must reproduce the sizes of every
    torch.rand call the reference made (envs/vss.py:283-325) and consume every draw."""
    import replay_draws as RD
    g = load(golden_dir, name)
    n = g["init_state"].shape[1]
    done = g["reset"] if "reset" in g else g["dones"][:, ::3 if "dma" in name else 1]
    calls = multi = 0
    for flat, ids, sz in _reset_calls(g, done):
        rows, rounds = RD.to_rows(flat, ids, n, call_sizes=sz)
        calls += len(ids) > 0
        multi += int((rounds > 1).sum())
        assert (rounds[ids] >= 1).all() and (np.delete(rounds, ids) == 0).all()
    assert calls >= 3, "fixture must exercise resets"
    if name.startswith("g4"):
        assert multi > 0, "G4 must exercise rejection re-draws (envs/vss.py:281-299)"
