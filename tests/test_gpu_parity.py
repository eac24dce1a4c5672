"""HIP step vs the CPU oracle, through the C ABI (needs a GPU: marked `gpu`).

Bar: bit-exact for every output — integers (progress, reset, time-outs, dones, rng counter)
and floats (state, observations, rewards) — because the kernel and the oracle evaluate the same
float32 operation sequence with FMA contraction off.  Free-running rollouts therefore stay
identical step after step (no teacher forcing needed).  At full size (65,536 fields) the tests
check size-independent properties (invariants, determinism, draw statistics).
"""
import numpy as np
import pytest
import torch

import oracle as O
from vss_amd import _native as N

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def make_vss(n, max_len=400, seed=1234, weights=(10.0, 2.0, 3.0, 0.0)):
    from envs.vss import VSS, default_cfg
    cfg = default_cfg(n)
    cfg["env"]["maxEpisodeLength"] = max_len
    cfg["env"]["seed"] = seed
    cfg["env"]["rew_weights"] = dict(goal=weights[0], grad=weights[1], move=weights[2], energy=weights[3])
    return VSS(cfg, DEV, DEV, 0, True, False, False)


def host_from(env) -> O.HostEnv:
    h = O.HostEnv(env.num_fields)
    h.state[:] = env.state.cpu().numpy()
    h.progress[:] = env.progress_buf.cpu().numpy()
    h.reset[:] = env.reset_buf.cpu().numpy()
    h.dof[:] = env.dof_velocity_buf.reshape(-1, 12).cpu().numpy()
    h.ctr[:] = env.rng_counter.cpu().numpy().view(np.uint32)
    return h


def oracle_params(env):
    return O.params(env.w_goal, env.w_grad, env.w_move, env.w_energy, env.clip_actions,
                    env.max_episode_length, env.seed)


def assert_env_equal(env, h, msg=""):
    torch.cuda.synchronize()
    np.testing.assert_array_equal(env.state.cpu().numpy(), h.state, err_msg=msg + " state")
    np.testing.assert_array_equal(env.progress_buf.cpu().numpy(), h.progress, err_msg=msg + " progress")
    np.testing.assert_array_equal(env.reset_buf.cpu().numpy(), h.reset, err_msg=msg + " reset")
    np.testing.assert_array_equal(env.dof_velocity_buf.reshape(-1, 12).cpu().numpy(), h.dof, err_msg=msg + " dof")
    np.testing.assert_array_equal(env.rng_counter.cpu().numpy().view(np.uint32), h.ctr, err_msg=msg + " ctr")


def bits(t):
    return t.detach().cpu().numpy().view(np.uint32) if t.dtype == torch.float32 else t.detach().cpu().numpy()


@pytest.mark.parametrize("n", [1, 63, 65, 4096])
def test_construction_reset_and_observe_bit_exact(n):
    env = make_vss(n)
    h = O.HostEnv(n)
    O.reset_dones(h, oracle_params(env))  # same template, external-reset purpose, ctr 0
    assert_env_equal(env, h, "ctor")
    for agents in (6, 3, 1):
        want = O.compute_obs(h, agents)
        got = env.compute_observations(torch.empty((n, agents, 52), device=DEV), agents)
        np.testing.assert_array_equal(bits(got).reshape(want.shape), want.view(np.uint32))


@pytest.mark.parametrize("n,steps,max_len", [(4096, 200, 50), (65, 120, 30), (1, 60, 9)])
def test_full_step_free_running_bit_exact(n, steps, max_len):
    """Config 2 of BASELINE.json at 4,096 fields: random actions, free-running, every step."""
    env = make_vss(n, max_len=max_len)
    h = host_from(env)
    prm = oracle_params(env)
    gen = np.random.default_rng(n)
    resets = goals = timeouts = 0
    for t in range(steps):
        a = gen.uniform(-1.3, 1.3, (n, 2, 3, 2)).astype(np.float32)
        if t % 17 == 5:  # push some balls into the goals (play.py-style external writes)
            k = max(1, n // 8)
            env.ball_pos[:k] = torch.tensor([0.74, 0.05], device=DEV)
            env.ball_vel[:k] = torch.tensor([1.0, 0.0], device=DEV)
            h.state[0, :k], h.state[1, :k], h.state[2, :k], h.state[3, :k] = 0.74, 0.05, 1.0, 0.0
        obs_dict, rew, reset, extras = env.step(torch.from_numpy(a).to(DEV))
        io = O.make_io(n, O.MODE_FULL)
        O.step(h, O.MODE_FULL, a.reshape(n, 12), io, prm)
        msg = f"step {t}"
        assert_env_equal(env, h, msg)
        np.testing.assert_array_equal(bits(obs_dict["obs"]).reshape(n, 312), io["obs"].view(np.uint32).reshape(n, 312), err_msg=msg)
        np.testing.assert_array_equal(bits(extras["terminal_observation"]).reshape(n, 312),
                                      io["terminal_obs"].view(np.uint32).reshape(n, 312), err_msg=msg)
        np.testing.assert_array_equal(bits(rew).reshape(n, 24), io["rew"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(extras["time_outs"].cpu().numpy().astype(np.uint8), io["time_outs"], err_msg=msg)
        np.testing.assert_array_equal(bits(extras["progress_buffer"]), io["progress_f"].view(np.uint32), err_msg=msg)
        resets += int(h.reset.sum())
        goals += int((np.abs(io["rew"][:, 0]) > 0).sum())
        timeouts += int(io["time_outs"].sum())
    assert resets > 0 and goals > 0 and timeouts > 0


def test_full_step_past_infinity_cache_bit_exact():
    """98,304 fields: the FULL footprint (3,101 B per field) is past the 256 MiB Infinity Cache, so
    the host sets nt_obs and the kernel streams `obs` with nontemporal stores (vss_step.hip,
    coop_store_obs).  Same bar as the free-running tests: every output bit-exact vs the oracle,
    over steps that include time-outs and resets."""
    n, steps = 98304, 3
    assert n > (256 << 20) // 3101
    env = make_vss(n, max_len=2)
    h = host_from(env)
    prm = oracle_params(env)
    gen = np.random.default_rng(7)
    resets = 0
    for t in range(steps):
        a = gen.uniform(-1.0, 1.0, (n, 2, 3, 2)).astype(np.float32)
        obs_dict, rew, reset, extras = env.step(torch.from_numpy(a).to(DEV))
        io = O.make_io(n, O.MODE_FULL)
        O.step(h, O.MODE_FULL, a.reshape(n, 12), io, prm)
        msg = f"step {t}"
        assert_env_equal(env, h, msg)
        np.testing.assert_array_equal(bits(obs_dict["obs"]).reshape(n, 312), io["obs"].view(np.uint32).reshape(n, 312), err_msg=msg)
        np.testing.assert_array_equal(bits(extras["terminal_observation"]).reshape(n, 312),
                                      io["terminal_obs"].view(np.uint32).reshape(n, 312), err_msg=msg)
        np.testing.assert_array_equal(bits(rew).reshape(n, 24), io["rew"].view(np.uint32), err_msg=msg)
        resets += int(h.reset.sum())
    assert resets > 0


@pytest.mark.parametrize("weights,clip", [((1.0, 0.0, 0.0, 0.0), 1.0),     # play.py's evaluation weights
                                          ((10.0, 2.0, 3.0, 0.5), 1.0),    # energy term on
                                          ((0.0, 0.0, 0.0, 0.0), 0.5),     # every term off, tighter clip
                                          ((10.0, 2.0, 3.0, 0.0), float("inf"))])  # no clip
def test_full_step_parameter_variants_bit_exact(weights, clip):
    """The reward-weight branches (a term is skipped when its weight is 0, envs/vss.py:240-258)
    and the VecTask action clamp, at parameters the other tests do not use; actions reach
    +-1.6 so the clamp is exercised."""
    n, steps = 257, 60
    env = make_vss(n, max_len=40, seed=77, weights=weights)
    env.clip_actions = clip
    h = host_from(env)
    prm = oracle_params(env)
    gen = np.random.default_rng(5)
    for t in range(steps):
        a = gen.uniform(-1.6, 1.6, (n, 2, 3, 2)).astype(np.float32)
        obs_dict, rew, reset, extras = env.step(torch.from_numpy(a).to(DEV))
        io = O.make_io(n, O.MODE_FULL)
        O.step(h, O.MODE_FULL, a.reshape(n, 12), io, prm)
        msg = f"step {t}"
        assert_env_equal(env, h, msg)
        np.testing.assert_array_equal(bits(obs_dict["obs"]).reshape(n, 312), io["obs"].view(np.uint32).reshape(n, 312), err_msg=msg)
        np.testing.assert_array_equal(bits(rew).reshape(n, 24), io["rew"].view(np.uint32), err_msg=msg)
    r = rew.cpu().numpy().reshape(n, 2, 3, 4)
    for c, w in enumerate(weights):
        if w == 0.0:
            assert np.all(r[..., c] == 0.0), c
    if weights[3] > 0:
        assert np.all(r[..., 3] <= 0.0) and np.any(r[..., 3] < 0.0)  # -mean|a| x w_energy
    d = env.dof_velocity_buf.cpu().numpy()
    assert np.all(np.abs(d) <= min(clip, 1.6) + 1e-7)


@pytest.mark.parametrize("mode", [O.MODE_SA, O.MODE_CMA, O.MODE_DMA])
@pytest.mark.parametrize("n", [4096, 67])
def test_wrapped_step_free_running_bit_exact(mode, n):
    from envs.wrappers import SingleAgent, CMA, DMA
    env = make_vss(n, max_len=40)
    W = {O.MODE_SA: SingleAgent, O.MODE_CMA: CMA, O.MODE_DMA: DMA}[mode](env)
    h = host_from(env)
    prm = oracle_params(env)
    gen = np.random.default_rng(100 + mode)
    rows = 3 * n if mode == O.MODE_DMA else n
    width = 6 if mode == O.MODE_CMA else 2
    io = O.make_io(n, mode)
    obs0 = W.reset()["obs"]
    np.testing.assert_array_equal(bits(obs0).reshape(-1), O.compute_obs(h, 3 if mode == O.MODE_DMA else 1).view(np.uint32).reshape(-1))
    for t in range(90):
        a = gen.uniform(-1.2, 1.2, (rows, width)).astype(np.float32)
        obs, reward, dones, info = W.step(torch.from_numpy(a).to(DEV))
        O.step(h, mode, a, io, prm)
        msg = f"mode {mode} step {t}"
        assert_env_equal(env, h, msg)
        np.testing.assert_array_equal(bits(W.action_buf).reshape(n, 12), io["ou_buf"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(bits(obs["obs"]).reshape(-1), io["obs"].view(np.uint32).reshape(-1), err_msg=msg)
        np.testing.assert_array_equal(bits(info["terminal_observation"]).reshape(-1), io["terminal_obs"].view(np.uint32).reshape(-1), err_msg=msg)
        np.testing.assert_array_equal(bits(info["rews"]).reshape(-1), io["rew"].view(np.uint32).reshape(-1), err_msg=msg)
        np.testing.assert_array_equal(bits(reward), io["reward_sum"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(info["time_outs"].cpu().numpy().astype(np.uint8), io["time_outs"], err_msg=msg)
        np.testing.assert_array_equal(bits(info["progress_buffer"]), io["progress_f"].view(np.uint32), err_msg=msg)
        want_dones = io["dones_rep"] if mode == O.MODE_DMA else h.reset
        np.testing.assert_array_equal(dones.cpu().numpy(), want_dones, err_msg=msg)
        assert tuple(obs["obs"].shape) == (rows, 52) and tuple(dones.shape) == (rows,)
    assert h.reset.sum() >= 0


def test_dma_65536_fields_config4_bit_exact():
    """BASELINE config 4: DMA at 65,536 fields = 196,608 agent rows (the reference needs
    num_envs % 3 == 0, envs/wrappers.py:30), free-running with episodes short enough to reset,
    every output bit-exact vs the oracle at full size, plus the DMA packing's shape contract."""
    from envs.wrappers import DMA
    n = 65536
    env = make_vss(n, max_len=12, seed=31)
    W = DMA(env)
    assert W.num_envs == 3 * n and env.num_envs == 3 * n  # DMA re-assigns num_environments (wrappers.py:154)
    h = host_from(env)
    prm = oracle_params(env)
    io = O.make_io(n, O.MODE_DMA)
    gen = torch.Generator(device=DEV).manual_seed(8)
    resets = 0
    for t in range(26):
        a = torch.rand((3 * n, 2), device=DEV, generator=gen) * 2.4 - 1.2
        obs, reward, dones, info = W.step(a)
        O.step(h, O.MODE_DMA, a.cpu().numpy(), io, prm)
        msg = f"step {t}"
        assert_env_equal(env, h, msg)
        np.testing.assert_array_equal(bits(W.action_buf).reshape(n, 12), io["ou_buf"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(bits(obs["obs"]), io["obs"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(bits(info["terminal_observation"]), io["terminal_obs"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(bits(info["rews"]), io["rew"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(bits(reward), io["reward_sum"].view(np.uint32), err_msg=msg)
        np.testing.assert_array_equal(dones.cpu().numpy(), io["dones_rep"], err_msg=msg)
        np.testing.assert_array_equal(info["time_outs"].cpu().numpy().astype(np.uint8), io["time_outs"], err_msg=msg)
        assert tuple(obs["obs"].shape) == (3 * n, 52) and tuple(reward.shape) == (3 * n,)
        d = dones.view(n, 3)
        assert torch.equal(d[:, 0], d[:, 1]) and torch.equal(d[:, 0], d[:, 2])  # repeat_interleave(3)
        resets += int(h.reset.sum())
    assert resets >= n  # every field has ended an episode at least once (max_len 12)


def test_external_reset_play_style():
    """play.py:132-133: envs.reset_buf[:] = 1; envs.reset_dones() re-samples every field."""
    n = 512
    env = make_vss(n)
    for _ in range(5):
        env.step(torch.zeros((n, 2, 3, 2), device=DEV))
    h = host_from(env)
    env.reset_buf[:] = 1
    h.reset[:] = 1
    env.reset_dones()
    O.reset_dones(h, oracle_params(env))
    assert_env_equal(env, h, "external reset")


def test_views_alias_state():
    """ball_pos / robots_pos / ... are writable views of the state the kernel reads."""
    env = make_vss(8)
    env.robots_pos[3, 1, 2] = torch.tensor([0.25, -0.125], device=DEV)
    env.ball_vel[2] = torch.tensor([0.5, 0.25], device=DEV)
    env.robots_quats[1, 0, 1] = torch.tensor([0.0, 0.0, 0.6, 0.8], device=DEV)
    s = env.state.cpu().numpy()
    assert s[N.CH_RX + 5, 3] == 0.25 and s[N.CH_RY + 5, 3] == -0.125
    assert s[N.CH_BALL_VX, 2] == 0.5 and s[N.CH_BALL_VY, 2] == 0.25
    assert s[N.CH_RQZ + 1, 1] == np.float32(0.6) and s[N.CH_RQW + 1, 1] == np.float32(0.8)
    assert tuple(env.robots_ang_vel.shape) == (8, 2, 3, 1)


def test_full_size_invariants_and_determinism():
    """65,536 fields (BASELINE config 3/4 size): bodies stay inside the walls, quaternions stay
    unit, no NaN, goals / time-outs bookkeeping is consistent, and the same seed gives the
    same bits."""
    n = 65536
    e1, e2 = make_vss(n, seed=77), make_vss(n, seed=77)
    gen = torch.Generator(device=DEV).manual_seed(5)
    for t in range(120):
        a = torch.rand((n, 2, 3, 2), device=DEV, generator=gen) * 2 - 1
        o1, r1, d1, x1 = e1.step(a)
        o2, r2, d2, x2 = e2.step(a)
    torch.cuda.synchronize()
    assert torch.equal(e1.state, e2.state) and torch.equal(o1["obs"], o2["obs"])
    s = e1.state
    assert torch.isfinite(s).all() and torch.isfinite(o1["obs"]).all()
    bx, by = s[0].abs(), s[1].abs()
    assert (by <= 0.65 + 1e-4).all() and (bx <= 0.85 + 1e-4).all()
    rx, ry = s[N.CH_RX:N.CH_RX + 6].abs(), s[N.CH_RY:N.CH_RY + 6].abs()
    assert (ry <= 0.65 - 0.04 + 1e-4).all() and (rx <= 0.85 - 0.04 + 1e-4).all()
    qn = s[N.CH_RQZ:N.CH_RQZ + 6] ** 2 + s[N.CH_RQW:N.CH_RQW + 6] ** 2
    assert ((qn - 1).abs() < 1e-5).all()
    assert (e1.progress_buf <= e1.max_episode_length).all()
    # resets happen exactly where a goal or the episode limit fired
    assert (x1["time_outs"] <= (d1 != 0)).all()


def test_reset_distribution_matches_reference_statistics():
    """Reset sampling (envs/vss.py:281-327): positions uniform in the +-field_scale/2 box with all
    21 pair distances >= 0.07, yaw uniform, ball velocity U[-0.5, 0.5)^2 — checked by moments
    over 65,536 fresh fields."""
    n = 65536
    env = make_vss(n, seed=99)
    s = env.state.cpu().numpy().astype(np.float64)
    xs = np.concatenate([s[0:1], s[N.CH_RX:N.CH_RX + 6]])
    ys = np.concatenate([s[1:2], s[N.CH_RY:N.CH_RY + 6]])
    assert np.abs(xs).max() <= 0.68 and np.abs(ys).max() <= 0.58
    d = np.sqrt((xs[:, None] - xs[None]) ** 2 + (ys[:, None] - ys[None]) ** 2)
    iu = np.triu_indices(7, 1)
    assert d[iu].min() >= 0.07
    # rejection conditions the marginals only slightly: mean ~0, var close to uniform's
    assert abs(xs.mean()) < 0.01 and abs(ys.mean()) < 0.01
    assert abs(xs.var() - 1.36 ** 2 / 12) < 0.01
    yaw = 2 * np.arctan2(s[N.CH_RQZ:N.CH_RQZ + 6], s[N.CH_RQW:N.CH_RQW + 6])
    yaw = (yaw + np.pi) % (2 * np.pi) - np.pi
    assert abs(yaw.mean()) < 0.02 and abs(yaw.var() - np.pi ** 2 / 3) < 0.05
    bv = s[2:4]
    assert np.abs(bv).max() <= 0.5 and abs(bv.var() - 1 / 12) < 0.002
    assert (s[N.CH_RVX:N.CH_RVX + 12] == 0).all() and (s[N.CH_RW:N.CH_RW + 6] == 0).all()


def test_ou_noise_statistics():
    """OU opponents (envs/wrappers.py:5-19): one step from zero gives clamp(N(0, 0.15^2))."""
    from envs.wrappers import SingleAgent
    n = 65536
    env = make_vss(n, seed=5)
    W = SingleAgent(env)
    W.step(torch.zeros((n, 2), device=DEV))
    ab = W.action_buf.reshape(n, 12).cpu().numpy().astype(np.float64)
    done = env.reset_buf.cpu().numpy().astype(bool)
    z = ab[~done][:, 2:]
    assert np.all(ab[:, :2][~done] == 0)
    assert abs(z.mean()) < 2e-3 and abs(z.std() - 0.15) < 2e-3
    # 4th moment of a normal: 3 sigma^4
    assert abs((z ** 4).mean() / 0.15 ** 4 - 3.0) < 0.1


def test_graph_replay_matches_eager():
    """vss_step captured into a hipGraph and replayed gives the same bits as eager launches (the
    per-field RNG counters live in device memory, so replays draw fresh randoms)."""
    n = 4096
    e1, e2 = make_vss(n, max_len=25, seed=3), make_vss(n, max_len=25, seed=3)
    acts = [torch.rand((n, 12), device=DEV) * 2 - 1 for _ in range(4)]
    lib = N.load()
    io2 = N.VssStepIO(0, None, e2.obs_buf.data_ptr(), e2.terminal_obs_buf.data_ptr(), e2.rew_buf.data_ptr(), None,
                      None, e2.timeout_buf.data_ptr(), e2.progress_f_buf.data_ptr())
    prm, st = e2._c_params(), e2._c_state()
    ios = []
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=s):
        for a in acts:
            io = N.VssStepIO.from_buffer_copy(io2)
            io.actions = a.data_ptr()
            ios.append(io)
            assert lib.vss_step(N.stream_of(torch.device(DEV)), n, 0, N.ctypes.byref(prm), N.ctypes.byref(st),
                                N.ctypes.byref(io)) == 0
    for rep in range(15):  # 60 steps: crosses two time-out waves (max_len 25)
        g.replay()
        for a in acts:
            e1.step(a)
    torch.cuda.synchronize()
    assert torch.equal(e1.state, e2.state)
    assert torch.equal(e1.obs_buf, e2.obs_buf) and torch.equal(e1.rew_buf, e2.rew_buf)
    assert torch.equal(e1.progress_buf, e2.progress_buf) and torch.equal(e1.rng_counter, e2.rng_counter)


def test_zero_fields_is_a_noop():
    lib = N.load()
    env = make_vss(4)
    prm, st = env._c_params(), env._c_state()
    io = N.VssStepIO(env.obs_buf.data_ptr(), None, env.obs_buf.data_ptr(), env.terminal_obs_buf.data_ptr(),
                     env.rew_buf.data_ptr(), None, None, env.timeout_buf.data_ptr(), env.progress_f_buf.data_ptr())
    before = env.state.clone()
    assert lib.vss_step(N.stream_of(env.device), 0, 0, N.ctypes.byref(prm), N.ctypes.byref(st), N.ctypes.byref(io)) == 0
    torch.cuda.synchronize()
    assert torch.equal(before, env.state)


def test_c_abi_rejects_misaligned_vector_buffers():
    """Straight through the C ABI: an obs or action pointer 4 B off its 16-B alignment is refused
    with VSS_E_ARG (the kernels move float4 vectors), the aligned call succeeds."""
    lib = N.load()
    env = make_vss(64)
    prm, st = env._c_params(), env._c_state()
    acts = torch.zeros(64 * 12 + 4, device=DEV)
    obs = torch.zeros(64 * 312 + 4, device=DEV)

    def call(a_off, o_off):
        io = N.VssStepIO(acts.data_ptr() + a_off, None, obs.data_ptr() + o_off, env.terminal_obs_buf.data_ptr(),
                         env.rew_buf.data_ptr(), None, None, env.timeout_buf.data_ptr(), env.progress_f_buf.data_ptr())
        return lib.vss_step(N.stream_of(env.device), 64, 0, N.ctypes.byref(prm), N.ctypes.byref(st), N.ctypes.byref(io))

    assert call(0, 4) == 1 and call(4, 0) == 1 and call(8, 0) == 1
    assert call(0, 0) == 0
    torch.cuda.synchronize()


def test_host_layer_rejects_bad_buffers_before_launch():
    """The kernels trust their pointers, so the env layer checks every caller buffer (size,
    dtype, device, contiguity) and raises before launching; the state is left untouched."""
    n = 64
    env = make_vss(n)
    before = env.state.clone()
    acts = torch.zeros((n, 2, 3, 2), device=DEV)
    good = dict(obs=env.obs_buf, terminal_obs=env.terminal_obs_buf, rew=env.rew_buf, reward_sum=None,
                time_outs=env.timeout_buf, progress_f=env.progress_f_buf)
    bad = [dict(good, obs=torch.zeros((n - 1, 2, 3, 52), device=DEV)),          # short
           dict(good, rew=torch.zeros((n, 2, 3, 4), device=DEV, dtype=torch.float64)),  # dtype
           dict(good, time_outs=torch.zeros(n, device=DEV)),                          # float, not bool
           dict(good, terminal_obs=torch.zeros((n, 2, 3, 104), device=DEV)[..., ::2]),  # strided
           dict(good, progress_f=torch.zeros(n))]                                     # host memory
    for io in bad:
        with pytest.raises(ValueError):
            env.native_step(N.MODE_FULL, acts, io)
    with pytest.raises(ValueError):  # wrapped modes need the OU buffer and reward_sum
        env.native_step(N.MODE_SA, torch.zeros((n, 2), device=DEV), dict(good, obs=torch.zeros((n, 52), device=DEV)))
    with pytest.raises(ValueError):
        env.native_step(N.MODE_FULL, torch.zeros((n + 1, 12), device=DEV), good)
    with pytest.raises(ValueError):
        env.rollout(torch.zeros((4, n, 2, 3, 2), device=DEV), out=dict(
            obs=torch.zeros((3, n, 2, 3, 52), device=DEV)))
    with pytest.raises(ValueError):
        env.compute_observations(out=torch.zeros((n, 52), device=DEV), n_agents=3)
    with pytest.raises(ValueError):
        env.compute_observations(n_agents=2)
    torch.cuda.synchronize()
    assert torch.equal(before, env.state)
    env.native_step(N.MODE_FULL, acts, good)  # and the good set still steps


@pytest.mark.parametrize("n,K", [(4096, 24), (65, 50)])
def test_rollout_equals_sequential_steps_and_oracle(n, K):
    """vss_rollout (K steps per launch) == K vss_step launches == K oracle steps, bit for bit."""
    e1, e2 = make_vss(n, max_len=20, seed=11), make_vss(n, max_len=20, seed=11)
    h = host_from(e1)
    prm = oracle_params(e1)
    acts = (torch.rand((K, n, 2, 3, 2), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4)) * 2.6 - 1.3)
    out = e2.rollout(acts)
    a_np = acts.cpu().numpy()
    for k in range(K):
        o, r, d, x = e1.step(acts[k])
        io = O.make_io(n, O.MODE_FULL)
        O.step(h, O.MODE_FULL, a_np[k].reshape(n, 12), io, prm)
        torch.cuda.synchronize()
        assert torch.equal(out["obs"][k], o["obs"]) and torch.equal(out["terminal_observation"][k], x["terminal_observation"])
        assert torch.equal(out["rew"][k], r) and torch.equal(out["dones"][k], d)
        assert torch.equal(out["time_outs"][k], x["time_outs"]) and torch.equal(out["progress_buffer"][k], x["progress_buffer"])
        np.testing.assert_array_equal(bits(out["obs"][k]).reshape(n, 312), io["obs"].view(np.uint32).reshape(n, 312))
        np.testing.assert_array_equal(out["dones"][k].cpu().numpy(), h.reset)
    for name in ("state", "progress_buf", "reset_buf", "dof_velocity_buf", "rng_counter"):
        assert torch.equal(getattr(e1, name), getattr(e2, name)), name
    assert_env_equal(e2, h, "after rollout")
    assert int(out["dones"].sum()) > 0


def test_returned_buffers_are_persistent_documented_semantics():
    """obs_dict['obs'], rew_buf, reset_buf and extras[...] are persistent buffers
    that the next step overwrites in place (the reference rebinds reset_buf and clones obs /
    terminal obs, envs/vss.py:196,198,258-265); callers that keep a step's outputs must clone."""
    n = 64
    env = make_vss(n, max_len=5)
    a = torch.zeros((n, 2, 3, 2), device=DEV)
    o1, r1, d1, x1 = env.step(a)
    kept = {k: t.clone() for k, t in (("obs", o1["obs"]), ("rew", r1), ("reset", d1),
                                      ("term", x1["terminal_observation"]), ("prog", x1["progress_buffer"]))}
    ptrs = (o1["obs"].data_ptr(), r1.data_ptr(), d1.data_ptr(), x1["terminal_observation"].data_ptr(),
            x1["progress_buffer"].data_ptr(), x1["time_outs"].data_ptr())
    for _ in range(4):  # progress reaches max_len: every field resets
        o2, r2, d2, x2 = env.step(a)
    assert ptrs == (o2["obs"].data_ptr(), r2.data_ptr(), d2.data_ptr(), x2["terminal_observation"].data_ptr(),
                    x2["progress_buffer"].data_ptr(), x2["time_outs"].data_ptr())
    assert o1["obs"] is o2["obs"] and d1 is env.reset_buf
    assert not torch.equal(kept["reset"], d1) and not torch.equal(kept["prog"], x1["progress_buffer"])
    assert not torch.equal(kept["obs"], o1["obs"])  # overwritten in place by the later steps


@pytest.mark.parametrize("mode", [O.MODE_SA, O.MODE_DMA])
def test_wrapped_modes_leave_vss_obs_and_rew_bufs_stale(mode):
    """the fused SA/CMA/DMA kernels write only the learner rows into the wrapper's
    own buffers; VSS.obs_buf / rew_buf keep their last FULL-mode contents (the reference's
    wrappers never read them after slicing, envs/wrappers.py:101-180)."""
    from envs.wrappers import DMA, SingleAgent
    n = 64
    env = make_vss(n)
    W = (SingleAgent if mode == O.MODE_SA else DMA)(env)
    before_obs, before_rew = env.obs_buf.clone(), env.rew_buf.clone()
    rows = n * (3 if mode == O.MODE_DMA else 1)
    for _ in range(3):
        obs, reward, dones, info = W.step(torch.rand((rows, 2), device=DEV) * 2 - 1)
    torch.cuda.synchronize()
    assert torch.equal(env.obs_buf, before_obs) and torch.equal(env.rew_buf, before_rew)
    # while the wrapper's outputs are current: they equal a fresh compute_obs of the blue rows
    agents = 3 if mode == O.MODE_DMA else 1
    fresh = env.compute_observations(torch.empty((n, agents, 52), device=DEV), agents)
    assert torch.equal(obs["obs"].view(n, agents, 52), fresh)
