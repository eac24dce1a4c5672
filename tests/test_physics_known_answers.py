"""Known answers for the 2D physics that replaces PhysX.

PhysX is closed and absent, so trajectory parity with the reference is unpinned; these tests pin
the build's model to the quantities the reference's own configuration implies:

  * straight drive: wheel target = action x 42 rad/s (envs/vss.py:48,186) on wheels of radius
    0.024 m (envs/vss_robot.urdf:28-33) -> terminal speed 1.008 m/s along the heading;
  * spin in place: wheels at y = +-0.03375 m (vss_robot.urdf:54-63) -> yaw rate
    2 x 1.008 / 0.0675 = 29.87 rad/s, no translation;
  * walls (envs/vss.py:449-518): side walls from |y| = 0.65, end walls from |x| = 0.75 beside the
    goal mouth (|y| >= 0.2), goal-pocket back walls from |x| = 0.85; restitution 0
    (envs/vss.py:375) -> bodies stop with their surface on the plane (robot disc r = 0.04, ball
    r = 0.02134, envs/vss.py:383) and no rebound;
  * the 180-degree mirror (envs/vss.py:533-560): the yellow view of a rotated, team-swapped state
    is the blue view of the original, and the dynamics commute with that symmetry;
  * robot-robot contact (bodies collide, envs/vss.py:404-425): a symmetric head-on push keeps
    the pair symmetric, conserves momentum and never interpenetrates;
  * ball-robot contact: a driving robot kicks a resting ball forward;
plus the model's own spec constants (traction-limited wheel acceleration 6 m/s^2 = 0.15 m/s per
0.025 s substep, ball rolling damping 0.15 1/s), so a changed constant fails here.

Every scenario runs on the CPU oracle (oracle/vss_oracle.c, physics only) and, as a `gpu` twin,
through the HIP kernel's `VSS.step` (FULL contract; no scenario scores a goal, so no reset
interferes).  The ball-into-goal case runs on the oracle only: a goal ends the episode in the
kernel's step (envs/vss.py:634-655), so its pocket walls are exercised there by a robot instead.
"""
import math

import numpy as np
import pytest

import oracle as O

F = np.float32
DT = 0.05
V_MAX = 42.0 * 0.024                       # 1.008 m/s
W_MAX = 2.0 * V_MAX / (2 * 0.03375)        # 29.8667 rad/s
ROBOT_R, BALL_R = 0.04, 0.02134

# bodies parked out of the way: (x, y) for robots 0..5 and the ball
PARK = [(-0.6, -0.5), (-0.6, 0.5), (0.0, -0.5), (0.6, -0.5), (0.6, 0.5), (0.3, 0.5)]
BALL_PARK = (-0.45, 0.25)


def make_state(n):
    s = np.zeros((O.STATE_CHANNELS, n), F)
    for r, (x, y) in enumerate(PARK):
        s[O.CH_RX + r], s[O.CH_RY + r] = x, y
    s[O.CH_RQW:O.CH_RQW + 6] = 1.0
    s[0], s[1] = BALL_PARK
    return s


def set_robot(s, f, r, x, y, yaw, vx=0.0, vy=0.0, w=0.0):
    s[O.CH_RX + r, f], s[O.CH_RY + r, f] = x, y
    s[O.CH_RQZ + r, f], s[O.CH_RQW + r, f] = math.sin(yaw / 2), math.cos(yaw / 2)
    s[O.CH_RVX + r, f], s[O.CH_RVY + r, f], s[O.CH_RW + r, f] = vx, vy, w


def set_ball(s, f, x, y, vx=0.0, vy=0.0):
    s[0, f], s[1, f], s[2, f], s[3, f] = x, y, vx, vy


def yaw_of(s, r):
    return 2.0 * np.arctan2(s[O.CH_RQZ + r].astype(np.float64), s[O.CH_RQW + r].astype(np.float64))


# ---------------------------------------------------------------------------------- runners
def run_oracle(state, actions):
    """Physics only (the fake gym.simulate hook): trajectory (K + 1, 58, n)."""
    s = state.copy()
    traj = [s.copy()]
    for a in actions:
        O.simulate(s, np.clip(a, -1, 1).reshape(s.shape[1], 12))
        traj.append(s.copy())
    return np.stack(traj)


def run_hip(state, actions):
    """The HIP step kernel through VSS.step (FULL contract), episodes long enough not to end."""
    import torch
    from envs.vss import VSS, default_cfg
    n = state.shape[1]
    cfg = default_cfg(n)
    cfg["env"]["maxEpisodeLength"] = 1_000_000
    env = VSS(cfg, "cuda:0", "cuda:0", 0, True, False, False)
    env.state.copy_(torch.from_numpy(state))
    env.reset_buf.zero_()
    env.progress_buf.zero_()
    traj = [state.copy()]
    for a in actions:
        _, _, reset, _ = env.step(torch.from_numpy(np.ascontiguousarray(a, F)).cuda())
        assert int(reset.sum()) == 0, "a known-answer scenario must not end an episode"
        traj.append(env.state.cpu().numpy())
    return np.stack(traj)


BACKENDS = [pytest.param(run_oracle, id="oracle"), pytest.param(run_hip, id="hip", marks=pytest.mark.gpu)]


def actions_for(n, k, per_field):
    """(k, n, 2, 3, 2) actions: zero except robot -> (left, right) per field from per_field."""
    a = np.zeros((k, n, 2, 3, 2), F)
    for f, (r, left, right) in enumerate(per_field):
        a[:, f, r // 3, r % 3] = (left, right)
    return a


# ---------------------------------------------------------------------------------- drive
@pytest.mark.parametrize("run", BACKENDS)
def test_straight_drive_reaches_wheel_limited_speed(run):
    """a = +-1 on both wheels: |v| -> 42 rad/s x 0.024 m = 1.008 m/s along the heading, no yaw."""
    yaws = [0.0, math.pi / 2, math.pi - 1e-3, -math.pi / 4, 2.0]
    signs = [1, 1, 1, -1, -1]
    n = len(yaws)
    s = make_state(n)
    for f, yaw in enumerate(yaws):
        set_robot(s, f, 0, 0.0, 0.0, yaw)
        s[O.CH_RX + 2, f], s[O.CH_RY + 2, f] = 0.45, -0.55  # clear robot 0's path
    k = 7
    traj = run(s, actions_for(n, k, [(0, sg, sg) for sg in signs]))
    end = traj[-1]
    for f, (yaw, sg) in enumerate(zip(yaws, signs)):
        v = np.array([end[O.CH_RVX, f], end[O.CH_RVY, f]], np.float64)
        assert abs(np.linalg.norm(v) - V_MAX) < 2e-5, (f, v)
        np.testing.assert_allclose(v, sg * V_MAX * np.array([math.cos(yaw), math.sin(yaw)]), atol=2e-5)
        assert abs(end[O.CH_RW, f]) < 1e-4
        assert abs(math.remainder(yaw_of(end, 0)[f] - yaw, 2 * math.pi)) < 1e-5
    # the model's traction limit (spec): +0.15 m/s per 0.025 s substep from rest
    sp = [float(np.hypot(traj[t][O.CH_RVX, 0], traj[t][O.CH_RVY, 0])) for t in range(5)]
    np.testing.assert_allclose(sp, [0.0, 0.30, 0.60, 0.90, V_MAX], atol=1e-6)


@pytest.mark.parametrize("run", BACKENDS)
def test_spin_in_place_reaches_track_limited_yaw_rate(run):
    """(left, right) = (-1, +1): yaw rate -> 2 x 1.008 / 0.0675 = 29.87 rad/s, counter-clockwise
    (left wheel at +y, vss_robot.urdf:54-55), no translation; (+1, -1) spins the other way."""
    n = 2
    s = make_state(n)
    for f in range(n):
        set_robot(s, f, 0, 0.1, -0.1, 0.3)
    k = 8
    traj = run(s, actions_for(n, k, [(0, -1.0, 1.0), (0, 1.0, -1.0)]))
    for f, sign in enumerate((1.0, -1.0)):
        w = traj[:, O.CH_RW, f]
        assert abs(w[-1] - sign * W_MAX) < 1e-3, w[-1]
        assert abs(W_MAX - 29.8667) < 1e-4
        assert np.abs(traj[:, O.CH_RX, f] - F(0.1)).max() < 1e-5 and np.abs(traj[:, O.CH_RY, f] - F(-0.1)).max() < 1e-5
        assert np.abs(traj[:, O.CH_RVX, f]).max() < 1e-5 and np.abs(traj[:, O.CH_RVY, f]).max() < 1e-5
        # traction-limited spin-up: each wheel's rim speed moves 0.15 m/s per substep toward its
        # target, so the yaw rate climbs by 2 x 0.15 / 0.0675 = 4.444 rad/s per substep
        np.testing.assert_allclose(w[:5], sign * np.array([0.0, 8.888889, 17.777779, 26.666668, W_MAX]), atol=2e-4)
        # at the terminal rate the heading turns by w * dt per control step
        dyaw = [math.remainder(yaw_of(traj[t + 1], 0)[f] - yaw_of(traj[t], 0)[f], 2 * math.pi) for t in (5, 6, 7)]
        np.testing.assert_allclose(dyaw, sign * math.remainder(W_MAX * DT, 2 * math.pi), atol=2e-4)


# ---------------------------------------------------------------------------------- ball
@pytest.mark.parametrize("run", BACKENDS)
def test_free_rolling_ball_damping(run):
    """A free ball keeps its direction and slows by the spec's rolling damping, 0.15 1/s: v(t) =
    v0 (1 - 0.15 h)^(t / h) with h = 0.025 s, ~ v0 exp(-0.15 t); it moves by sum(v h)."""
    n = 2
    s = make_state(n)
    set_ball(s, 0, -0.3, 0.0, 0.4, 0.1)
    set_ball(s, 1, 0.2, -0.2, -0.1, 0.25)
    k = 20
    traj = run(s, np.zeros((k, n, 2, 3, 2), F))
    for f in range(n):
        v0 = traj[0, 2:4, f].astype(np.float64)
        vk = traj[-1, 2:4, f].astype(np.float64)
        np.testing.assert_allclose(vk, v0 * (1 - 0.15 * 0.025) ** (2 * k), rtol=2e-6)
        np.testing.assert_allclose(vk, v0 * math.exp(-0.15 * k * DT), rtol=1e-3)
        # exact float recurrence of the spec: v <- v * 0.99625; x <- x + v * h, twice per step
        x, v = traj[0, 0:2, f].copy(), traj[0, 2:4, f].copy()
        for _ in range(2 * k):
            v = v * F(0.99625)
            x = x + v * F(0.025)
        np.testing.assert_array_equal(traj[-1, 0:2, f], x)
        np.testing.assert_array_equal(traj[-1, 2:4, f], v)


# ---------------------------------------------------------------------------------- walls
WALL_CASES = [
    # (robot start x, y, yaw, expected stop coordinate index, value)  -- robot 0 at full speed
    ((0.40, 0.45, 0.0), "x", 0.75 - ROBOT_R),              # end wall beside the goal mouth
    ((-0.40, -0.45, math.pi), "x", -(0.75 - ROBOT_R)),
    ((0.10, 0.30, math.pi / 2), "y", 0.65 - ROBOT_R),      # side wall
    ((-0.10, -0.30, -math.pi / 2), "y", -(0.65 - ROBOT_R)),
    ((0.55, 0.00, 0.0), "x", 0.85 - ROBOT_R),              # into the goal pocket: back wall
    ((-0.55, 0.05, math.pi), "x", -(0.85 - ROBOT_R)),
]


@pytest.mark.parametrize("run", BACKENDS)
def test_robot_stops_at_wall_planes(run):
    n = len(WALL_CASES)
    s = make_state(n)
    for f, ((x, y, yaw), _, _) in enumerate(WALL_CASES):
        set_robot(s, f, 0, x, y, yaw)
        for r in range(1, 6):  # park the others in the opposite half, clear of robot 0
            s[O.CH_RX + r, f] = -0.3 * np.sign(x) + (r - 3) * 0.1
            s[O.CH_RY + r, f] = -0.3 * np.sign(y or 1.0)
        set_ball(s, f, -0.5 * np.sign(x), 0.55 * np.sign(-(y or 1.0)))
    k = 16
    traj = run(s, actions_for(n, k, [(0, 1.0, 1.0)] * n))
    end = traj[-1]
    for f, (_, axis, want) in enumerate(WALL_CASES):
        ch, vch = (O.CH_RX, O.CH_RVX) if axis == "x" else (O.CH_RY, O.CH_RVY)
        assert abs(end[ch, f] - want) < 1e-6, (f, end[ch, f], want)
        assert end[vch, f] == 0.0, (f, end[vch, f])  # restitution 0: no rebound
        # never beyond the plane on the way
        assert (np.abs(traj[:, ch, f]) <= abs(want) + 1e-6).all()
    # inside the pocket the side faces |y| = 0.2 also bound a robot: it stays within |y| <= 0.16
    assert abs(end[O.CH_RY, 4]) <= 0.2 - ROBOT_R + 1e-6


@pytest.mark.parametrize("run", BACKENDS)
def test_ball_stops_at_end_and_side_walls(run):
    cases = [((0.55, 0.45, 1.5, 0.0), 0, 0.75 - BALL_R), ((-0.55, -0.45, -1.5, 0.0), 0, -(0.75 - BALL_R)),
             ((0.2, 0.45, 0.0, 1.5), 1, 0.65 - BALL_R), ((0.2, -0.45, 0.0, -1.5), 1, -(0.65 - BALL_R))]
    n = len(cases)
    s = make_state(n)
    for f, (b, _, _) in enumerate(cases):
        set_ball(s, f, *b)
    traj = run(s, np.zeros((6, n, 2, 3, 2), F))
    for f, (_, ax, want) in enumerate(cases):
        assert abs(traj[-1, ax, f] - want) < 1e-6 and traj[-1, 2 + ax, f] == 0.0
        assert (np.abs(traj[:, ax, f]) <= abs(want) + 1e-6).all()


def test_ball_into_goal_stops_at_pocket_back_wall():
    """Oracle only (a goal ends the episode in the step kernel): past the goal line the ball is
    bounded by the pocket's back wall at |x| = 0.85 and its side faces at |y| = 0.2."""
    s = make_state(2)
    set_ball(s, 0, 0.6, 0.05, 2.0, 0.0)
    set_ball(s, 1, -0.6, -0.1, -2.0, -0.6)
    traj = run_oracle(s, np.zeros((6, 2, 2, 3, 2), F))
    assert abs(traj[-1, 0, 0] - (0.85 - BALL_R)) < 1e-6 and traj[-1, 2, 0] == 0.0
    assert abs(traj[-1, 0, 1] + (0.85 - BALL_R)) < 1e-6 and abs(traj[-1, 1, 1]) <= 0.2 - BALL_R + 1e-6
    assert (np.abs(traj[:, 0, :]) > 0.75).any(axis=0).all()  # they did cross the goal line


# ---------------------------------------------------------------------------------- symmetry
def rot180_swap(s):
    """Rotate a (58, n) state by 180 degrees about the centre and swap the teams."""
    m = np.empty_like(s)
    m[0:4] = -s[0:4]
    for r in range(6):
        q = (r + 3) % 6  # blue r <-> yellow r
        m[O.CH_RX + q], m[O.CH_RY + q] = -s[O.CH_RX + r], -s[O.CH_RY + r]
        m[O.CH_RVX + q], m[O.CH_RVY + q] = -s[O.CH_RVX + r], -s[O.CH_RVY + r]
        m[O.CH_RW + q] = s[O.CH_RW + r]
        # yaw + pi: (qz, qw) -> (qw, -qz)
        m[O.CH_RQZ + q], m[O.CH_RQW + q] = s[O.CH_RQW + r], -s[O.CH_RQZ + r]
        m[O.CH_RQX + q], m[O.CH_RQY + q] = s[O.CH_RQX + r], s[O.CH_RQY + r]
    return m


def separated_states(n, seed):
    """Random states with every body pair far enough apart that no contact happens in a step."""
    gen = np.random.default_rng(seed)
    s = np.zeros((O.STATE_CHANNELS, n), F)
    for f in range(n):
        while True:
            p = np.c_[gen.uniform(-0.62, 0.62, 7), gen.uniform(-0.52, 0.52, 7)]
            d = np.linalg.norm(p[:, None] - p[None], axis=-1) + np.eye(7)
            if d.min() > 0.25:
                break
        s[0, f], s[1, f] = p[0]
        s[2:4, f] = gen.uniform(-0.6, 0.6, 2)
        for r in range(6):
            yaw = gen.uniform(-math.pi, math.pi)
            set_robot(s, f, r, p[1 + r, 0], p[1 + r, 1], yaw, *gen.uniform(-0.8, 0.8, 2), gen.uniform(-20, 20))
    return s


def test_yellow_view_of_mirrored_state_is_blue_view():
    """compute_obs mirror (envs/vss.py:533-560): obs[yellow r](rot180_swap(S), swapped actions)
    == obs[blue r](S), bit for bit (the quaternion mirror (qz, qw) -> (qw, -qz) negates the
    algebraic cos / sin exactly)."""
    n = 64
    s = separated_states(n, 3)
    a = np.random.default_rng(4).uniform(-1, 1, (n, 2, 3, 2)).astype(F)
    h, hm = O.HostEnv(n), O.HostEnv(n)
    h.state[:] = s
    h.dof[:] = a.reshape(n, 12)
    hm.state[:] = rot180_swap(s)
    hm.dof[:] = a[:, ::-1].reshape(n, 12)
    obs, obs_m = O.compute_obs(h, 6).reshape(n, 2, 3, 52), O.compute_obs(hm, 6).reshape(n, 2, 3, 52)
    np.testing.assert_array_equal(obs_m[:, 1].view(np.uint32), obs[:, 0].view(np.uint32))
    np.testing.assert_array_equal(obs_m[:, 0].view(np.uint32), obs[:, 1].view(np.uint32))


@pytest.mark.parametrize("run", BACKENDS)
def test_dynamics_commute_with_the_mirror(run):
    """step(rot180_swap(S), swapped actions) == rot180_swap(step(S, actions)) bit for bit for
    contact-free states (drive, integration, damping and the folded walls are exactly odd in x, y)."""
    n = 48
    s = separated_states(n, 5)
    a = np.random.default_rng(6).uniform(-1, 1, (1, n, 2, 3, 2)).astype(F)
    t1 = run(s, a)[-1]
    t2 = run(rot180_swap(s), a[:, :, ::-1].copy())[-1]
    live = [c for c in range(O.STATE_CHANNELS) if not (O.CH_RQX <= c < O.CH_RQZ)]
    np.testing.assert_array_equal(t2[live].view(np.uint32), rot180_swap(t1)[live].view(np.uint32))


# ---------------------------------------------------------------------------------- contacts
@pytest.mark.parametrize("run", BACKENDS)
def test_symmetric_head_on_push(run):
    """Blue 0 and yellow 0 drive into each other at full speed: they meet, stay mirror images of
    each other about x = 0, keep zero total momentum (equal masses, equal and opposite impulses)
    and never overlap (discs of r = 0.04)."""
    n = 1
    s = make_state(n)
    set_robot(s, 0, 0, -0.15, 0.0, 0.0)
    set_robot(s, 0, 3, 0.15, 0.0, math.pi)
    k = 10
    a = np.zeros((k, n, 2, 3, 2), F)
    a[:, 0, 0, 0] = (1.0, 1.0)
    a[:, 0, 1, 0] = (1.0, 1.0)
    traj = run(s, a)
    x0, x3 = traj[:, O.CH_RX, 0], traj[:, O.CH_RX + 3, 0]
    np.testing.assert_allclose(x0, -x3, atol=1e-6)
    np.testing.assert_allclose(traj[:, O.CH_RVX, 0] + traj[:, O.CH_RVX + 3, 0], 0.0, atol=1e-6)
    assert (x3 - x0 >= 2 * ROBOT_R - 1e-6).all()
    assert abs((x3 - x0)[-1] - 2 * ROBOT_R) < 1e-5  # they end pressed together
    np.testing.assert_allclose(traj[:, O.CH_RY, 0], 0.0, atol=1e-6)


@pytest.mark.parametrize("run", BACKENDS)
def test_robot_kicks_resting_ball_forward(run):
    """A robot driving at a resting ball pushes it ahead: after contact the ball is in front of
    the robot's face (0.035 m half-width + ball radius), moving forward at least as fast as the
    robot (perfectly inelastic normal contact), and keeps rolling when the robot stops."""
    n = 1
    s = make_state(n)
    set_robot(s, 0, 0, -0.3, 0.0, 0.0)
    set_ball(s, 0, -0.1, 0.0)
    k = 12
    a = np.zeros((k, n, 2, 3, 2), F)
    a[:6, 0, 0, 0] = (1.0, 1.0)
    traj = run(s, a)
    t_hit = 4  # the robot covers 0.2 - 0.035 - 0.021 m within 4 steps at <= 1.008 m/s
    bx, rx = traj[:, 0, 0], traj[:, O.CH_RX, 0]
    assert (bx[t_hit:] - rx[t_hit:] >= 0.035 + BALL_R - 1e-5).all()
    assert traj[6, 2, 0] >= traj[6, O.CH_RVX, 0] - 1e-6 and traj[6, 2, 0] > 0.5
    assert abs(traj[6, 3, 0]) < 1e-6 and (np.diff(bx[6:]) > 0).all()
