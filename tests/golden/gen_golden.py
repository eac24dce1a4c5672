#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own Python.

Runs only in the build container (it imports /root/reference, which does not exist on the
GPU box).  Nothing of the reference is copied: the reference is imported as-is from
/root/reference and only arrays (inputs + the reference's outputs) are written.

The reference needs Isaac Gym / IsaacGymEnvs / gym / hydra, none of which are installed, so
this script provides stub modules:
  * gym: Wrapper / ObservationWrapper / spaces.Box;
  * isaacgym.gymapi: a fake scene recorder whose `simulate` is a physics HOOK;
  * isaacgym.gymtorch: identity wrap/unwrap;
  * isaacgym.torch_utils: get_euler_xyz / quat_from_angle_axis / torch_rand_float, restated
    from public Isaac Gym (Ext);
  * isaacgymenvs...VecTask: restated VecTask.__init__/step/reset (Ext, IsaacGymEnvs @ dee7c567);
  * torch.utils.tensorboard: SummaryWriter stub (only for importing `Agent`).
The physics hook is the build's CPU oracle (oracle/oracle.py `simulate`): PhysX is closed and
absent, so the dynamics are the build's own model; everything else (pre/post physics step,
rewards, dones, obs, reset sampling, OU wrappers, time-outs) is the reference's own code.
All torch.rand / torch.normal draws are recorded so the oracle can replay them.

Usage:  python tests/golden/gen_golden.py [g1 g4 g5 g6]   (writes tests/golden/*.npz; default all)
"""
from __future__ import annotations

import os
import sys
import tempfile
import textwrap
import types

os.environ["PYTORCH_JIT"] = "0"  # compute_obs is @torch.jit.script; eager lets us redirect cuda:0

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

# ----------------------------------------------------------------------------------------------
# stubs
# ----------------------------------------------------------------------------------------------
STUB_GYM = '''
import numpy as np
class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype
class Wrapper:
    def __init__(self, env):
        self.env = env
        self._action_space = None
        self._observation_space = None
    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)
    @property
    def action_space(self):
        return self._action_space if self._action_space is not None else self.env.action_space
    @action_space.setter
    def action_space(self, v):
        self._action_space = v
    @property
    def observation_space(self):
        return self._observation_space if self._observation_space is not None else self.env.observation_space
    @observation_space.setter
    def observation_space(self, v):
        self._observation_space = v
    @property
    def unwrapped(self):
        return self.env.unwrapped if hasattr(self.env, "unwrapped") else self.env
    def step(self, action):
        return self.env.step(action)
    def reset(self, **kw):
        return self.env.reset(**kw)
class ObservationWrapper(Wrapper):
    def reset(self, **kw):
        return self.observation(self.env.reset(**kw))
    def step(self, action):
        o, r, d, i = self.env.step(action)
        return self.observation(o), r, d, i
'''

STUB_GYMAPI = '''
import numpy as np
import torch
SIM_PHYSX = 1
DOF_MODE_VEL = 2
MESH_VISUAL = 1
class Vec3:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = x, y, z
    def __neg__(self):
        return Vec3(-self.x, -self.y, -self.z)
    def __truediv__(self, k):
        return Vec3(self.x / k, self.y / k, self.z / k)
class Transform:
    def __init__(self, p=None, r=None):
        self.p = p if p is not None else Vec3()
class PlaneParams:
    pass
class AssetOptions:
    pass
class _Shape:
    def __init__(self):
        self.friction = 1.0
        self.filter = 0
class FakeGym:
    hook = None
    def create_sim(self, *a, **k):
        self.envs = []
        self.root = None
        self.pending = None
        self.targets = None
        return "sim"
    def add_ground(self, *a):
        pass
    def create_env(self, sim, lo, hi, n):
        self.envs.append([])
        return len(self.envs) - 1
    def create_sphere(self, *a):
        return "sphere"
    def create_box(self, *a):
        return "box"
    def load_asset(self, **k):
        return "robot"
    def create_actor(self, env, asset, pose, name=None, group=0, filter=0):
        self.envs[env].append((pose.p.x, pose.p.y, pose.p.z))
        return len(self.envs[env]) - 1
    def set_rigid_body_color(self, *a):
        pass
    def get_actor_rigid_shape_properties(self, env, actor):
        return [_Shape() for _ in range(5)]
    def set_actor_rigid_shape_properties(self, *a):
        pass
    def get_actor_dof_properties(self, env, actor):
        return {k: np.zeros(2) for k in ("driveMode", "stiffness", "damping", "armature", "friction", "velocity")}
    def set_actor_dof_properties(self, *a):
        pass
    def prepare_sim(self, sim):
        n = len(self.envs)
        root = torch.zeros((n * 15, 13), dtype=torch.float)
        for e, actors in enumerate(self.envs):
            for a, p in enumerate(actors):
                root[e * 15 + a, 0:3] = torch.tensor(p)
                root[e * 15 + a, 6] = 1.0
        self.root = root
    def acquire_actor_root_state_tensor(self, sim):
        return self.root
    def refresh_actor_root_state_tensor(self, sim):
        if self.pending is not None:
            self.root.copy_(self.pending)
            self.pending = None
    def set_actor_root_state_tensor(self, sim, t):
        self.pending = None
    def set_dof_velocity_target_tensor(self, sim, t):
        self.targets = t.clone()
    def simulate(self, sim):
        self.pending = FakeGym.hook(self.root.clone())
_GYM = FakeGym()
def acquire_gym():
    return _GYM
'''

STUB_TORCH_UTILS = '''
import torch
import numpy as np
def normalize(x, eps=1e-9):
    return x / x.norm(p=2, dim=-1).clamp(min=eps, max=None).unsqueeze(-1)
def quat_unit(a):
    return normalize(a)
def quat_from_angle_axis(angle, axis):
    theta = (angle / 2).unsqueeze(-1)
    xyz = normalize(axis) * theta.sin()
    w = theta.cos()
    return quat_unit(torch.cat([xyz, w], dim=-1))
def get_euler_xyz(q):
    qx, qy, qz, qw = 0, 1, 2, 3
    sinr_cosp = 2.0 * (q[:, qw] * q[:, qx] + q[:, qy] * q[:, qz])
    cosr_cosp = q[:, qw] * q[:, qw] - q[:, qx] * q[:, qx] - q[:, qy] * q[:, qy] + q[:, qz] * q[:, qz]
    roll = torch.atan2(sinr_cosp, cosr_cosp)
    sinp = 2.0 * (q[:, qw] * q[:, qy] - q[:, qz] * q[:, qx])
    pitch = torch.where(torch.abs(sinp) >= 1, torch.sign(sinp) * np.pi / 2.0, torch.asin(sinp))
    siny_cosp = 2.0 * (q[:, qw] * q[:, qz] + q[:, qx] * q[:, qy])
    cosy_cosp = q[:, qw] * q[:, qw] + q[:, qx] * q[:, qx] - q[:, qy] * q[:, qy] - q[:, qz] * q[:, qz]
    yaw = torch.atan2(siny_cosp, cosy_cosp)
    return roll % (2 * np.pi), pitch % (2 * np.pi), yaw % (2 * np.pi)
def torch_rand_float(lower, upper, shape, device):
    return (upper - lower) * torch.rand(*shape, device=device) + lower
'''

STUB_VEC_TASK = '''
import numpy as np
import torch
from gym.spaces import Box
from isaacgym import gymapi
class VecTask:
    def __init__(self, config, rl_device, sim_device, graphics_device_id, headless,
                 virtual_screen_capture=False, force_render=False):
        self.cfg = config
        self.rl_device = rl_device
        self.sim_device = sim_device
        self.device = sim_device
        self.device_id = 0
        self.graphics_device_id = graphics_device_id
        self.headless = headless
        self.num_environments = config["env"]["numEnvs"]
        self.num_agents = config["env"].get("numAgents", 1)
        self.num_observations = config["env"]["numObservations"]
        self.num_states = config["env"].get("numStates", 0)
        self.num_actions = config["env"]["numActions"]
        self.control_freq_inv = config["env"].get("controlFrequencyInv", 1)
        self.clip_obs = config["env"].get("clipObservations", np.inf)
        self.clip_actions = config["env"].get("clipActions", np.inf)
        self.obs_space = Box(-np.inf, np.inf, (self.num_observations,))
        self.act_space = Box(-1.0, 1.0, (self.num_actions,))
        self.physics_engine = gymapi.SIM_PHYSX
        self.sim_params = None
        self.viewer = None
        self.gym = gymapi.acquire_gym()
        self.create_sim()
        self.gym.prepare_sim(self.sim)
        self.allocate_buffers()
        self.obs_dict = {}
    @property
    def num_envs(self):
        return self.num_environments
    @property
    def num_obs(self):
        return self.num_observations
    @property
    def observation_space(self):
        return self.obs_space
    @property
    def action_space(self):
        return self.act_space
    def create_sim(self, compute_device, graphics_device, physics_engine, sim_params):
        return self.gym.create_sim(compute_device, graphics_device, physics_engine, sim_params)
    def step(self, actions):
        action_tensor = torch.clamp(actions, -self.clip_actions, self.clip_actions)
        self.pre_physics_step(action_tensor)
        for _ in range(self.control_freq_inv):
            self.gym.simulate(self.sim)
        self.post_physics_step()
        self.timeout_buf = (self.progress_buf >= self.max_episode_length - 1) & (self.reset_buf != 0)
        self.extras["time_outs"] = self.timeout_buf.to(self.rl_device)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        return self.obs_dict, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), self.extras
    def reset(self):
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        return self.obs_dict
'''


def install_stubs():
    d = tempfile.mkdtemp(prefix="vss_ref_stubs_")

    def w(rel, src):
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(textwrap.dedent(src))

    w("gym/__init__.py", STUB_GYM + "\nfrom gym import spaces\n")
    w("gym/spaces.py", "from gym import Box\n")
    w("isaacgym/__init__.py", "")
    w("isaacgym/gymapi.py", STUB_GYMAPI)
    w("isaacgym/gymtorch.py", "def wrap_tensor(t):\n    return t\ndef unwrap_tensor(t):\n    return t\n")
    w("isaacgym/torch_utils.py", STUB_TORCH_UTILS)
    w("isaacgymenvs/__init__.py", "")
    w("isaacgymenvs/tasks/__init__.py", "")
    w("isaacgymenvs/tasks/base/__init__.py", "")
    w("isaacgymenvs/tasks/base/vec_task.py", STUB_VEC_TASK)
    sys.path.insert(0, d)
    sys.path.insert(1, REF)
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    sys.modules["torch.utils.tensorboard"] = tb


# ----------------------------------------------------------------------------------------------
# draw recording and the cuda:0 redirect (envs/vss.py:533-538 hard-codes device="cuda:0")
# ----------------------------------------------------------------------------------------------
class Recorder:
    def __init__(self):
        self.uniforms: list[np.ndarray] = []
        self.normals: list[np.ndarray] = []
        self.u_sizes: list[int] = []  # size of every torch.rand call (the reference's batch shapes)
        self._rand, self._normal, self._tensor = torch.rand, torch.normal, torch.tensor

    def install(self):
        rec = self

        def rand(*a, **k):
            k.pop("device", None)
            out = rec._rand(*a, **k)
            rec.uniforms.append(out.detach().reshape(-1).numpy().copy())
            rec.u_sizes.append(out.numel())
            return out

        def normal(*a, **k):
            k.pop("device", None)
            out = rec._normal(*a, **k)
            rec.normals.append(out.detach().reshape(-1).numpy().copy())
            return out

        def tensor(*a, **k):
            if k.get("device") == "cuda:0":
                k["device"] = "cpu"
            return rec._tensor(*a, **k)

        torch.rand, torch.normal, torch.tensor = rand, normal, tensor

    def take(self):
        u = np.concatenate(self.uniforms) if self.uniforms else np.zeros(0, np.float32)
        z = np.concatenate(self.normals) if self.normals else np.zeros(0, np.float32)
        self.uniforms, self.normals = [], []
        return u.astype(np.float32), z.astype(np.float32)

    def take_sizes(self) -> np.ndarray:
        """Sizes of the torch.rand calls since the last call (rejection rounds, yaws, ball vel)."""
        out = np.array(self.u_sizes, np.int64)
        self.u_sizes = []
        return out


# ----------------------------------------------------------------------------------------------
# root-state (N,15,13) <-> oracle SoA state (58, N)
# ----------------------------------------------------------------------------------------------
def root_to_state(root: torch.Tensor, n: int) -> np.ndarray:
    r = root.view(n, 15, 13).numpy()
    s = np.zeros((O.STATE_CHANNELS, n), np.float32)
    s[0], s[1], s[2], s[3] = r[:, 0, 0], r[:, 0, 1], r[:, 0, 7], r[:, 0, 8]
    for k in range(6):
        a = r[:, 1 + k]
        s[O.CH_RX + k], s[O.CH_RY + k] = a[:, 0], a[:, 1]
        s[O.CH_RQX + k], s[O.CH_RQY + k] = a[:, 3], a[:, 4]
        s[O.CH_RQZ + k], s[O.CH_RQW + k] = a[:, 5], a[:, 6]
        s[O.CH_RVX + k], s[O.CH_RVY + k] = a[:, 7], a[:, 8]
        s[O.CH_RW + k] = a[:, 12]
    return s


def state_to_root(s: np.ndarray, root: torch.Tensor, n: int) -> torch.Tensor:
    r = root.view(n, 15, 13)
    t = torch.from_numpy
    r[:, 0, 0], r[:, 0, 1], r[:, 0, 7], r[:, 0, 8] = t(s[0]), t(s[1]), t(s[2]), t(s[3])
    for k in range(6):
        r[:, 1 + k, 0], r[:, 1 + k, 1] = t(s[O.CH_RX + k]), t(s[O.CH_RY + k])
        r[:, 1 + k, 5], r[:, 1 + k, 6] = t(s[O.CH_RQZ + k]), t(s[O.CH_RQW + k])
        r[:, 1 + k, 7], r[:, 1 + k, 8] = t(s[O.CH_RVX + k]), t(s[O.CH_RVY + k])
        r[:, 1 + k, 12] = t(s[O.CH_RW + k])
    return root


LIVE = [0, 1, 2, 3] + [c + k for c in (O.CH_RX, O.CH_RY, O.CH_RQZ, O.CH_RQW, O.CH_RVX, O.CH_RVY, O.CH_RW)
                       for k in range(6)]


def make_cfg(n, max_len=400, w=(10.0, 2.0, 3.0, 0.0)):
    import yaml
    with open(os.path.join(REF, "envs", "vss.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["env"]["numEnvs"] = n
    cfg["env"]["maxEpisodeLength"] = max_len
    cfg["env"]["rew_weights"] = dict(goal=w[0], grad=w[1], move=w[2], energy=w[3])
    return cfg


def make_env(n, max_len, w=(10.0, 2.0, 3.0, 0.0)):
    from isaacgym import gymapi
    from envs.vss import VSS
    env_box = {}

    def hook(root):
        env = env_box["env"]
        s = root_to_state(root, env.num_fields)
        O.simulate(s, env.dof_velocity_buf.reshape(env.num_fields, 12).numpy())
        return state_to_root(s, root, env.num_fields)

    gymapi.FakeGym.hook = staticmethod(hook)
    env = VSS(make_cfg(n, max_len, w), "cpu", "cpu", 0, True, False, False)
    env_box["env"] = env
    return env


# ----------------------------------------------------------------------------------------------
# fixtures
# ----------------------------------------------------------------------------------------------
def random_state(gen: np.random.Generator, n: int) -> np.ndarray:
    s = np.zeros((O.STATE_CHANNELS, n), np.float32)
    s[0] = gen.uniform(-0.8, 0.8, n)
    s[1] = gen.uniform(-0.6, 0.6, n)
    s[2:4] = gen.uniform(-1.5, 1.5, (2, n))
    s[O.CH_RX:O.CH_RX + 6] = gen.uniform(-0.75, 0.75, (6, n))
    s[O.CH_RY:O.CH_RY + 6] = gen.uniform(-0.65, 0.65, (6, n))
    yaw = gen.uniform(-np.pi, np.pi, (6, n))
    yaw[:, :4] = [0.0, np.pi - 1e-6, -np.pi + 1e-6, 1e-7]  # yaw near 0 / +-pi
    s[O.CH_RQZ:O.CH_RQZ + 6] = np.sin(yaw / 2)
    s[O.CH_RQW:O.CH_RQW + 6] = np.cos(yaw / 2)
    s[O.CH_RVX:O.CH_RVX + 12] = gen.uniform(-1.2, 1.2, (12, n))
    s[O.CH_RW:O.CH_RW + 6] = gen.uniform(-30, 30, (6, n))
    return s


def gen_obs_and_rewards(rec: Recorder):
    """G1 compute_obs, G2 goal/dones edge cases, G3 grad/move/energy (envs/vss.py:530-655)."""
    from envs import vss as V
    gen = np.random.default_rng(1234)
    n = 64
    s = random_state(gen, n)
    acts = gen.uniform(-1, 1, (n, 2, 3, 2)).astype(np.float32)
    root = torch.zeros((n * 15, 13))
    state_to_root(s, root, n)
    r = root.view(n, 15, 13)
    rp = r[..., 0:2][:, 1:7].reshape(n, 2, 3, 2)
    rq = r[..., 3:7][:, 1:7].reshape(n, 2, 3, 4)
    rv = r[..., 7:9][:, 1:7].reshape(n, 2, 3, 2)
    rw = r[..., 12][:, 1:7].reshape(n, 2, 3, 1)
    perms = torch.tensor([[0, 1, 2], [1, 2, 0], [2, 0, 1]])
    mirror = torch.tensor([-1.0, -1.0, -1.0, -1.0, -1.0, -1.0, 1.0, 1.0, 1.0])
    obs = V.compute_obs(r[:, 0, 0:2], r[:, 0, 7:9], rp, rv, rq, rw, torch.from_numpy(acts), perms, mirror)

    # G2: goal / done edge cases: |x| = 0.75 +- 1ulp, |y| = 0.2 +- 1ulp, progress 399/400
    f32 = np.float32
    xs = [np.nextafter(f32(0.75), f32(0)), f32(0.75), np.nextafter(f32(0.75), f32(1)), f32(0.8), f32(0.0)]
    ys = [np.nextafter(f32(0.2), f32(0)), f32(0.2), np.nextafter(f32(0.2), f32(1)), f32(0.0)]
    balls = []
    for x in xs:
        for y in ys:
            for sx in (1, -1):
                for sy in (1, -1):
                    balls.append((sx * x, sy * y))
    balls = np.array(balls, np.float32)
    m = len(balls)
    progress = np.tile(np.array([0, 398, 399, 400, 401], np.int64), m // 5 + 1)[:m]
    goal = V.compute_goal_rew(torch.zeros(m, dtype=torch.long), torch.from_numpy(balls), 1.5, 0.4)
    dones = V.compute_vss_dones(torch.from_numpy(balls), torch.zeros(m, dtype=torch.long),
                                torch.from_numpy(progress), 400, 1.5, 0.4)

    # G3: grad / move / energy
    prev_ball = gen.uniform(-0.8, 0.8, (n, 2)).astype(np.float32)
    ball = (prev_ball + gen.normal(0, 0.05, (n, 2))).astype(np.float32)
    prev_rob = gen.uniform(-0.7, 0.7, (n, 2, 3, 2)).astype(np.float32)
    rob = (prev_rob + gen.normal(0, 0.05, (n, 2, 3, 2))).astype(np.float32)
    yellow_goal = torch.tensor([0.75, 0.0])
    grad = V.compute_grad_rew(torch.from_numpy(prev_ball), torch.from_numpy(ball), yellow_goal)
    move = V.compute_move_rew(torch.from_numpy(prev_rob), torch.from_numpy(rob),
                              torch.from_numpy(prev_ball), torch.from_numpy(ball))
    energy = V.compute_energy_rew(torch.from_numpy(acts))
    np.savez_compressed(
        os.path.join(HERE, "g1_g3_kernels.npz"),
        obs_state=s, obs_actions=acts.reshape(n, 12), obs=obs.numpy(),
        goal_ball=balls, goal_progress=progress, goal=goal.numpy(), dones=dones.numpy(),
        prev_ball=prev_ball, ball=ball, prev_rob=prev_rob.reshape(n, 12), rob=rob.reshape(n, 12),
        grad=grad.numpy(), move=move.numpy(), energy=energy.numpy(),
    )
    print("G1-G3: obs", tuple(obs.shape), "edge balls", m)


def gen_full_rollout(rec: Recorder, n=16, steps=1000, max_len=400):
    """G4 (BASELINE config 1: 16 fields, random actions, 1,000 steps): the reference's VSS.step
    bookkeeping, physics = oracle hook.  Goals are forced (play.py-style external writes through
    the reference's views) into a field still in its first episode at steps max_len - 3 and
    max_len - 2 -- the time-out edge (time_outs = progress >= max_len - 1 & reset) -- and into a
    few more fields later on."""
    torch.manual_seed(1)
    rec.take()
    rec.take_sizes()
    env = make_env(n, max_len)
    init_u, _ = rec.take()  # draws of the construction-time reset_dones (envs/vss.py:72)
    init_sizes = rec.take_sizes()
    init_state = root_to_state(env.root_state.reshape(-1, 13), n)
    # external writes (play.py-style, through the reference's views) to force goals
    env.ball_pos[0] = torch.tensor([0.70, 0.05]); env.ball_vel[0] = torch.tensor([1.0, 0.0])
    env.ball_pos[1] = torch.tensor([-0.70, -0.10]); env.ball_vel[1] = torch.tensor([-1.2, 0.1])
    env.gym.set_actor_root_state_tensor(env.sim, env.root_state)
    start_state = root_to_state(env.root_state.reshape(-1, 13), n)
    gen = np.random.default_rng(7)
    keep = {k: [] for k in ("actions", "state", "rew", "reset", "progress", "time_outs", "progress_f",
                            "dof", "u_count")}
    obs_steps, obs_keep, tobs_keep, uniforms, u_sizes, u_ncalls = [], [], [], [], [], []
    forced_steps, forced_fields, forced_state = [], [], []
    edge = {max_len - 3: None, max_len - 2: None}
    for t in range(steps):
        a = gen.uniform(-1.3, 1.3, (n, 2, 3, 2)).astype(np.float32)  # > clip to exercise clamp
        push = []
        if t in edge:  # a field still in its first episode (progress == t before this step)
            cand = [f for f in range(n) if int(env.progress_buf[f]) == t and f not in edge.values()]
            edge[t] = cand[0]
            push = [(cand[0], 1.0), ((cand[0] + 5) % n, -1.0)]
        elif t % 97 == 50:
            push = [(t % n, 1.0 if t % 2 else -1.0)]
        if push:
            for f, side in push:
                env.ball_pos[f] = torch.tensor([0.74 * side, 0.05]); env.ball_vel[f] = torch.tensor([1.0 * side, 0.0])
            env.gym.set_actor_root_state_tensor(env.sim, env.root_state)
            forced_steps.append(t)
            forced_fields.append(edge.get(t) if t in edge else -1)
            forced_state.append(root_to_state(env.root_state.reshape(-1, 13), n)[LIVE])
        obs_dict, rew, reset, extras = env.step(torch.from_numpy(a))
        u, _ = rec.take()
        sz = rec.take_sizes()
        uniforms.append(u)
        u_sizes.append(sz)
        u_ncalls.append(len(sz))
        keep["actions"].append(a.reshape(n, 12))
        keep["state"].append(root_to_state(env.root_state.reshape(-1, 13), n)[LIVE])
        keep["rew"].append(rew.numpy().reshape(n, 24).copy())
        keep["reset"].append(reset.numpy().copy())
        keep["progress"].append(env.progress_buf.numpy().copy())
        keep["time_outs"].append(extras["time_outs"].numpy().astype(np.uint8))
        keep["progress_f"].append(extras["progress_buffer"].numpy().copy())
        keep["dof"].append(env.dof_velocity_buf.numpy().reshape(n, 12).copy())
        keep["u_count"].append(len(u))
        if t < 4 or reset.any():
            obs_steps.append(t)
            obs_keep.append(obs_dict["obs"].numpy().reshape(n, 312).copy())
            tobs_keep.append(extras["terminal_observation"].numpy().reshape(n, 312).copy())
    out = {k: np.stack(v) for k, v in keep.items()}
    np.savez_compressed(
        os.path.join(HERE, "g4_full_rollout.npz"), forced_steps=np.array(forced_steps),
        forced_fields=np.array(forced_fields), forced_state=np.stack(forced_state),
        edge_steps=np.array(sorted(edge)), edge_fields=np.array([edge[k] for k in sorted(edge)]),
        init_uniforms=init_u, init_u_sizes=init_sizes, init_state=init_state,
        start_state=start_state, live_channels=np.array(LIVE), uniforms=np.concatenate(uniforms),
        u_sizes=np.concatenate(u_sizes), u_ncalls=np.array(u_ncalls),
        obs_steps=np.array(obs_steps), obs=np.stack(obs_keep), terminal_obs=np.stack(tobs_keep),
        max_len=np.array(max_len), **out)
    print("G4: fields", n, "steps", steps, "resets", int(out["reset"].sum()), "goals",
          int((np.abs(out["rew"][:, :, 0]) > 0).sum()), "time-outs", int(out["time_outs"].sum()),
          "obs steps", len(obs_steps))


def gen_wrapped(rec: Recorder, mode: str, n=6, steps=60, max_len=25):
    """G5: SingleAgent / CMA / DMA wrappers (envs/wrappers.py:89-180) on the reference VSS.
    Goals are forced (play.py-style external writes through the reference's views, as in G4) at
    both ends of the field and at several points of an episode: blue and yellow scoring at the
    first step and mid-episode, and into fields still in their first episode at steps max_len - 3
    (a goal done with time_outs = 0) and max_len - 2 (the time-out edge: time_outs = 1), so the
    wrapped path's goal channel, mid-episode OU-buffer zeroing and time_outs on a goal done are
    all pinned (envs/wrappers.py:101-115, 133-148, 163-180; envs/vss.py:578-594)."""
    from envs.wrappers import SingleAgent, CMA, DMA
    torch.manual_seed(3)
    rec.take()
    rec.take_sizes()
    env = make_env(n, max_len)
    init_u, _ = rec.take()
    init_sizes = rec.take_sizes()
    init_state = root_to_state(env.root_state.reshape(-1, 13), n)
    W = {"sa": SingleAgent, "cma": CMA, "dma": DMA}[mode](env)
    rows = n * 3 if mode == "dma" else n
    adim = 6 if mode == "cma" else 2
    gen = np.random.default_rng(11)
    keep = {k: [] for k in ("actions", "obs", "terminal_obs", "reward", "rews", "dones", "time_outs",
                            "progress_f", "state", "action_buf", "n_u", "n_z")}
    U, Z, S, NC = [], [], [], []
    forced_steps, forced_state = [], []
    edge = {max_len - 3: None, max_len - 2: None}
    schedule = {0: [(3, -1.0)], 7: [(0, 1.0), (1, -1.0)], 40: [(4, -1.0), (5, 1.0)]}
    for t in range(steps):
        a = gen.uniform(-1.2, 1.2, (rows, adim)).astype(np.float32)
        push = list(schedule.get(t, []))
        if t in edge:  # a field still in its first episode (progress == t before this step)
            cand = [f for f in range(n) if int(env.progress_buf[f]) == t and f not in edge.values()]
            assert cand, f"no first-episode field left at step {t}"
            edge[t] = cand[0]
            push.append((cand[0], 1.0 if t % 2 else -1.0))
        if push:
            for f, side in push:
                env.ball_pos[f] = torch.tensor([0.74 * side, 0.05]); env.ball_vel[f] = torch.tensor([1.0 * side, 0.0])
            env.gym.set_actor_root_state_tensor(env.sim, env.root_state)
            forced_steps.append(t)
            forced_state.append(root_to_state(env.root_state.reshape(-1, 13), n)[LIVE])
        obs, reward, dones, info = W.step(torch.from_numpy(a))
        u, z = rec.take()
        sz = rec.take_sizes()
        U.append(u); Z.append(z); S.append(sz); NC.append(len(sz))
        keep["actions"].append(a)
        keep["obs"].append(obs["obs"].numpy().copy())
        keep["terminal_obs"].append(info["terminal_observation"].numpy().copy())
        keep["reward"].append(reward.numpy().copy())
        keep["rews"].append(info["rews"].numpy().copy())
        keep["dones"].append(dones.numpy().copy())
        keep["time_outs"].append(info["time_outs"].numpy().astype(np.uint8))
        keep["progress_f"].append(info["progress_buffer"].numpy().copy())
        keep["state"].append(root_to_state(env.root_state.reshape(-1, 13), n)[LIVE])
        keep["action_buf"].append(W.action_buf.numpy().reshape(n, 12).copy())
        keep["n_u"].append(len(u)); keep["n_z"].append(len(z))
    out = {k: np.stack(v) for k, v in keep.items()}
    np.savez_compressed(os.path.join(HERE, f"g5_wrapped_{mode}.npz"), init_uniforms=init_u, init_u_sizes=init_sizes,
                        u_sizes=np.concatenate(S), u_ncalls=np.array(NC),
                        init_state=init_state, uniforms=np.concatenate(U), normals=np.concatenate(Z),
                        live_channels=np.array(LIVE), max_len=np.array(max_len), num_envs=np.array(W.num_envs),
                        forced_steps=np.array(forced_steps), forced_state=np.stack(forced_state),
                        edge_steps=np.array(sorted(edge)), edge_fields=np.array([edge[k] for k in sorted(edge)]),
                        **out)
    goal = np.abs(out["rews"][..., 0]) > 0
    print(f"G5 {mode}: rows {rows} steps {steps} dones {int(out['dones'].sum())} goal rows {int(goal.sum())} "
          f"goal dones with time_outs=0 {int((goal & (out['time_outs'] == 0)).sum())} num_envs {W.num_envs}")


def gen_agent():
    """G6: the reference Agent (ppo_continuous_action_isaacgym.py:121-164) from seeded init."""
    from collections import namedtuple
    import gym
    import ppo_continuous_action_isaacgym as P
    Env = namedtuple("Env", ["single_observation_space", "single_action_space"])
    res = {}
    for act_dim in (2, 6):
        torch.manual_seed(42)
        agent = P.Agent(Env(gym.spaces.Box(-np.inf, np.inf, (52,)), gym.spaces.Box(-1.0, 1.0, (act_dim,))))
        sd = agent.state_dict()
        gen = torch.Generator().manual_seed(5)
        x = torch.randn(32, 52, generator=gen)
        a = torch.randn(32, act_dim, generator=gen) * 0.3
        with torch.no_grad():
            _, logp, ent, val = agent.get_action_and_value(x, a)
            mean = agent.actor_mean(x)
        res[f"a{act_dim}_keys"] = np.array(list(sd.keys()))
        res[f"a{act_dim}_shapes"] = np.array([str(tuple(v.shape)) for v in sd.values()])
        res[f"a{act_dim}_param_sums"] = np.array([float(v.double().sum()) for v in sd.values()])
        res[f"a{act_dim}_param_abs_sums"] = np.array([float(v.double().abs().sum()) for v in sd.values()])
        res[f"a{act_dim}_nparams"] = np.array(sum(v.numel() for v in sd.values()))
        res[f"a{act_dim}_x"] = x.numpy(); res[f"a{act_dim}_a"] = a.numpy()
        res[f"a{act_dim}_logp"] = logp.numpy(); res[f"a{act_dim}_ent"] = ent.numpy()
        res[f"a{act_dim}_val"] = val.numpy(); res[f"a{act_dim}_mean"] = mean.numpy()
    np.savez_compressed(os.path.join(HERE, "g6_agent.npz"), torch_version=np.array(torch.__version__), **res)
    print("G6: agent params", int(res["a2_nparams"]), int(res["a6_nparams"]))


def main(which=("g1", "g4", "g5", "g6")):
    install_stubs()
    O.build()
    rec = Recorder()
    rec.install()
    if "g1" in which:
        gen_obs_and_rewards(rec)
    if "g4" in which:
        gen_full_rollout(rec)
    if "g5" in which:
        for mode in ("sa", "cma", "dma"):
            gen_wrapped(rec, mode)
    if "g6" in which:
        gen_agent()


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ("g1", "g4", "g5", "g6"))
