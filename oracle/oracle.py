"""ctypes binding of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It wraps oracle/_build/libvss_oracle.so (built by `make -C oracle`) over numpy host buffers
laid out exactly like the device ABI (include/vss.h), so a test can feed the oracle and the
HIP kernel the same bytes and compare the outputs.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libvss_oracle.so")

MODE_FULL, MODE_SA, MODE_CMA, MODE_DMA = 0, 1, 2, 3
STATE_CHANNELS = 58
CH_BALL = 0
CH_RX, CH_RY, CH_RQX, CH_RQY, CH_RQZ, CH_RQW, CH_RVX, CH_RVY, CH_RW = 4, 10, 16, 22, 28, 34, 40, 46, 52


class VssParams(ctypes.Structure):
    _fields_ = [
        ("w_goal", ctypes.c_float),
        ("w_grad", ctypes.c_float),
        ("w_move", ctypes.c_float),
        ("w_energy", ctypes.c_float),
        ("clip_actions", ctypes.c_float),
        ("max_episode_length", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
    ]


class VssState(ctypes.Structure):
    _fields_ = [
        ("state", ctypes.c_void_p),
        ("progress_buf", ctypes.c_void_p),
        ("reset_buf", ctypes.c_void_p),
        ("dof_velocity_buf", ctypes.c_void_p),
        ("rng_counter", ctypes.c_void_p),
    ]


class VssStepIO(ctypes.Structure):
    _fields_ = [
        ("actions", ctypes.c_void_p),
        ("ou_buf", ctypes.c_void_p),
        ("obs", ctypes.c_void_p),
        ("terminal_obs", ctypes.c_void_p),
        ("rew", ctypes.c_void_p),
        ("reward_sum", ctypes.c_void_p),
        ("dones_rep", ctypes.c_void_p),
        ("time_outs", ctypes.c_void_p),
        ("progress_f", ctypes.c_void_p),
    ]


class OracleDraws(ctypes.Structure):
    _fields_ = [
        ("uniforms", ctypes.c_void_p),
        ("n_uniforms", ctypes.c_int64),
        ("uniform_pos", ctypes.c_int64),
        ("normals", ctypes.c_void_p),
        ("n_normals", ctypes.c_int64),
        ("normal_pos", ctypes.c_int64),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_step.argtypes = [ctypes.c_int64, ctypes.c_int32, P, P, P, P]
        L.oracle_reset_dones.argtypes = [ctypes.c_int64, P, P, P]
        L.oracle_compute_observations.argtypes = [ctypes.c_int64, P, P, ctypes.c_int32]
        L.oracle_simulate.argtypes = [ctypes.c_int64, P, P]
        L.oracle_goal_rew.argtypes = [ctypes.c_int64, P, P]
        L.oracle_grad_rew.argtypes = [ctypes.c_int64, P, P, P]
        L.oracle_move_rew.argtypes = [ctypes.c_int64, P, P, P, P, P]
        L.oracle_vss_dones.argtypes = [ctypes.c_int64, P, P, ctypes.c_int64, P]
        L.oracle_philox.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P, P]
        L.oracle_logf.argtypes = [ctypes.c_float]
        L.oracle_logf.restype = ctypes.c_float
        L.oracle_sincosf.argtypes = [ctypes.c_float, P, P]
        _lib = L
    return _lib


def _p(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle buffers must be C-contiguous"
    return a.ctypes.data


def params(w_goal=10.0, w_grad=2.0, w_move=3.0, w_energy=0.0, clip_actions=1.0,
           max_episode_length=400, seed=1) -> VssParams:
    return VssParams(w_goal, w_grad, w_move, w_energy, clip_actions, max_episode_length, seed)


class HostEnv:
    """Host buffers of `n` fields in the device layout of include/vss.h."""

    def __init__(self, n: int):
        self.n = n
        self.state = np.zeros((STATE_CHANNELS, n), np.float32)
        self.state[CH_RQW:CH_RQW + 6] = 1.0
        self.progress = np.zeros(n, np.int64)
        self.reset = np.ones(n, np.int64)
        self.dof = np.zeros((n, 12), np.float32)
        self.ctr = np.zeros(n, np.uint32)

    def copy(self) -> "HostEnv":
        e = HostEnv.__new__(HostEnv)
        e.n = self.n
        for k in ("state", "progress", "reset", "dof", "ctr"):
            setattr(e, k, getattr(self, k).copy())
        return e

    def c_state(self) -> VssState:
        return VssState(_p(self.state), _p(self.progress), _p(self.reset), _p(self.dof), _p(self.ctr))


def make_io(n: int, mode: int):
    agents = {MODE_FULL: 6, MODE_SA: 1, MODE_CMA: 1, MODE_DMA: 3}[mode]
    R = 3 if mode == MODE_DMA else 1
    rew_shape = {MODE_FULL: (n, 24), MODE_SA: (n, 4), MODE_CMA: (n, 4), MODE_DMA: (n * 3, 4)}[mode]
    io = dict(
        obs=np.zeros((n * agents, 52), np.float32),
        terminal_obs=np.zeros((n * agents, 52), np.float32),
        rew=np.zeros(rew_shape, np.float32),
        reward_sum=np.zeros(n * (3 if mode == MODE_DMA else 1), np.float32),
        dones_rep=np.zeros(n * 3, np.int64) if mode == MODE_DMA else None,
        time_outs=np.zeros(n * R, np.uint8),
        progress_f=np.zeros(n * R, np.float32),
        ou_buf=np.zeros((n, 12), np.float32) if mode != MODE_FULL else None,
    )
    return io


def step(env: HostEnv, mode: int, actions: np.ndarray, io: dict, prm: VssParams,
         draws: OracleDraws | None = None) -> int:
    actions = np.ascontiguousarray(actions, np.float32)
    cio = VssStepIO(_p(actions), _p(io.get("ou_buf")), _p(io["obs"]), _p(io["terminal_obs"]),
                    _p(io["rew"]), _p(io.get("reward_sum")), _p(io.get("dones_rep")),
                    _p(io["time_outs"]), _p(io["progress_f"]))
    st = env.c_state()
    rc = lib().oracle_step(env.n, mode, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(cio),
                           ctypes.byref(draws) if draws is not None else None)
    if rc != 0:
        raise RuntimeError(f"oracle_step failed: {rc}")
    return rc


def reset_dones(env: HostEnv, prm: VssParams, draws: OracleDraws | None = None) -> None:
    st = env.c_state()
    rc = lib().oracle_reset_dones(env.n, ctypes.byref(prm), ctypes.byref(st),
                                  ctypes.byref(draws) if draws is not None else None)
    if rc != 0:
        raise RuntimeError(f"oracle_reset_dones failed: {rc}")


def compute_obs(env: HostEnv, n_agents: int = 6) -> np.ndarray:
    obs = np.zeros((env.n, n_agents, 52), np.float32)
    st = env.c_state()
    rc = lib().oracle_compute_observations(env.n, ctypes.byref(st), _p(obs), n_agents)
    if rc != 0:
        raise RuntimeError(f"oracle_compute_observations failed: {rc}")
    return obs


def simulate(state: np.ndarray, actions: np.ndarray) -> None:
    """Physics only, in place on a (58, n) state with clamped (n, 12) actions."""
    assert state.dtype == np.float32 and state.shape[0] == STATE_CHANNELS
    actions = np.ascontiguousarray(actions, np.float32)
    rc = lib().oracle_simulate(state.shape[1], _p(state), _p(actions))
    if rc != 0:
        raise RuntimeError("oracle_simulate failed")


def make_draws(uniforms: np.ndarray, normals: np.ndarray):
    """Injected-draw provider; keep the returned arrays alive while the struct is used."""
    u = np.ascontiguousarray(uniforms, np.float32)
    z = np.ascontiguousarray(normals, np.float32)
    d = OracleDraws(_p(u), u.size, 0, _p(z), z.size, 0)
    return d, (u, z)


def philox(key: int, ctr) -> np.ndarray:
    c = np.asarray(ctr, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().oracle_philox(key & 0xFFFFFFFF, (key >> 32) & 0xFFFFFFFF, _p(c), _p(o))
    return o


def sincosf(x: float):
    s = np.zeros(1, np.float32)
    c = np.zeros(1, np.float32)
    lib().oracle_sincosf(x, _p(s), _p(c))
    return float(s[0]), float(c[0])


def logf(x: float) -> float:
    return float(lib().oracle_logf(x))
