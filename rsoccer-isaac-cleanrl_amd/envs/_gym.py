"""gym 0.23 surface used by the env API (Box, Wrapper, ObservationWrapper).

Uses the real `gym` when it is installed (the reference pins gym==0.23.1,
.devcontainer/Dockerfile:18); otherwise a minimal equivalent with the same semantics for the
attributes the reference touches (`env`, `_action_space`, `_observation_space`, attribute
forwarding, `step` / `reset` pass-through).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - depends on the environment
    import gym as _gym

    Box = _gym.spaces.Box
    Wrapper = _gym.Wrapper
    ObservationWrapper = _gym.ObservationWrapper
    HAVE_GYM = True
except ImportError:
    HAVE_GYM = False

    class Box:  # noqa: D401 - mirrors gym.spaces.Box(low, high, shape)
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high = low, high
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.dtype = np.dtype(dtype)

        def __repr__(self):
            return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"

    class Wrapper:
        def __init__(self, env):
            self.env = env
            self._action_space = None
            self._observation_space = None

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(f"attempted to get missing private attribute '{name}'")
            return getattr(self.env, name)

        @property
        def action_space(self):
            return self.env.action_space if self._action_space is None else self._action_space

        @action_space.setter
        def action_space(self, space):
            self._action_space = space

        @property
        def observation_space(self):
            return self.env.observation_space if self._observation_space is None else self._observation_space

        @observation_space.setter
        def observation_space(self, space):
            self._observation_space = space

        @property
        def unwrapped(self):
            return getattr(self.env, "unwrapped", self.env)

        def step(self, action):
            return self.env.step(action)

        def reset(self, **kwargs):
            return self.env.reset(**kwargs)

        def close(self):
            return getattr(self.env, "close", lambda: None)()

    class ObservationWrapper(Wrapper):
        def reset(self, **kwargs):
            return self.observation(self.env.reset(**kwargs))

        def step(self, action):
            observation, reward, done, info = self.env.step(action)
            return self.observation(observation), reward, done, info

        def observation(self, observation):
            raise NotImplementedError
