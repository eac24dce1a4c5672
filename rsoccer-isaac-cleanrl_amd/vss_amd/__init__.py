"""MI355X-native VSS match step: ctypes binding of the HIP C ABI (include/vss.h) and its build.

The drop-in Python API lives next to this package, mirroring the reference's layout:
`envs/vss.py` (class VSS), `envs/wrappers.py` (make_env, SingleAgent, CMA, DMA,
RecordEpisodeStatisticsTorch) and `ppo_continuous_action_isaacgym.py` (Agent, train loop).
"""
from . import _native as native  # noqa: F401
from .build import build  # noqa: F401
