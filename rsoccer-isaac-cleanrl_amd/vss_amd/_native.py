"""ctypes binding of libvss_amd.so — the C ABI declared in include/vss.h.

The shared library is built in-tree by `make -C rsoccer-isaac-cleanrl_amd/csrc` (or
`__graft_entry__.build()`).  There is no fallback: if the library is missing, was built from other
sources than the tree's (its `vss_source_hash()` stamp differs from the hash of the sources here),
or the device is not a ROCm GPU, the calls raise.  torch is imported first so that the HIP runtime the library
links against (libamdhip64.so.7) is the one torch already loaded — one runtime, one set of
streams.
"""
from __future__ import annotations

import ctypes
import hashlib
import os

import torch  # noqa: F401  (loads torch's HIP runtime before the library resolves it)

HERE = os.path.dirname(os.path.abspath(__file__))
TOOLS = os.path.join(os.path.dirname(os.path.dirname(HERE)), "tools")


def _lib_path() -> str:
    """The in-tree libvss_amd.so; VSS_LIB_PATH may name a variant build of the same sources for A/B
    measurements, and only one under the repository's tools/ (it still has to pass the source-stamp check)."""
    alt = os.environ.get("VSS_LIB_PATH")
    if not alt:
        return os.path.join(HERE, "libvss_amd.so")
    alt = os.path.realpath(alt)
    if not alt.startswith(os.path.realpath(TOOLS) + os.sep):
        raise RuntimeError(f"VSS_LIB_PATH={alt}: only variant builds under {TOOLS} are accepted")
    import warnings
    warnings.warn(f"libvss_amd: loading the variant build {alt} (VSS_LIB_PATH)", RuntimeWarning)
    return alt


LIB_PATH = _lib_path()
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "vss.h")

# the sources the Makefile stamps into the library, in its order (csrc/Makefile STAMPED)
STAMPED = (os.path.join(CSRC, "vss_step.hip"), os.path.join(CSRC, "vss_update.hip"),
           os.path.join(CSRC, "vss_policy.hip"), os.path.join(CSRC, "vss_gemm_x6.hip"),
           os.path.join(CSRC, "vss_loss.hip"), os.path.join(CSRC, "vss_optim.hip"),
           os.path.join(CSRC, "vss_loss_row.h"), HEADER,
           os.path.join(CSRC, "Makefile"))

ABI_VERSION = 2
MODE_FULL, MODE_SA, MODE_CMA, MODE_DMA = 0, 1, 2, 3
STATE_CHANNELS = 58
CH_BALL_X, CH_BALL_Y, CH_BALL_VX, CH_BALL_VY = 0, 1, 2, 3
CH_RX, CH_RY, CH_RQX, CH_RQY, CH_RQZ, CH_RQW, CH_RVX, CH_RVY, CH_RW = 4, 10, 16, 22, 28, 34, 40, 46, 52
EXPORTED = ("vss_abi_version", "vss_source_hash", "vss_error_string", "vss_step", "vss_step_replay", "vss_rollout", "vss_reset_dones",
            "vss_reset_dones_replay",
            "vss_compute_observations", "vss_mlp_packed_size", "vss_mlp_pack", "vss_policy_forward",
            "vss_value_forward_masked", "vss_policy_sample", "vss_episode_stats", "vss_tanh_grad_chunks", "vss_tanh_grad_bias",
            "vss_linear_tanh", "vss_linear_tanh_out", "vss_linear_tanh_backward_chunks", "vss_linear_tanh_backward",
            "vss_output_backward_chunks", "vss_output_backward", "vss_linear_tanh_bf16x6",
            "vss_linear_tanh_out_bf16x6", "vss_linear_tanh_backward_chunks_bf16x6", "vss_linear_tanh_backward_bf16x6",
            "vss_weight_grad_chunks_bf16x6", "vss_weight_grad_bf16x6", "vss_first_weight_grad_chunks_bf16x6",
            "vss_first_weight_grad_bf16x6", "vss_weight_planes_bf16x6", "vss_ppo_loss_scratch_floats", "vss_ppo_loss",
            "vss_grad_sq_partials_count", "vss_grad_sq_partials", "vss_adam_step_clipped", "vss_sum_parts",
            "vss_output_backward_direct_chunks", "vss_output_backward_direct", "vss_ppo_loss_direct_scratch_floats",
            "vss_ppo_loss_direct", "vss_minibatch_gather_parts", "vss_minibatch_gather", "vss_adv_part_sum",
            "vss_first_layer_bf16x6", "vss_linear_tanh_loss_blocks_bf16x6", "vss_linear_tanh_loss_bf16x6",
            "vss_ppo_loss_fused_finish", "vss_randperm_scratch_bytes", "vss_randperm", "vss_randperm_bits")


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
    _fields_ = [(k, ctypes.c_void_p) for k in
                ("state", "progress_buf", "reset_buf", "dof_velocity_buf", "rng_counter")]


class VssStepIO(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in
                ("actions", "ou_buf", "obs", "terminal_obs", "rew", "reward_sum", "dones_rep",
                 "time_outs", "progress_f")]


class VssRolloutIO(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in
                ("actions", "obs", "terminal_obs", "rew", "dones", "time_outs", "progress_f")]


class VssReplayDraws(ctypes.Structure):
    """Recorded reference draws for the parity entries (include/vss.h vss_replay_draws)."""
    _fields_ = [("uniforms", ctypes.c_void_p), ("uniform_stride", ctypes.c_int64), ("normals", ctypes.c_void_p)]


class NativeError(RuntimeError):
    pass


_lib = None


def source_hash() -> str:
    """sha256 (first 16 hex digits) of the stamped sources as they are in this tree."""
    h = hashlib.sha256()
    for path in STAMPED:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def verify_source_hash(lib: ctypes.CDLL, expected: str | None = None) -> None:
    """Raise unless the library was built from the tree's sources (a stale prebuilt .so)."""
    want = source_hash() if expected is None else expected
    try:
        fn = lib.vss_source_hash
    except AttributeError:  # a library older than the stamp: stale by definition
        fn = None
    if fn is not None:
        fn.restype = ctypes.c_char_p
    built = fn().decode() if fn is not None else "<no vss_source_hash symbol>"
    if built != want:
        raise NativeError(
            f"{LIB_PATH} was built from other sources (stamp {built}, tree {want}); rebuild it with "
            f"`make -C {CSRC}` or `python -c 'import __graft_entry__ as g; g.build()'`")


def load() -> ctypes.CDLL:
    """Load libvss_amd.so (raises if it has not been built, or was built from other sources)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"VSS HIP library not found at {LIB_PATH}; build it with "
            f"`make -C {CSRC}` or `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    verify_source_hash(L)
    P, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    L.vss_abi_version.restype = ctypes.c_int
    L.vss_error_string.argtypes = [ctypes.c_int]
    L.vss_error_string.restype = ctypes.c_char_p
    L.vss_step.argtypes = [P, i64, i32, P, P, P]
    L.vss_step.restype = ctypes.c_int
    L.vss_step_replay.argtypes = [P, i64, i32, P, P, P, P]
    L.vss_step_replay.restype = ctypes.c_int
    L.vss_reset_dones_replay.argtypes = [P, i64, P, P, P]
    L.vss_reset_dones_replay.restype = ctypes.c_int
    L.vss_rollout.argtypes = [P, i64, i32, P, P, P]
    L.vss_rollout.restype = ctypes.c_int
    L.vss_reset_dones.argtypes = [P, i64, P, P]
    L.vss_reset_dones.restype = ctypes.c_int
    L.vss_compute_observations.argtypes = [P, i64, P, P, i32]
    L.vss_compute_observations.restype = ctypes.c_int
    L.vss_mlp_packed_size.argtypes = [i32]
    L.vss_mlp_packed_size.restype = i64
    L.vss_mlp_pack.argtypes = [P, i32, P, P, P]
    L.vss_mlp_pack.restype = ctypes.c_int
    L.vss_policy_forward.argtypes = [P, i64, i32, P, P, P, P, ctypes.c_uint64, ctypes.c_uint64] + [P] * 6
    L.vss_policy_forward.restype = ctypes.c_int
    L.vss_value_forward_masked.argtypes = [P, i64, i32, P, P, P, P, ctypes.c_uint64, ctypes.c_uint64] + [P] * 7
    L.vss_value_forward_masked.restype = ctypes.c_int
    L.vss_policy_sample.argtypes = [P, i64, i32, P, P, ctypes.c_uint64, ctypes.c_uint64, P, P, P, P]
    L.vss_policy_sample.restype = ctypes.c_int
    L.vss_episode_stats.argtypes = [P, i64] + [P] * 7
    L.vss_episode_stats.restype = ctypes.c_int
    L.vss_tanh_grad_chunks.argtypes = [i64, i32]
    L.vss_tanh_grad_chunks.restype = i64
    L.vss_tanh_grad_bias.argtypes = [P, i64, i32, P, P, P, P]
    L.vss_tanh_grad_bias.restype = ctypes.c_int
    L.vss_linear_tanh.argtypes = [P, i64, i32, i32, P, P, P, P]
    L.vss_linear_tanh.restype = ctypes.c_int
    L.vss_linear_tanh_out.argtypes = [P, i64, i32, i32, P, P, P, P, i32, P, P]
    L.vss_linear_tanh_out.restype = ctypes.c_int
    L.vss_linear_tanh_backward_chunks.argtypes = [i64, i32, i32]
    L.vss_linear_tanh_backward_chunks.restype = i64
    L.vss_linear_tanh_backward.argtypes = [P, i64, i32, i32, P, P, P, P, P]
    L.vss_linear_tanh_backward.restype = ctypes.c_int
    L.vss_output_backward_chunks.argtypes = [i64, i32, i32]
    L.vss_output_backward_chunks.restype = i64
    L.vss_output_backward.argtypes = [P, i64, i32, i32, P, P, P, P, P, P]
    L.vss_output_backward.restype = ctypes.c_int
    L.vss_linear_tanh_bf16x6.argtypes = [P, i64, i32, i32, P, P, P, P, P]
    L.vss_linear_tanh_bf16x6.restype = ctypes.c_int
    L.vss_linear_tanh_out_bf16x6.argtypes = [P, i64, i32, i32, P, P, P, P, i32, P, P, P]
    L.vss_linear_tanh_out_bf16x6.restype = ctypes.c_int
    L.vss_linear_tanh_backward_chunks_bf16x6.argtypes = [i64, i32, i32]
    L.vss_linear_tanh_backward_chunks_bf16x6.restype = i64
    L.vss_linear_tanh_backward_bf16x6.argtypes = [P, i64, i32, i32, P, P, P, P, P, P]
    L.vss_linear_tanh_backward_bf16x6.restype = ctypes.c_int
    L.vss_weight_grad_chunks_bf16x6.argtypes = [i64, i32, i32]
    L.vss_weight_grad_chunks_bf16x6.restype = i64
    L.vss_weight_grad_bf16x6.argtypes = [P, i64, i32, i32, P, P, P]
    L.vss_weight_grad_bf16x6.restype = ctypes.c_int
    L.vss_first_weight_grad_chunks_bf16x6.argtypes = [i64, i32, i32]
    L.vss_first_weight_grad_chunks_bf16x6.restype = i64
    L.vss_first_weight_grad_bf16x6.argtypes = [P, i64, i32, i32, P, P, P]
    L.vss_first_weight_grad_bf16x6.restype = ctypes.c_int
    L.vss_weight_planes_bf16x6.argtypes = [P, i32, P, P, P, P, P]
    L.vss_weight_planes_bf16x6.restype = ctypes.c_int
    f32 = ctypes.c_float
    L.vss_ppo_loss_scratch_floats.argtypes = [i64, i32]
    L.vss_ppo_loss_scratch_floats.restype = i64
    L.vss_ppo_loss.argtypes = [P, i64, i64, i32] + [P] * 8 + [f32] * 5 + [i32] + [P] * 6
    L.vss_ppo_loss.restype = ctypes.c_int
    L.vss_grad_sq_partials_count.argtypes = [i64]
    L.vss_grad_sq_partials_count.restype = i64
    L.vss_grad_sq_partials.argtypes = [P, i64, P, P]
    L.vss_grad_sq_partials.restype = ctypes.c_int
    L.vss_adam_step_clipped.argtypes = [P, i64, i32, P] + [f32] * 5 + [i64] + [P] * 5
    L.vss_adam_step_clipped.restype = ctypes.c_int
    L.vss_sum_parts.argtypes = [P, i32] + [P] * 8
    L.vss_sum_parts.restype = ctypes.c_int
    L.vss_output_backward_direct_chunks.argtypes = [i64, i32, i32]
    L.vss_output_backward_direct_chunks.restype = i64
    L.vss_output_backward_direct.argtypes = [P, i64, i32, i32, P, P, P, P, P, P]
    L.vss_output_backward_direct.restype = ctypes.c_int
    L.vss_ppo_loss_direct_scratch_floats.argtypes = [i64, i32]
    L.vss_ppo_loss_direct_scratch_floats.restype = i64
    L.vss_ppo_loss_direct.argtypes = ([P, i64, i64, i32, P, i32, P, P, i32, P] + [P] * 4 + [P, i32, ctypes.c_double]
                                      + [P, P] + [f32] * 5 + [i32] + [P] * 8)
    L.vss_ppo_loss_direct.restype = ctypes.c_int
    L.vss_minibatch_gather_parts.argtypes = [i64]
    L.vss_minibatch_gather_parts.restype = i64
    L.vss_minibatch_gather.argtypes = [P, i64, i64, i64, P, i64, i64] + [P] * 13
    L.vss_minibatch_gather.restype = ctypes.c_int
    L.vss_adv_part_sum.argtypes = [P, i32, P, P]
    L.vss_adv_part_sum.restype = ctypes.c_int
    L.vss_first_layer_bf16x6.argtypes = [P, i64, i32, i32, P, P, P, P]
    L.vss_first_layer_bf16x6.restype = ctypes.c_int
    L.vss_linear_tanh_loss_blocks_bf16x6.argtypes = [i64, i32, i32]
    L.vss_linear_tanh_loss_blocks_bf16x6.restype = i64
    L.vss_linear_tanh_loss_bf16x6.argtypes = ([P, i32, i64, i64, i32, i32, P, P, i32, P, P] + [P] * 4
                                              + [i32, ctypes.c_double] + [P] * 3 + [f32] * 4 + [i32] + [P] * 5)
    L.vss_linear_tanh_loss_bf16x6.restype = ctypes.c_int
    L.vss_ppo_loss_fused_finish.argtypes = [P, i64, i32, i64, P, i64, P, P, f32, f32] + [P] * 5
    L.vss_ppo_loss_fused_finish.restype = ctypes.c_int
    L.vss_randperm_scratch_bytes.argtypes = [i64]
    L.vss_randperm_scratch_bytes.restype = i64
    L.vss_randperm.argtypes = [P, i64, P, P, P, i64]
    L.vss_randperm.restype = ctypes.c_int
    L.vss_randperm_bits.argtypes = [P, i64, ctypes.c_int32, P, P, P, i64]
    L.vss_randperm_bits.restype = ctypes.c_int
    if L.vss_abi_version() != ABI_VERSION:
        raise NativeError(f"libvss_amd ABI {L.vss_abi_version()} != expected {ABI_VERSION}")
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().vss_error_string(rc).decode()
        raise NativeError(f"{what} failed: {msg} (code {rc})")


def ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def stream_of(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(device) -> torch.device:
    """The product path runs on a ROCm GPU only (no CPU fallback)."""
    device = torch.device(device)
    if device.type != "cuda":
        raise NativeError(f"VSS runs on a ROCm GPU (got device {device}); there is no CPU path")
    if not torch.cuda.is_available():
        raise NativeError("VSS needs a ROCm GPU but torch.cuda.is_available() is False")
    load()
    return device
