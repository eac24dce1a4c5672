"""Reference-ordered reset draws -> the per-field rows of the replay C ABI — TEST INFRASTRUCTURE.

The golden fixtures (tests/golden/gen_golden.py) record every torch.rand output of the
reference's `reset_dones` (envs/vss.py:267-333) as one flat stream per call, in the reference's
batch order:

  round 0:  torch.rand((len(env_ids), 7, 2))        one (7, 2) row per resetting field, ascending
  round r:  torch.rand((len(close_ids), 7, 2))      rows only for the fields still too close
  yaws:     torch_rand_float(-pi, pi, (len(env_ids), 6))
  ball vel: torch.rand((len(env_ids), 2))

`vss_step_replay` / `vss_reset_dones_replay` (include/vss.h `vss_replay_draws`) take the same
draws regrouped per field: field f's row is its round chunks (14 each), then its 6 yaw draws and
its 2 ball-velocity draws.  Regrouping needs to know which fields were still too close after
each round; `to_rows` re-evaluates the reference's placement test (envs/vss.py:292-298) on the
drawn positions and checks the resulting round sizes against the sizes of the reference's own
torch.rand calls, which the fixtures record (`u_sizes`) -- so the grouping is the reference's,
not an assumption of this build.
"""
from __future__ import annotations

import numpy as np

SCALE = np.array([np.float32(1.5) - np.float32(0.14), np.float32(1.3) - np.float32(0.14)], np.float32)  # envs/vss.py:142-147
MIN_DIST = np.float32(0.07)  # min_robot_placement_dist, envs/vss.py:48-49
MAX_ROUNDS = 64  # the kernels' rejection bound (csrc/vss_step.hip kMaxRejectRounds)
PAIRS = [(i, j) for i in range(7) for j in range(i + 1, 7)]  # entities_pairs (all 21)


def too_close(chunks: np.ndarray) -> np.ndarray:
    """(m, 14) round draws -> (m,) bool: any of the 21 pair distances < 0.07 (envs/vss.py:292-298)."""
    pos = (chunks.reshape(-1, 7, 2).astype(np.float32) - np.float32(0.5)) * SCALE
    out = np.zeros(len(chunks), bool)
    for i, j in PAIRS:
        d = pos[:, i] - pos[:, j]
        out |= np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) < MIN_DIST
    return out


def to_rows(flat: np.ndarray, env_ids, n_fields: int, call_sizes=None):
    """Regroup one reset_dones call's draws into (n_fields, stride) rows; returns (rows, rounds)
    with rounds[f] = rejection rounds field f used (0 for fields that do not reset)."""
    flat = np.asarray(flat, np.float32)
    ids = [int(f) for f in env_ids]
    rounds = np.zeros(n_fields, np.int64)
    chunks: dict[int, list[np.ndarray]] = {f: [] for f in ids}
    pos, close, sizes = 0, list(ids), []
    while close:
        m = len(close)
        block = flat[pos:pos + 14 * m].reshape(m, 14)
        assert block.shape == (m, 14), "draw stream shorter than the rejection rounds need"
        pos += 14 * m
        sizes.append(14 * m)
        for i, f in enumerate(close):
            chunks[f].append(block[i])
            rounds[f] += 1
        close = [f for f, c in zip(close, too_close(block)) if c]
    k = len(ids)
    yaw = flat[pos:pos + 6 * k].reshape(k, 6)
    vel = flat[pos + 6 * k:pos + 8 * k].reshape(k, 2)
    if k:
        sizes += [6 * k, 2 * k]
    pos += 8 * k
    assert pos == len(flat), f"consumed {pos} of {len(flat)} reference draws"
    if call_sizes is not None:
        assert list(sizes) == [int(c) for c in call_sizes], f"round sizes {sizes} != reference calls {list(call_sizes)}"
    assert rounds.max(initial=0) <= MAX_ROUNDS, "more rejection rounds than the kernels bound (vss_step.hip kMaxRejectRounds)"
    stride = 14 * max(1, int(rounds.max(initial=0))) + 8
    rows = np.zeros((n_fields, stride), np.float32)
    for i, f in enumerate(ids):
        r = rounds[f]
        rows[f, :14 * r] = np.concatenate(chunks[f])
        rows[f, 14 * r:14 * r + 6] = yaw[i]
        rows[f, 14 * r + 6:14 * r + 8] = vel[i]
    return rows, rounds


def split_steps(flat: np.ndarray, counts) -> list[np.ndarray]:
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return [flat[off[t]:off[t + 1]] for t in range(len(counts))]
