"""Frames for capture_video / play.py video (envs/render.py): the top-down drawing of one field,
VSS.render on the device state, and the RecordVideo / play_matches recorders (GIF clips)."""
import os

import numpy as np
import pytest
import torch

from envs.render import COLORS, FrameRecorder, _to_px, render_field


def _at(frame, x, y):
    px, py = _to_px(x, y, frame.shape[1], frame.shape[0])
    return tuple(frame[int(round(py)), int(round(px))])


def test_render_field_draws_ball_robots_and_field():
    robots = np.array([[-0.5, 0.3, 0.0], [-0.3, -0.3, 1.0], [-0.1, 0.5, 2.0],
                       [0.5, 0.3, 0.0], [0.3, -0.3, -1.0], [0.1, -0.5, 3.0]])
    f = render_field((0.25, 0.1), robots)
    assert f.shape == (300, 400, 3) and f.dtype == np.uint8
    assert _at(f, 0.25, 0.1) == COLORS["ball"]
    assert _at(f, -0.3, -0.3 + 0.02) == COLORS["blue"]      # off the heading tick
    assert _at(f, 0.3, -0.3 + 0.02) == COLORS["yellow"]
    assert _at(f, 0.4, 0.45) == COLORS["grass"]
    assert _at(f, 0.95, 0.6) == COLORS["wall"]             # outside the field, beside a goal
    assert _at(f, 0.8, 0.0) == COLORS["grass"]             # inside a goal pocket


def test_frame_recorder_trigger_and_length(tmp_path):
    frames = iter(range(1000))
    rec = FrameRecorder(lambda: np.full((4, 4, 3), next(frames) % 255, np.uint8), str(tmp_path),
                        lambda step: step % 10 == 0, video_length=3, name_prefix="clip")
    for _ in range(25):
        rec.on_step()
    rec.flush()
    names = sorted(os.path.basename(p) for p in rec.paths)
    assert names == ["clip-step-0.gif", "clip-step-10.gif", "clip-step-20.gif"]
    from PIL import Image
    assert Image.open(rec.paths[0]).n_frames == 3


@pytest.mark.gpu
def test_vss_render_and_record_video_gpu(tmp_path):
    from envs.render import RecordVideo
    from envs.vss import VSS, default_cfg
    from envs.wrappers import SingleAgent
    from vss_amd import _native as N
    env = VSS(default_cfg(64), "cuda:0", "cuda:0", 0, True, False, False)
    s = env.state[:, 5].cpu().numpy().astype(np.float64)
    yaw = np.arctan2(2 * s[N.CH_RQW:N.CH_RQW + 6] * s[N.CH_RQZ:N.CH_RQZ + 6],
                     s[N.CH_RQW:N.CH_RQW + 6] ** 2 - s[N.CH_RQZ:N.CH_RQZ + 6] ** 2)
    want = render_field(s[[0, 1]], np.stack([s[N.CH_RX:N.CH_RX + 6], s[N.CH_RY:N.CH_RY + 6], yaw], 1))
    assert np.array_equal(env.render("rgb_array", env_id=5), want)
    assert env.render("human") is None
    W = RecordVideo(SingleAgent(env), str(tmp_path), step_trigger=lambda t: t % 4 == 0, video_length=2)
    for _ in range(6):
        W.step(torch.zeros(64, 2, device="cuda"))
    W.close()
    from PIL import Image
    files = sorted(os.listdir(tmp_path))
    assert files == ["rl-video-step-0.gif", "rl-video-step-4.gif"]
    assert Image.open(os.path.join(tmp_path, files[0])).n_frames == 2


@pytest.mark.gpu
def test_play_matches_video_gpu(tmp_path):
    from envs.vss import VSS, default_cfg
    from play import get_team, play_matches
    env = VSS(default_cfg(256), "cuda:0", "cuda:0", 0, True, False, False)
    env.w_goal, env.w_grad, env.w_move, env.w_energy = 1.0, 0.0, 0.0, 0.0
    play_matches(env, get_team("ou"), get_team("zero"), 4, video_path=str(tmp_path))
    from PIL import Image
    gif = os.path.join(tmp_path, "video.000-step-0.gif")
    assert os.path.exists(gif) and Image.open(gif).n_frames >= 1
