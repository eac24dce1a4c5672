"""Top-down frames of one VSS field and a frame recorder — the build's stand-in for the Isaac Gym
viewer capture behind `capture_video` (ppo_continuous_action_isaacgym.py:213-221 wraps the env in
gym.wrappers.RecordVideo; play.py:134-142 records the first 300 steps of an evaluation).

Isaac Gym renders field 0 through its viewer camera (virtual_screen_capture); here `VSS.render`
copies field `env_id`'s state (one small D2H copy) and draws it with PIL: field and goal outlines
(envs/vss.py:342-345, 449-518), the ball (r = 0.02134), and each robot as its 0.07 m body square
rotated by its yaw, in team colour with a heading tick.  `RecordVideo` keeps gym 0.23's
constructor (video_folder, step_trigger, video_length, name_prefix) and writes animated GIFs
(there is no ffmpeg in the image).  Off the hot path: nothing here runs unless a frame is asked for.
"""
from __future__ import annotations

import math
import os

import numpy as np

# drawing extents (m): the whole arena incl. goal pockets (envs/vss.py:342-345: total 2.0 x 1.5)
ARENA_X, ARENA_Y = 1.0, 0.75
FIELD_HX, FIELD_HY, GOAL_HY, GOAL_BACK = 0.75, 0.65, 0.2, 0.85
BALL_R, ROBOT_HALF = 0.02134, 0.035  # robot collision box 0.07 x 0.07 (envs/vss_robot.urdf:2-20)
COLORS = {
    "grass": (34, 110, 52), "line": (235, 235, 235), "wall": (40, 40, 40), "ball": (255, 140, 0),
    "blue": (40, 90, 230), "yellow": (245, 215, 40), "tick": (250, 250, 250),
}


def _to_px(x, y, width, height):
    sx = (width - 1) / (2 * ARENA_X)
    sy = (height - 1) / (2 * ARENA_Y)
    return (x + ARENA_X) * sx, (ARENA_Y - y) * sy


def render_field(ball, robots, width: int = 400, height: int = 300) -> np.ndarray:
    """ball: (x, y); robots: (6, 3) rows (x, y, yaw) in the reference order (blue 0-2, yellow 0-2).
    Returns an (height, width, 3) uint8 frame."""
    from PIL import Image, ImageDraw

    img = Image.new("RGB", (width, height), COLORS["wall"])
    d = ImageDraw.Draw(img)
    px = lambda x, y: _to_px(x, y, width, height)  # noqa: E731
    # playing field and the two goal pockets
    d.rectangle([px(-FIELD_HX, FIELD_HY), px(FIELD_HX, -FIELD_HY)], fill=COLORS["grass"])
    for s in (-1, 1):
        x0, x1 = sorted((s * FIELD_HX, s * GOAL_BACK))
        d.rectangle([px(x0, GOAL_HY), px(x1, -GOAL_HY)], fill=COLORS["grass"])
    d.rectangle([px(-FIELD_HX, FIELD_HY), px(FIELD_HX, -FIELD_HY)], outline=COLORS["line"])
    d.line([px(0, FIELD_HY), px(0, -FIELD_HY)], fill=COLORS["line"])
    r = 0.2 * (width - 1) / (2 * ARENA_X)
    cx, cy = px(0, 0)
    d.ellipse([cx - r, cy - r, cx + r, cy + r], outline=COLORS["line"])
    # robots: body square rotated by yaw, heading tick from the centre to the front face
    for i, (x, y, yaw) in enumerate(np.asarray(robots, dtype=np.float64).reshape(6, 3)):
        c, s = math.cos(yaw), math.sin(yaw)
        corners = [px(x + c * u - s * v, y + s * u + c * v)
                   for u, v in ((ROBOT_HALF, ROBOT_HALF), (-ROBOT_HALF, ROBOT_HALF),
                                (-ROBOT_HALF, -ROBOT_HALF), (ROBOT_HALF, -ROBOT_HALF))]
        d.polygon(corners, fill=COLORS["blue" if i < 3 else "yellow"])
        d.line([px(x, y), px(x + c * ROBOT_HALF, y + s * ROBOT_HALF)], fill=COLORS["tick"], width=2)
    bx, by = px(float(ball[0]), float(ball[1]))
    br = max(2.0, BALL_R * (width - 1) / (2 * ARENA_X))
    d.ellipse([bx - br, by - br, bx + br, by + br], fill=COLORS["ball"])
    return np.asarray(img, dtype=np.uint8)


def write_gif(frames, path: str, fps: int = 20) -> str:
    from PIL import Image

    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    imgs = [Image.fromarray(f) for f in frames]
    imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=int(1000 / fps), loop=0)
    return path


class FrameRecorder:
    """gym 0.23 RecordVideo's trigger logic (step_trigger(step_id) starts a clip of video_length
    frames) without the env wrapping; `RecordVideo` and play.py's evaluation use it."""

    def __init__(self, render, video_folder: str, step_trigger, video_length: int = 100,
                 name_prefix: str = "rl-video"):
        self.render, self.video_folder = render, video_folder
        self.step_trigger, self.video_length, self.name_prefix = step_trigger, int(video_length), name_prefix
        self.step_id, self.frames, self.start, self.paths = 0, None, 0, []

    def on_step(self):
        if self.frames is None and self.step_trigger(self.step_id):
            self.frames, self.start = [], self.step_id
        if self.frames is not None:
            self.frames.append(self.render())
            if len(self.frames) >= self.video_length:
                self.flush()
        self.step_id += 1

    def flush(self):
        if self.frames:
            path = os.path.join(self.video_folder, f"{self.name_prefix}-step-{self.start}.gif")
            self.paths.append(write_gif(self.frames, path))
        self.frames = None


class RecordVideo:
    """gym.wrappers.RecordVideo(env, video_folder, step_trigger, video_length, name_prefix) as the
    reference uses it (ppo…:213-221, play.py:134-142): forwards everything to `env`, and records
    `env.render("rgb_array")` after each step of a triggered clip."""

    def __init__(self, env, video_folder: str, step_trigger=None, video_length: int = 100,
                 name_prefix: str = "rl-video", episode_trigger=None):
        if step_trigger is None:
            step_trigger = (lambda step: step == 0) if episode_trigger is None else episode_trigger
        self.env = env
        self.recorder = FrameRecorder(lambda: env.render("rgb_array"), video_folder, step_trigger, video_length,
                                      name_prefix)

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, action):
        out = self.env.step(action)
        self.recorder.on_step()
        return out

    def close(self):
        self.recorder.flush()
        return getattr(self.env, "close", lambda: None)()
