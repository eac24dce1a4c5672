"""The train loop's scalar writer (ppo_continuous_action_isaacgym.py:197-201 of the reference: a TensorBoard
SummaryWriter): TensorBoard when installed, else the same add_scalar calls appended to `<run>/scalars.csv`,
nothing on ranks other than 0 or with --log false."""
from __future__ import annotations

import os


class NullWriter:
    def add_scalar(self, *a, **k):
        pass

    def add_text(self, *a, **k):
        pass

    def close(self):
        pass


class CsvWriter:
    """The SummaryWriter calls the loop makes, appended to `<run>/scalars.csv` (tag,value,step)
    when TensorBoard is not installed, so the learning curves are kept either way."""

    def __init__(self, path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        self._f = open(path, "w")
        self._f.write("tag,value,step\n")

    def add_scalar(self, tag, value, step):
        self._f.write(f"{tag},{float(value)!r},{int(step)}\n")

    def add_text(self, *a, **k):
        pass

    def close(self):
        self._f.close()


def make_writer(args, run_name, rank):
    if rank != 0 or not args.log:
        return NullWriter()
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(f"{args.save_path}/{run_name}")
    except ImportError:  # tensorboard not installed
        return CsvWriter(f"{args.save_path}/{run_name}/scalars.csv")
