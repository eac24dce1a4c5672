"""Build libvss_amd.so for gfx950 (hipcc cross-compiles; no GPU needed)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")


def build(arch: str = "gfx950", verbose: bool = False) -> str:
    out = os.path.join(HERE, "libvss_amd.so")
    cmd = ["make", "-C", CSRC, f"ARCH={arch}"]
    if not verbose:
        cmd.insert(1, "-s")
    subprocess.run(cmd, check=True)
    if not os.path.exists(out):
        raise RuntimeError(f"build did not produce {out}")
    return out
