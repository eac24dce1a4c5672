"""The C ABI driven from plain C (examples/vss_host_demo.c): hipMalloc'd buffers, reset, FULL
steps on a HIP stream, the misaligned-buffer refusal and state invariants — no Python or torch
in the process that runs the kernels."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_host_steps_65536_fields(tmp_path):
    out = os.path.join(tmp_path, "vss_host_demo")
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "examples"), f"OUT={out}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([out, "65536", "100"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["status"] == "ok" and res["bad_values"] == 0 and res["fields"] == 65536
    assert res["env_steps_per_s"] > 0
