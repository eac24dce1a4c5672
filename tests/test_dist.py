"""Multi-rank paths on CPU (gloo, world size 2) and, on the GPU box, bench.py with 2 ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reduce_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, REPO)
    import bench
    q.put((rank, bench.reduce_max([1.0 + rank, 5.0 - rank])))
    dist.destroy_process_group()


def test_bench_timing_is_max_over_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_reduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert out[0] == out[1] == [2.0, 5.0]


@pytest.mark.gpu
@pytest.mark.parametrize("launcher", ["torchrun", "self"])
def test_bench_two_ranks_rehearsal(launcher):
    """bench.py as the driver launches it for N>1 (torch.distributed.run) and as a user runs it
    by hand (`bench.py --gpus 2` starts the launcher itself), 2 ranks sharing the one GPU with
    gloo for the barrier/timing reduce: one JSON line, value counts both ranks; the PPO leg runs
    on both ranks with the gradient all-reduce and reports whole-job env-steps."""
    port = _free_port()
    run = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] if launcher == "torchrun" else [sys.executable]
    cmd = run + [os.path.join(REPO, "bench.py"),
                 "--gpus", "2", "--steps", "20", "--warmup", "2", "--fields", "8192", "--dist-backend", "gloo",
                 "--share-gpu", "--no-cpu-baseline",
                 "--ppo-updates", "1", "--rollout-k", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["scaling"] == "weak" and j["value"] > 0
    assert abs(j["value"] - 2 * 8192 * 20 / (j["ms_per_step"] * 1e-3 * 20)) / j["value"] < 1e-6
    ppo = j["ppo"]
    assert ppo["n_gpus"] == 2 and ppo["num_envs"] == 2 * 8192 and ppo["batch"] == 2 * 8192 * 128
    assert "all-reduce" in ppo["gradient_exchange"] and ppo["train_env_steps_per_s"] > 0
