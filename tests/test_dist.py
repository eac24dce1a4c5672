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


_RCCL_SCRIPT = r"""
import os, sys
import torch, torch.distributed as dist
sys.path.insert(0, {pkg!r})
import ppo_continuous_action_isaacgym as P
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
assert dist.get_backend() == "nccl"
dev = torch.device("cuda:0")
net = torch.nn.Sequential(torch.nn.Linear(52, 256), torch.nn.Tanh(), torch.nn.Linear(256, 2)).to(dev)
fg = P.FlatGrads(net)
g = torch.Generator(device=dev).manual_seed(3)
fg.flat.copy_(torch.randn(fg.flat.numel(), device=dev, generator=g))
before = fg.flat.clone()
dist.all_reduce(fg.flat, op=dist.ReduceOp.SUM)  # the DP gradient exchange's collective, one rank
assert torch.equal(fg.flat, before)
assert net[0].weight.grad.data_ptr() == fg.flat.data_ptr()
adv = torch.randn(4096, device=dev, generator=g) * 3 + 1
glob = P.normalize_advantages(adv, world=2, global_stats=True)  # the all-reduced (sum, sumsq, n) path
loc = (adv - adv.mean()) / (adv.std() + 1e-8)
assert torch.allclose(glob, loc, rtol=1e-5, atol=1e-5), (glob - loc).abs().max()
t = torch.tensor([1.0, 2.0], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's timing reduce
assert t.tolist() == [1.0, 2.0]
dist.barrier()
dist.destroy_process_group()
print("RCCL_OK")
"""


@pytest.mark.gpu
def test_rccl_collectives_world1():
    """The RCCL ("nccl") code path on the real GPU: process-group init with a device id (as
    setup_distributed does for N>1), the flat-gradient all-reduce, the global advantage
    statistics' all-reduce (normalize_advantages) and bench.py's max-reduce, one rank.  RCCL
    refuses two ranks on one device, so more ranks than GPUs are rehearsed with gloo above."""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    script = _RCCL_SCRIPT.format(pkg=os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, cwd=REPO,
                       env=env)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
