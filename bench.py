#!/usr/bin/env python3
"""Benchmark of the hot path: the VSS match step (BASELINE.json north_star) on MI355X.

One *step* = one `vss_step` launch advancing every field of this rank by one control step
(dt = 0.05 s) under synthetic random actions, with the reference's full VecTask.step output
contract (obs + terminal obs (N,2,3,52), rewards (N,2,3,4), dones, time-outs, progress) —
BASELINE.json configs[1]/[2] at 65,536 fields per GPU.  Fields are independent, so ranks shard
them with no data-path collective (weak scaling); the only collectives are the timing barrier
and the max-over-ranks of the elapsed time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--fields F] [--mode full|sa|cma|dma]

Rank 0 prints ONE JSON line (value = env-steps/s summed over all ranks = fields x ranks x K /
max-over-ranks time).  `roofline.achieved` = algorithmic bytes per launch / mean launch time
measured with HIP events on the launch stream; `cpu_baseline` = the C oracle (oracle/, the only
use of it here) on the host's cores (one 4,096-field shard per thread, up to 16: 65,536 fields on a 16-core share) over a bounded
sample, with one-thread rates at the SURVEY §8(d) shapes (16 fields x 1,000 steps = config 1,
4,096 and 65,536 fields) beside it.  `past_l3` repeats the FULL timing at 131,072 fields, whose
406 MB per launch cannot sit in the 256 MiB Infinity Cache, so its fraction is HBM-backed.
`roofline.traffic` comes from the committed rocprofv3 PMC passes (profiles/pmc_traffic*.json,
tools/pmc_summary.py) and is reported only if that profile was taken of the current
csrc/vss_step.hip (source hash), else null.
"""
from __future__ import annotations

import argparse
import gc
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# before anything initialises the GPU: the PPO legs run with ROCm's graph packet capture off, and the
# captured minibatch checks that the runtime started that way (vss_amd.minibatch; it also checks itself)
from vss_amd.minibatch import disable_graph_packet_capture  # noqa: E402

disable_graph_packet_capture()

METRIC = "env-steps/s (num_envs×horizon) at 65 536 envs; PPO wall-clock to 1e8 steps"
HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip table (spec)

# Algorithmic HBM bytes per field-step of each contract:
#   state 46 live fp32 channels read+write (368), progress/reset int64 r+w (32), rng counter r+w (8)
#   FULL: actions 48 + dof_velocity_buf write 48 + obs 1248 + terminal obs 1248 + rew 96
#         + time_out 1 + progress_f 4                                           = 3101 B
#   SA:   learner action 8 + OU buffer r+w 96 + dof 48 + obs 208 + terminal obs 208 + rew 16
#         + reward 4 + time_out 1 + progress_f 4                                  = 1001 B
BYTES = {
    "full": 368 + 32 + 8 + 48 + 48 + 1248 + 1248 + 96 + 1 + 4,
    "sa": 368 + 32 + 8 + 8 + 96 + 48 + 208 + 208 + 16 + 4 + 1 + 4,
    "cma": 368 + 32 + 8 + 24 + 96 + 48 + 208 + 208 + 16 + 4 + 1 + 4,
    "dma": 368 + 32 + 8 + 24 + 96 + 48 + 624 + 624 + 48 + 12 + 24 + 3 + 12,
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--fields", type=int, default=65536, help="fields (3v3 matches) per GPU")
    p.add_argument("--mode", default="full", choices=["full", "sa", "cma", "dma"])
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--rollout-k", type=int, default=16,
                   help="also time vss_rollout with K steps per launch (0 = skip)")
    p.add_argument("--ppo-updates", type=int, default=None,
                   help="PPO-SA training updates run after the env-step benchmark, on every rank (default: until "
                        "1e8 env-steps, 12 at 65,536 envs on one GPU; the train clock at 1e8 is the metric's "
                        "second half; 0 = skip)")
    p.add_argument("--ppo-dma-updates", type=int, default=2,
                   help="PPO-DMA updates at the same fields per GPU (3 agent rows per field, BASELINE config 4); "
                        "the last one is timed (0 = skip)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (= RCCL) for real multi-GPU runs; gloo + --share-gpu to rehearse ranks on one GPU")
    p.add_argument("--share-gpu", action="store_true", help="map every rank to cuda:0 (rehearsal only)")
    p.add_argument("--graph", type=int, default=0, help="replay the launches from a HIP graph (1) or launch eagerly (0)")
    p.add_argument("--l3-check-fields", type=int, default=131072,
                   help="FULL launches timed again at this many fields (past the 256 MiB Infinity Cache; 0 = skip)")
    return p.parse_args()


def _oracle_shard(O, n: int, seed: int, deadline: float, out: list, slot: int):
    """One host thread stepping its own n-field oracle shard until `deadline` (the C call
    releases the GIL, so shards run in parallel)."""
    h = O.HostEnv(n)
    prm = O.params(seed=seed)
    O.reset_dones(h, prm)
    io = O.make_io(n, O.MODE_FULL)
    gen = np.random.default_rng(seed)
    acts = [gen.uniform(-1, 1, (n, 12)).astype(np.float32) for _ in range(8)]
    steps = 0
    while time.perf_counter() < deadline:
        O.step(h, O.MODE_FULL, acts[steps % 8], io, prm)
        steps += 1
    out[slot] = steps


def host_threads() -> int:
    """Host cores this process may use, capped at 16 (the GPU box's CPU share per GPU)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(16, avail))


def _oracle_fixed(O, n: int, steps: int, seed: int = 1) -> float:
    """One thread, n fields, exactly `steps` steps: env-steps/s."""
    h = O.HostEnv(n)
    prm = O.params(seed=seed)
    O.reset_dones(h, prm)
    io = O.make_io(n, O.MODE_FULL)
    gen = np.random.default_rng(seed)
    acts = [gen.uniform(-1, 1, (n, 12)).astype(np.float32) for _ in range(8)]
    t0 = time.perf_counter()
    for k in range(steps):
        O.step(h, O.MODE_FULL, acts[k % 8], io, prm)
    return n * steps / (time.perf_counter() - t0)


def cpu_baseline(seconds: float):
    """The C oracle on the same workload shape (FULL contract, random actions).  Reported value:
    one 4,096-field shard per available core (up to 16 = 65,536 fields), ≈1/2 of the budget.
    Beside it, one thread at the SURVEY §8(d) shapes: 16 fields x 1,000 steps (config 1),
    4,096 fields (≈1/4 of the budget) and 65,536 fields (≈1/4)."""
    import threading

    import oracle as O
    n = 4096
    res = {}
    shapes = {"16_fields_x_1000_steps_1_thread": _oracle_fixed(O, 16, 1000)}
    t0 = time.perf_counter()
    big_steps = 0
    h = O.HostEnv(65536)
    prm = O.params(seed=3)
    O.reset_dones(h, prm)
    io = O.make_io(65536, O.MODE_FULL)
    a = np.random.default_rng(3).uniform(-1, 1, (65536, 12)).astype(np.float32)
    while time.perf_counter() - t0 < seconds / 4 or big_steps < 2:
        O.step(h, O.MODE_FULL, a, io, prm)
        big_steps += 1
    shapes["65536_fields_1_thread"] = 65536 * big_steps / (time.perf_counter() - t0)
    for threads, share in ((1, 1 / 4), (host_threads(), 1 / 2)):
        counts = [0] * threads
        t0 = time.perf_counter()
        deadline = t0 + seconds * share
        pool = [threading.Thread(target=_oracle_shard, args=(O, n, 1 + i, deadline, counts, i)) for i in range(threads)]
        for t in pool:
            t.start()
        for t in pool:
            t.join()
        el = time.perf_counter() - t0
        res[threads if threads == 1 else "all"] = (n * sum(counts) / el, counts, el, threads)
    v1, c1, e1, _ = res[1]
    vn, cn, en, tn = res["all"]
    shapes["4096_fields_1_thread"] = v1
    shapes[f"{tn * n}_fields_{tn}_threads"] = vn
    return {"value": vn, "unit": "env-steps/s", "cores": tn, "kind": "port",
            "single_thread_value": v1, "shapes": shapes,
            "sample": f"oracle/vss_oracle.c FULL contract, random actions, {tn} host threads x {n} fields "
                      f"({sum(cn)} shard-steps in {en:.1f} s; 1 thread: {n} fields x {c1[0]} steps in "
                      f"{e1:.1f} s = {v1:.3g} env-steps/s; 65,536 fields x {big_steps} steps on 1 thread; "
                      f"16 fields x 1,000 steps on 1 thread), host CPU: {cpu_model()}"}


def step_source_sha() -> str:
    with open(os.path.join(REPO, "rsoccer-isaac-cleanrl_amd", "csrc", "vss_step.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def past_l3_leg(n: int, steps: int, dev) -> dict:
    """FULL launches at `n` fields (131,072 by default: 406 MB per launch, past the 256 MiB
    Infinity Cache) timed with HIP events on the launch stream: the HBM-backed fraction."""
    from envs.vss import VSS, default_cfg
    from vss_amd import _native as N
    cfg = default_cfg(n)
    cfg["env"]["seed"] = 11
    env = VSS(cfg, str(dev), str(dev), 0, True, False, False)
    gen = torch.Generator(device=dev).manual_seed(77)
    pool = [torch.rand((n, 12), device=dev, generator=gen) * 2 - 1 for _ in range(4)]
    lib, stream = N.load(), N.stream_of(dev)
    prm, st = env._c_params(), env._c_state()
    cios = [N.VssStepIO(a.data_ptr(), None, N.ptr(env.obs_buf), N.ptr(env.terminal_obs_buf), N.ptr(env.rew_buf),
                        None, None, N.ptr(env.timeout_buf), N.ptr(env.progress_f_buf)) for a in pool]
    byref = N.ctypes.byref
    for k in range(10):
        N.check(lib.vss_step(stream, n, N.MODE_FULL, byref(prm), byref(st), byref(cios[k % 4])), "vss_step")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rc = 0
    e0.record()
    for k in range(steps):
        rc |= lib.vss_step(stream, n, N.MODE_FULL, byref(prm), byref(st), byref(cios[k % 4]))
    e1.record()
    torch.cuda.synchronize()
    N.check(rc, "vss_step (past_l3 timed launches)")  # a failed launch must not report a rate
    ms = e0.elapsed_time(e1) / steps
    algo = BYTES["full"] * n
    del env
    torch.cuda.empty_cache()
    return {"fields": n, "launches": steps, "kernel_ms": ms, "algorithmic_bytes_per_launch": algo,
            "achieved": algo / (ms * 1e-3) / 1e9, "unit": "GB/s", "frac": algo / (ms * 1e-3) / HBM_PEAK,
            "env_steps_per_s": n / (ms * 1e-3)}


def rollout_leg(env, K: int, steps: int, gen, dev, allocations: int = 6) -> dict:
    """vss_rollout: K FULL steps per launch for a pre-supplied random action sequence (the
    open-loop form of the same workload; state on chip between steps).  Bytes per field-step:
    actions 48 + obs 1248 + terminal obs 1248 + rew 96 + done 8 + time-out 1 + progress 4, plus
    the state / bookkeeping / dof read+write (456 B) once per launch.

    The launch time depends on the physical pages behind the K-step output streams (DESIGN §5.1:
    30.5-34.3 us per step over fresh allocations, reproducible within one), so the launches are
    timed on `allocations` output buffers held at the same time (distinct pages) and the line reports
    the MEDIAN allocation, with the spread beside it."""
    n = env.num_fields
    # episodes desynchronised (progress uniform over the episode length, as in a running training
    # loop) rather than all at the progress the FULL leg left; the progress distribution was measured
    # not to move this figure (profiles/r02_rollout_progress_distribution.log)
    env.progress_buf.random_(0, int(env.max_episode_length), generator=gen)
    acts = torch.rand((K, n, 2, 3, 2), device=dev, generator=gen) * 2 - 1
    outs = [env.rollout(acts) for _ in range(allocations)]
    launches = max(1, steps // K)
    per_alloc_ms, walls = [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for out in outs:
        env.rollout(acts, out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(launches):
            env.rollout(acts, out)
        e1.record()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        per_alloc_ms.append(e0.elapsed_time(e1) / launches)
    del outs
    torch.cuda.empty_cache()
    order = sorted(range(allocations), key=lambda i: per_alloc_ms[i])
    med = order[allocations // 2]
    launch_ms = per_alloc_ms[med]
    per_step_bytes = 48 + 1248 + 1248 + 96 + 8 + 1 + 4
    algo = n * (K * per_step_bytes + 368 + 32 + 8 + 48)
    achieved = algo / (launch_ms * 1e-3)
    fr = [algo / (ms * 1e-3) / HBM_PEAK for ms in per_alloc_ms]
    return {"steps_per_launch": K, "launches": launches, "value": n * K * launches / walls[med], "unit": "env-steps/s",
            "ms_per_step": launch_ms / K,
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, "algorithmic_bytes_per_launch": algo, "kernel_ms": launch_ms,
                         "allocations": allocations, "statistic": "median over the output allocations",
                         "frac_min": min(fr), "frac_max": max(fr),
                         "ms_per_step_each_allocation": [round(ms / K, 5) for ms in per_alloc_ms]}}


def sa_leg(env, steps: int, gen, dev) -> dict:
    """The SA contract (SingleAgent fused into the step: what ppo-sa drives) on the same fields,
    after the FULL measurement: `steps` launches timed with HIP events on the launch stream."""
    from envs import wrappers as Wr
    from vss_amd import _native as N
    n = env.num_fields
    W = Wr.SingleAgent(env)
    pool = [torch.rand((n, 2), device=dev, generator=gen) * 2 - 1 for _ in range(16)]
    io = dict(ou_buf=W.action_buf, obs=W._obs, terminal_obs=W._terminal_obs, rew=W._rews,
              reward_sum=W._reward, dones_rep=None, time_outs=W._time_outs, progress_f=W._progress)
    for k in range(20):
        env.native_step(N.MODE_SA, pool[k % 16], io)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for k in range(steps):
        env.native_step(N.MODE_SA, pool[k % 16], io)
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / steps
    algo = BYTES["sa"] * n
    achieved = algo / (ms * 1e-3)
    return {"value": n * steps / wall, "unit": "env-steps/s", "steps": steps, "ms_per_step": ms,
            "note": "wall time includes the Python wrapper's per-call buffer checks; kernel time is ms_per_step",
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, "algorithmic_bytes_per_launch": algo, "kernel_ms": ms}}


def ppo_updates_to_1e8(n_envs: int, world: int, num_steps: int = 128) -> int:
    """Updates until the global step count reaches 1e8 (ceil; the reference's total_timesteps //
    batch_size with --total-timesteps 1e8 stops one update short of it)."""
    import math
    return math.ceil(1e8 / (n_envs * num_steps * world))


def ppo_wallclock(n_envs: int, updates: int, dev, world: int = 1) -> dict:
    """The full SA PPO loop (ppo_continuous_action_isaacgym.py, reference defaults: T=128,
    8 epochs x 4 minibatches, fp32) at `n_envs` envs per rank, for `updates` updates (by default
    until 1e8 env-steps: 12 at 65,536 envs on one GPU).  `wallclock_to_1e8_steps_s` is MEASURED: the
    train loop's own clock (ppo…:244, start before envs.reset()) at the end of the first update whose
    global step reaches 1e8; the last update's rollout + update times projected to 1e8 are kept as
    `projected_*`.  Runs on EVERY rank: at N > 1 each rank owns its own `n_envs` fields and the
    gradients are averaged by one flat all-reduce per minibatch (RCCL), so the figures here are
    max-over-ranks times and whole-job (all-rank) env-steps."""
    import ppo_continuous_action_isaacgym as P
    from vss_amd import minibatch as MB, mlp as M
    args = P.parse_args(["--env-id", "sa", "--num-envs", str(n_envs), "--num-updates", str(updates),
                         "--log", "false", "--seed", "1"])
    torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    _, hist = P.train(args)
    call_s = time.perf_counter() - t0
    mem = device_memory(dev)
    last = hist[-1]
    red = dev if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu"
    roll_s, upd_s, call_s = reduce_max([last["rollout_s"], last["update_s"], call_s], red)
    walls = reduce_max([h["wall_s"] for h in hist], red)
    per_update = roll_s + upd_s
    batch = args.batch_size * world
    # steady state vs first use: each update's share of the train clock (max over ranks); the steady
    # figure is the median over updates 2.. (the first carries the first kernel uses, the graph capture
    # and the env reset); the 1e8 wall-clock at N GPUs = first update + (updates - 1) x steady, so the
    # scaling of train throughput is read from steady_train_env_steps_per_s, not from the 1e8 clock
    # (quantised: 12 updates at 1 GPU, 2 at 8)
    deltas = [walls[0]] + [b - a for a, b in zip(walls, walls[1:])]
    steady = float(np.median(deltas[1:])) if len(deltas) > 1 else None
    updates_1e8 = ppo_updates_to_1e8(n_envs, world, args.num_steps)
    reached = next((i for i, h in enumerate(hist) if h["global_step"] >= 1e8), None)
    ref_updates = int(1e8) // batch  # the reference's num_updates for --total-timesteps 1e8 (ppo…:247)
    return {"env": "sa", "n_gpus": world, "num_envs": n_envs * world, "num_envs_per_gpu": n_envs,
            "num_steps": args.num_steps, "batch": batch, "update_epochs": args.update_epochs,
            "num_minibatches": args.num_minibatches, "dtype": "f32",
            "update_gemm": {"x6": "fp32 arithmetic on the bf16 matrix cores (exact 3-way bf16 split, six partial "
                                  "products, fp32 accumulation; csrc/vss_gemm_x6.hip)",
                            "fp32": "fp32 MFMA (csrc/vss_update.hip)"}.get(M.UPDATE_GEMM, M.UPDATE_GEMM),
            "update_minibatch": ("one captured HIP graph per minibatch (forward, losses, backward), "
                                 f"rows padded to {MB.MLP_ROW_PAD}, replay {MB.GRAPH_CHECK_REPLAY} checked against eager"
                                 if args.update_graph else "eager"),
            "graph_packet_capture_env": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "<unset>"),
            "gradient_exchange": ("one flat fp32 all-reduce per minibatch "
                                  f"({dist.get_backend() if dist.is_initialized() else 'none'})") if world > 1 else "none",
            "updates_run": len(hist), "env_steps_run": hist[-1]["global_step"],
            "wallclock_to_1e8_steps_s": walls[reached] if reached is not None else None,
            "wallclock_to_1e8_steps": ("measured: train() clock at the end of update "
                                       f"{reached + 1} ({hist[reached]['global_step']} env-steps)")
            if reached is not None else f"not reached in {len(hist)} updates (see projected_wallclock_to_1e8_steps_s)",
            "wallclock_reference_num_updates_s": walls[ref_updates - 1] if 0 < ref_updates <= len(hist) else None,
            "reference_num_updates": ref_updates,
            "wall_s_per_update": walls, "train_call_s": call_s,
            "rollout_s": roll_s, "update_s": upd_s, "timed_update": len(hist),
            "rollout_env_steps_per_s": batch / roll_s, "train_env_steps_per_s": batch / per_update,
            "steady_s_per_update": steady,
            "steady_train_env_steps_per_s": batch / steady if steady else None,
            "first_update_s": deltas[0],
            "first_update_overhead_s": deltas[0] - steady if steady else None,
            "steady_state_note": ("steady = median of the per-update train-clock deltas after the first (max over "
                                  "ranks); first_update_overhead_s = the first update's delta minus it (env reset, the "
                                  "minibatch graph capture, remaining first uses)"),
            "kernel_warmup_s": getattr(args, "kernel_warmup_s", 0.0),
            "graph_prepare_s": getattr(args, "graph_prepare_s", 0.0),
            "kernel_warmup": ("BEFORE the train clock (ppo…:244), outside wallclock_to_1e8_steps_s: one 8-step update of "
                              "the same loop on a throwaway 16,384-env env and Agent copy (--kernel-warmup, "
                              "warmup_kernels), so the runtime's first-use code-object loading of the loop's kernels "
                              "happens before the clock; RNG states restored, training unchanged"
                              if getattr(args, "kernel_warmup", False) else "off"),
            "projected_wallclock_to_1e8_steps_s": updates_1e8 * per_update, "updates_to_1e8": updates_1e8,
            "device_memory": mem}


def device_memory(dev) -> dict:
    """This rank's device memory after a leg: the caching allocator's peaks over the leg (the minibatch graph's
    pool included) and the device's free memory as the driver reports it (all processes on the device)."""
    free, total = torch.cuda.mem_get_info(dev)
    return {"max_reserved_gib": torch.cuda.max_memory_reserved(dev) / 2 ** 30,
            "max_allocated_gib": torch.cuda.max_memory_allocated(dev) / 2 ** 30,
            "reserved_gib_after": torch.cuda.memory_reserved(dev) / 2 ** 30,
            "device_free_gib_after": free / 2 ** 30, "device_total_gib": total / 2 ** 30}


def ppo_dma_leg(n_fields: int, updates: int, dev, world: int = 1) -> dict:
    """BASELINE config 4: PPO-DMA (decentralised: every blue robot one agent row, envs/wrappers.py:
    150-180) at `n_fields` fields per rank = 3 x n_fields agent rows, reference defaults; the last
    update's rollout and update times (max over ranks)."""
    import ppo_continuous_action_isaacgym as P
    args = P.parse_args(["--env-id", "dma", "--num-envs", str(3 * n_fields), "--num-updates", str(updates),
                         "--log", "false", "--seed", "1"])
    torch.cuda.reset_peak_memory_stats(dev)
    _, hist = P.train(args)
    mem = device_memory(dev)
    last = hist[-1]
    red = dev if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu"
    roll_s, upd_s, first_upd_s = reduce_max([last["rollout_s"], last["update_s"], hist[0]["update_s"]], red)
    walls = reduce_max([h["wall_s"] for h in hist], red)
    deltas = [walls[0]] + [b - a for a, b in zip(walls, walls[1:])]
    steady = float(np.median(deltas[1:])) if len(deltas) > 1 else None
    rows = args.num_envs * world
    return {"env": "dma", "n_gpus": world, "fields_per_gpu": n_fields, "agent_rows": rows,
            "num_steps": args.num_steps, "batch": args.batch_size * world, "minibatch_rows": args.minibatch_size,
            "updates_run": len(hist), "rollout_s": roll_s, "update_s": upd_s,
            "first_update_s": deltas[0], "steady_s_per_update": steady,
            "kernel_warmup_s": getattr(args, "kernel_warmup_s", 0.0), "graph_prepare_s": getattr(args, "graph_prepare_s", 0.0),
            "first_update_update_s": first_upd_s, "first_to_steady_update_ratio": first_upd_s / upd_s,
            "first_update_note": ("first_update_s / steady_s_per_update: the train clock's first delta and the median of "
                                  "the later ones (max over ranks); first_update_update_s: the first update's update phase "
                                  "(it holds the eager first minibatch, the capture and the replay-12 self-check, all in "
                                  "one memory pool) against the last one's update_s"),
            "rollout_agent_steps_per_s": rows * args.num_steps / roll_s,
            "train_agent_steps_per_s": rows * args.num_steps / (roll_s + upd_s),
            "mean_return_last": last["mean_return"], "v_loss_last": last["v_loss"], "entropy_last": last["entropy"],
            "update_s_per_update": [h["update_s"] for h in hist], "device_memory": mem}


def update_gemm_roofline(dev, rows: int = 2097152, reps: int = 10) -> dict:
    """The update's dominant kernel, the 512 -> 512 hidden-layer forward in fp32 arithmetic on the bf16
    matrix cores (csrc/vss_gemm_x6.hip), at the update's minibatch size, timed with HIP events on its
    launch stream.  Achieved = fp32 FLOP (2 rows K N) / launch time; peaks: the x6 form's (the dense bf16
    MFMA rate / 6 products, MI355X_MICROARCH.md ~2.5 PF dense bf16) and the fp32 MFMA peak."""
    from vss_amd.update import linear_tanh_x6
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.tanh(torch.randn(rows, 512, device=dev, generator=g))
    w = torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5
    b = torch.zeros(512, device=dev)
    y = torch.empty(rows, 512, device=dev)
    for _ in range(2):
        linear_tanh_x6(x, w, b, out=y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        linear_tanh_x6(x, w, b, out=y)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = 2.0 * rows * 512 * 512 / (ms * 1e-3) / 1e12
    peak_x6, peak_fp32 = 2500.0 / 6, 157.3
    del x, y
    torch.cuda.empty_cache()
    return {"kernel": "vss_linear_tanh_bf16x6 512->512 (update forward, 2,097,152 rows)", "bound": "mfma",
            "achieved": tf, "peak": peak_x6, "unit": "TFLOP/s (fp32 FLOP)", "frac": tf / peak_x6,
            "fp32_mfma_peak": peak_fp32, "vs_fp32_mfma_peak": tf / peak_fp32, "kernel_ms": ms}


def reduce_max(values, device="cpu"):
    """Max over ranks of the per-rank timings (the only cross-rank data besides barriers)."""
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` by hand: start the one-process-per-GPU launcher as a child
        # (no exec, nothing has touched the GPU yet) and exit with its status
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    # the rank's device first, so that nothing (the process group's set-up included) creates a context or a
    # queue on another rank's GPU
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":  # RCCL on ROCm
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device(f"cuda:{local}")

    from envs.vss import VSS, default_cfg
    from envs import wrappers as Wr
    from vss_amd import _native as N

    n = args.fields
    cfg = default_cfg(n)
    cfg["env"]["seed"] = 1 + rank  # per-rank stream (seed + rank)
    env = VSS(cfg, str(dev), str(dev), 0, True, False, False)
    mode = {"full": N.MODE_FULL, "sa": N.MODE_SA, "cma": N.MODE_CMA, "dma": N.MODE_DMA}[args.mode]

    # inputs resident in HBM before the timed region: a pool of random action batches
    rows, width = {"full": (n, 12), "sa": (n, 2), "cma": (n, 6), "dma": (3 * n, 2)}[args.mode]
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [torch.rand((rows, width), device=dev, generator=gen) * 2 - 1 for _ in range(16)]
    if mode == N.MODE_FULL:
        io = dict(obs=env.obs_buf, terminal_obs=env.terminal_obs_buf, rew=env.rew_buf, reward_sum=None,
                  time_outs=env.timeout_buf, progress_f=env.progress_f_buf)
    else:
        W = {"sa": Wr.SingleAgent, "cma": Wr.CMA, "dma": Wr.DMA}[args.mode](env)
        io = dict(ou_buf=W.action_buf, obs=W._obs, terminal_obs=W._terminal_obs, rew=W._rews,
                  reward_sum=W._reward, dones_rep=W._dones, time_outs=W._time_outs, progress_f=W._progress)

    # pre-built ctypes arguments: the timed loop is launch-only (no per-step Python allocation)
    lib = N.load()
    stream = N.stream_of(dev)
    prm, st = env._c_params(), env._c_state()
    cios = [N.VssStepIO(a.data_ptr(), N.ptr(io.get("ou_buf")), N.ptr(io["obs"]), N.ptr(io["terminal_obs"]),
                        N.ptr(io["rew"]), N.ptr(io.get("reward_sum")), N.ptr(io.get("dones_rep")),
                        N.ptr(io["time_outs"]), N.ptr(io["progress_f"])) for a in pool]
    byref = N.ctypes.byref

    def launch(k):
        rc = lib.vss_step(stream, n, mode, byref(prm), byref(st), byref(cios[k % len(cios)]))
        if rc:
            N.check(rc, "vss_step")

    for k in range(args.warmup):
        launch(k)
    torch.cuda.synchronize()

    graph = None
    if args.graph:
        # capture one launch per pool entry into a HIP graph (torch's current stream is the
        # capture stream, so the ctypes launch is captured); replay covers the K timed steps
        g_stream = torch.cuda.Stream(device=dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=g_stream):
            cap_stream = N.stream_of(dev)
            for k in range(len(cios)):
                rc = lib.vss_step(cap_stream, n, mode, byref(prm), byref(st), byref(cios[k]))
                if rc:
                    N.check(rc, "vss_step (capture)")
        graph.replay()
        torch.cuda.synchronize()

    # ---- timed region: the K launches only (no per-launch host work besides the launch) ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events over the timed region, on the launch stream (torch's current stream, which the
    # ctypes launches use): average launch duration = region / K, back to back
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    r0.record()
    if graph is not None:
        for _ in range(args.steps // len(cios)):
            graph.replay()
        for k in range(args.steps % len(cios)):  # remainder launched eagerly, same stream
            launch(k)
    else:
        for k in range(args.steps):
            launch(k)
    r1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    region_ms = r0.elapsed_time(r1) / args.steps

    # ---- diagnostic: per-launch HIP events (a separate pass of the same launches; each event
    # pair adds its own overhead, so this reads ~2-3 % above the region average) ----
    n_ev = min(args.steps, 100)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_ev)]
    for k in range(n_ev):
        ev[k][0].record()
        launch(k)
        ev[k][1].record()
    torch.cuda.synchronize()
    per_launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    elapsed, kern_ms, per_launch_ms = reduce_max([elapsed, region_ms, per_launch_ms],
                                                 dev if args.dist_backend == "nccl" else "cpu")

    # ---- the PPO train loop on every rank (its gradient all-reduce is the one real exchange
    # step of the path); after the env-step timing, before the rank-0-only legs ----
    ppo = ppo_dma = None
    ppo_updates = args.ppo_updates if args.ppo_updates is not None else ppo_updates_to_1e8(n, world)
    if args.share_gpu:
        os.environ["VSS_LOCAL_DEVICE"] = "0"
    if ppo_updates > 0:
        if world > 1:
            dist.barrier()
        ppo = ppo_wallclock(n, ppo_updates, dev, world)
        gc.collect()
        torch.cuda.empty_cache()
        if rank == 0:
            ppo["update_gemm_roofline"] = update_gemm_roofline(dev)
    if args.ppo_dma_updates > 0:
        if world > 1:
            dist.barrier()
        ppo_dma = ppo_dma_leg(n, args.ppo_dma_updates, dev, world)
        gc.collect()
        torch.cuda.empty_cache()

    if rank == 0:
        agents = 3 if args.mode == "dma" else 1
        value = n * world * args.steps / elapsed
        algo = BYTES[args.mode] * n
        achieved = algo / (kern_ms * 1e-3)
        traffic, traffic_source = None, None
        # HBM bytes per launch from the committed rocprofv3 PMC passes of the same command
        # (tools/pmc_summary.py); null unless that profile matches this mode and size AND was
        # taken of the current kernel source (so a changed kernel cannot report stale traffic)
        tfile = os.path.join(REPO, "profiles", "pmc_traffic.json" if args.mode == "full" else f"pmc_traffic_{args.mode}.json")
        if os.path.exists(tfile):
            try:
                tj = json.load(open(tfile))
                if tj.get("fields") == n and tj.get("mode") == args.mode and tj.get("source_sha") == step_source_sha():
                    traffic = tj.get("hbm_bytes_per_launch")
                    traffic_source = (f"{os.path.relpath(tfile, REPO)} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes, "
                                      f"tag {tj.get('tag')}, vss_step.hip sha {tj.get('source_sha')})")
                else:
                    traffic_source = f"{os.path.relpath(tfile, REPO)} does not match this kernel source / config: not used"
            except (OSError, ValueError):
                traffic = None
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (uniform random actions in [-1,1], resident in HBM)",
            "config": {"workload": f"vss_step {args.mode.upper()} contract: {n} fields/GPU, one launch per "
                                   f"control step, random actions (BASELINE configs[1]/[2] shape)",
                       "fields_per_gpu": n, "mode": args.mode, "agent_rows_per_field": agents,
                       "launch": "hipGraph replay (16 captured steps)" if args.graph else "eager ctypes launches",
                       "parallelism": f"fields sharded over {world} GPU(s), no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_source": traffic_source,
                         "algorithmic_bytes_per_launch": algo, "kernel_ms": kern_ms,
                         "kernel_ms_per_launch_events": per_launch_ms},
        }
        if args.l3_check_fields > 0 and mode == N.MODE_FULL:
            out["past_l3"] = past_l3_leg(args.l3_check_fields, args.steps, dev)
        if args.rollout_k > 0 and mode == N.MODE_FULL:
            out["rollout"] = rollout_leg(env, args.rollout_k, args.steps, gen, dev)
        if mode == N.MODE_FULL:
            out["sa_step"] = sa_leg(env, args.steps, gen, dev)
        if ppo is not None:
            out["ppo"] = ppo
        if ppo_dma is not None:
            out["ppo_dma"] = ppo_dma
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
