#!/usr/bin/env python3
"""Profiling-only: time ablated builds of the step kernel (VSS_PROF_* knobs) at 65,536 fields.

Builds each variant of csrc/vss_step.hip into tools/_build/, loads it with ctypes beside the
product library and times `vss_step` (FULL) with HIP events.  The numbers say which phase the
kernel's time goes to; the ablated outputs are wrong by construction and never used."""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import _native as N  # noqa: E402

VARIANTS = {"full": [], "no_physics": ["-DVSS_PROF_SKIP_PHYSICS"], "no_obs": ["-DVSS_PROF_SKIP_OBS"],
            "no_physics_no_obs": ["-DVSS_PROF_SKIP_PHYSICS", "-DVSS_PROF_SKIP_OBS"]}
# extra variants: ABLATE_EXTRA="name=flag flag;name2=flag"
for item in [v for v in os.environ.get("ABLATE_EXTRA", "").split(";") if v]:
    k, _, flags = item.partition("=")
    VARIANTS[k] = flags.split()
VARIANTS = {k: v for k, v in VARIANTS.items()
            if os.path.exists(os.path.join(REPO, "tools", "_build", f"libvss_{k}.so")) or len(sys.argv) > 1}


def build(name, flags):
    out = os.path.join(REPO, "tools", "_build", f"libvss_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    src = os.path.join(REPO, "rsoccer-isaac-cleanrl_amd", "csrc", "vss_step.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                    "-ffp-contract=off", *flags, "-o", out, src], check=True)
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        for k, v in VARIANTS.items():
            build(k, v)
        return
    from envs.vss import VSS, default_cfg
    n = int(os.environ.get("FIELDS", 65536))
    cfg = default_cfg(n)
    cfg["env"]["seed"] = 3
    env = VSS(cfg, "cuda:0", "cuda:0", 0, True, False, False)
    mode_name = os.environ.get("ABLATE_MODE", "full")
    mode = {"full": N.MODE_FULL, "sa": N.MODE_SA, "cma": N.MODE_CMA, "dma": N.MODE_DMA}[mode_name]
    # episodes desynchronised (progress uniform over the episode length): with every field at
    # progress 0 the timeouts arrive in one burst every max_episode_length steps, and whether a
    # burst of resets lands inside a variant's timed window decides its rollout figure
    env.progress_buf.random_(0, int(cfg["env"]["maxEpisodeLength"]))
    prm, st = env._c_params(), env._c_state()
    if mode == N.MODE_FULL:
        acts = torch.rand((n, 12), device="cuda:0") * 2 - 1
        io = N.VssStepIO(acts.data_ptr(), None, env.obs_buf.data_ptr(), env.terminal_obs_buf.data_ptr(),
                         env.rew_buf.data_ptr(), None, None, env.timeout_buf.data_ptr(), env.progress_f_buf.data_ptr())
    else:
        from envs import wrappers as Wr
        W = {"sa": Wr.SingleAgent, "cma": Wr.CMA, "dma": Wr.DMA}[mode_name](env)
        rows, width = {"sa": (n, 2), "cma": (n, 6), "dma": (3 * n, 2)}[mode_name]
        acts = torch.rand((rows, width), device="cuda:0") * 2 - 1
        io = N.VssStepIO(acts.data_ptr(), W.action_buf.data_ptr(), W._obs.data_ptr(), W._terminal_obs.data_ptr(),
                         W._rews.data_ptr(), W._reward.data_ptr(), N.ptr(getattr(W, "_dones", None)),
                         W._time_outs.data_ptr(), W._progress.data_ptr())
    stream = N.stream_of(env.device)
    import glob
    names = sorted(os.path.basename(p)[7:-3] for p in glob.glob(os.path.join(REPO, "tools", "_build", "libvss_*.so")))
    if os.environ.get("ABLATE_ONLY"):  # one variant per process (rocprofv3 --pmc passes)
        names = [nm for nm in names if nm == os.environ["ABLATE_ONLY"]]
    libs = []
    for name in names:
        L = ctypes.CDLL(os.path.join(REPO, "tools", "_build", f"libvss_{name}.so"))
        L.vss_step.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 3
        libs.append((name, L))
    K, reps = 100, int(os.environ.get("ABLATE_REPS", 3))
    times = {name: [] for name, _ in libs}
    RK = int(os.environ.get("ABLATE_ROLLOUT_K", 0))  # also time vss_rollout with RK steps per launch
    if RK:
        racts = torch.rand((RK, n, 2, 3, 2), device="cuda:0") * 2 - 1
        rout = env.rollout(racts)
        rio = N.VssRolloutIO(racts.data_ptr(), rout["obs"].data_ptr(), rout["terminal_observation"].data_ptr(),
                             rout["rew"].data_ptr(), rout["dones"].data_ptr(), rout["time_outs"].data_ptr(),
                             rout["progress_buffer"].data_ptr())
        rtimes = {name: [] for name, _ in libs}
    for _ in range(reps):  # interleaved repetitions: run-to-run drift hits every variant alike
        for name, L in libs:
            for _ in range(20):
                L.vss_step(stream, n, mode, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(io))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(K):
                L.vss_step(stream, n, mode, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(io))
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / K * 1e3)
            if RK:
                L.vss_rollout.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 3
                for _ in range(2):
                    L.vss_rollout(stream, n, RK, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(rio))
                torch.cuda.synchronize()
                e0.record()
                for _ in range(10):
                    L.vss_rollout(stream, n, RK, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(rio))
                e1.record()
                torch.cuda.synchronize()
                rtimes[name].append(e0.elapsed_time(e1) / (10 * RK) * 1e3)
    for name, L in libs:
        t = sorted(times[name])
        extra = ""
        if RK:
            r = sorted(rtimes[name])
            extra = f"   rollout K={RK}: {r[len(r) // 2]:.1f} us/step (min {r[0]:.1f})"
        print(f"{name:20s} {t[len(t) // 2]:8.1f} us/step (median of {reps}; min {t[0]:.1f}){extra}")
        if hasattr(L, "vss_prof_read"):
            buf = (ctypes.c_ulonglong * 8)()
            L.vss_prof_read(buf)  # includes the warm-up launches too
            waves = (n + 63) // 64 * (K + 20) * reps
            pn = ["drive", "integrate", "robot-robot", "ball-robot", "walls"]
            tot = sum(buf[:5])
            print("   stamps (s_memtime ticks per wave-step): " + ", ".join(
                f"{nm} {buf[i] / waves:.0f} ({100 * buf[i] / max(tot, 1):.0f}%)" for i, nm in enumerate(pn)))

if __name__ == "__main__":
    main()
