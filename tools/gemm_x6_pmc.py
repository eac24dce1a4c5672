#!/usr/bin/env python3
"""Profiling-only: one bf16x6 GEMM shape (GEMM_DIR=fwd|bwd|wgrad, K, N; ROWS = 2,097,152) launched REPS
times, for rocprofv3 --pmc / --kernel-trace runs of csrc/vss_gemm_x6.hip; the summary of the passes is
tools/gemm_x6_pmc.py --summary <dir>..."""
import collections
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))


def summary(dirs):
    m = collections.defaultdict(list)
    for d in dirs:
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            if "gemm_x6_kernel" in r["Kernel_Name"]:
                m[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in m.items()}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        m["kernel_cycles_per_xcd"] = m["GRBM_GUI_ACTIVE"] / 8
        m["mfma_utilization"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["kernel_cycles_per_xcd"] * 1024)
    if "SQ_WAVE_CYCLES" in m:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if c in m:
                m[c + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
    print(json.dumps(m, indent=1))


if len(sys.argv) > 2 and sys.argv[1] == "--summary":
    summary(sys.argv[2:])
    sys.exit(0)

import torch  # noqa: E402

from vss_amd.update import linear_tanh_backward_x6, linear_tanh_x6, weight_grad_x6  # noqa: E402

rows = int(os.environ.get("ROWS", 2097152))
k, n = int(os.environ.get("K", 512)), int(os.environ.get("N", 512))
reps = int(os.environ.get("REPS", 10))
g = torch.Generator(device="cuda").manual_seed(0)
mode = os.environ.get("GEMM_DIR", "fwd")
if mode == "fwd":
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.zeros(n, device="cuda")
    fn = lambda: linear_tanh_x6(x, w, b)  # noqa: E731
elif mode == "bwd":
    gn = torch.randn(rows, k, device="cuda", generator=g)
    wn = torch.randn(k, n, device="cuda", generator=g) / k ** 0.5
    y = torch.tanh(torch.randn(rows, n, device="cuda", generator=g))
    fn = lambda: linear_tanh_backward_x6(gn, wn, y)  # noqa: E731
elif mode == "loss":  # the actor's last hidden layer with the output layer and loss (EPI_LOSS_A), k_out 2
    from vss_amd.update import linear_tanh_loss_x6, weight_planes  # noqa: E402
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.zeros(n, device="cuda")
    wo, bo = torch.randn(2, n, device="cuda", generator=g) / 16, torch.zeros(2, device="cuda")
    pl = weight_planes([(w, False)])[0]
    act = torch.randn(rows, 2, device="cuda", generator=g) * 0.3
    logp, adv = torch.randn(rows, device="cuda", generator=g) - 1, torch.randn(rows, device="cuda", generator=g)
    ls = torch.zeros(1, 2, device="cuda")
    fn = lambda: linear_tanh_loss_x6(x, w, b, wo, bo, rows, True, planes=pl, act=act, logp=logp, adv=adv,  # noqa: E731
                                     logstd=ls)
else:
    gz = torch.randn(rows, n, device="cuda", generator=g)
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    fn = lambda: weight_grad_x6(gz, x)  # noqa: E731
if os.environ.get("LIB"):  # a tools/_build variant of vss_gemm_x6.hip (new API), forward only
    import ctypes
    L = ctypes.CDLL(os.environ["LIB"])
    L.vss_linear_tanh_bf16x6.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 5
    y = torch.empty(rows, n, device="cuda")
    ws = torch.empty(3 * n * k, device="cuda", dtype=torch.int16)
    st = torch.cuda.current_stream().cuda_stream
    fn = lambda: L.vss_linear_tanh_bf16x6(st, rows, k, n, x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(),  # noqa: E731
                                          ws.data_ptr())
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("done", mode, rows, k, n, reps)
