#!/usr/bin/env python3
"""Profiling-only prototype measurement (needs tools/x6_qdma_prototype.patch applied to csrc/vss_gemm_x6.hip): the x6 forward y = tanh(x W^T + b)
with its activation operand split in the K loop from fp32 rows (today's ST_ROW staging) against the same
GEMM reading the activations' tile-ordered bf16 plane images by global_load_lds (ST_QDMA,
vss_linear_tanh_qdma_bf16x6; the images made beforehand by vss_act_image_bf16x6, whose time is printed
apart -- in the planned design the producing layer's epilogue writes them).  Both compute the same six
products in the same order: y must match bit for bit.  HIP events over REPS launches, alternating."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd"))
import torch  # noqa: E402

from vss_amd import _native as N  # noqa: E402
from vss_amd.update import linear_tanh_x6, weight_planes  # noqa: E402

reps = int(os.environ.get("REPS", 10))
rows = int(os.environ.get("ROWS", 2097152))
lib = N.load()
P, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
lib.vss_act_image_bf16x6.argtypes = [P, i64, i32, P, P]
lib.vss_linear_tanh_qdma_bf16x6.argtypes = [P, i64, i32, i32, P, P, P, P]
g = torch.Generator(device="cuda").manual_seed(0)
st = N.stream_of(torch.device("cuda"))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for k, n in ((512, 512), (256, 512), (512, 256)):
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g))
    w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
    b = torch.randn(n, device="cuda", generator=g) * 0.1
    planes = weight_planes([(w, False)])[0]
    img = torch.empty(3 * rows * k, dtype=torch.int16, device="cuda")
    y0, y1 = torch.empty(rows, n, device="cuda"), torch.empty(rows, n, device="cuda")

    def row():
        linear_tanh_x6(x, w, b, out=y0, planes=planes)

    def image():
        N.check(lib.vss_act_image_bf16x6(st, rows, k, x.data_ptr(), img.data_ptr()), "vss_act_image_bf16x6")

    def qdma():
        N.check(lib.vss_linear_tanh_qdma_bf16x6(st, rows, k, n, img.data_ptr(), b.data_ptr(), y1.data_ptr(),
                                                planes.data_ptr()), "vss_linear_tanh_qdma_bf16x6")

    image()
    ts = {"row": [], "qdma": [], "image": []}
    for _ in range(3):
        ts["row"].append(timed(row))
        ts["qdma"].append(timed(qdma))
        ts["image"].append(timed(image))
    same = torch.equal(y0, y1)
    fl = 2.0 * rows * k * n
    tr, tq, ti = min(ts["row"]), min(ts["qdma"]), min(ts["image"])
    print(f"forward {k}->{n} rows {rows}: ST_ROW {tr:.1f} us ({fl / tr / 1e6:.1f} TF)  ST_QDMA {tq:.1f} us "
          f"({fl / tq / 1e6:.1f} TF, {tr / tq:.3f}x)  image {ti:.1f} us  y bit-equal {same}", flush=True)
    del x, w, img, y0, y1
    torch.cuda.empty_cache()
