import os, sys, torch
sys.path.insert(0, "/root/repo/rsoccer-isaac-cleanrl_amd"); sys.path.insert(0, "/root/repo/tools")
from gemm_fused_bench import timeit
from vss_amd import _native as N
lib = N.load(); st = torch.cuda.current_stream().cuda_stream
rows = 2097152
for k in (52, 56, 64):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.tanh(torch.randn(rows, k, device="cuda", generator=g)); w = torch.randn(256, k, device="cuda", generator=g) / 8
    b = torch.randn(256, device="cuda", generator=g); y = torch.empty(rows, 256, device="cuda")
    t = timeit(lambda: lib.vss_linear_tanh(st, rows, k, 256, x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr()))
    ref = torch.addmm(b, x, w.t()).tanh_()
    print(f"FWD K {k} N 256: {t:7.0f} us  {2*rows*k*256/t/1e6:5.1f} TF  {(rows*(k+256)*4)/t/1e3:5.2f} TB/s  err {float((y-ref).abs().max()):.1e}", flush=True)
