"""Throughput of the DCT GEMM kernels on uniform shapes: dctae_dct2 (two GEMMs
per image, rows then columns, full DCT matrices) on (B, 3, H, W) images,
timed with HIP events; TFLOP/s counted as fp32 GEMM flops (2 M N K).
    python tools/gemm_bench.py [B H W]"""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from importlib import import_module
import _pkgload

_pkgload.load()
ops = import_module("dct_autoencoder_amd._ops")
B, H, W = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (8, 1024, 1024)
x = torch.randn(B, 3, H, W, device="cuda")
flop = 2.0 * B * 3 * (H * W * W + H * H * W)
for x3 in (1, 0):
    ops.set_option("gemm_x3", x3)
    for _ in range(3):
        ops.dct2(x, inverse=False, color=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        ops.dct2(x, inverse=False, color=False)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"gemm_x3={x3} B={B} {H}x{W}: {ms:.3f} ms  {flop / ms / 1e9:.1f} TFLOP/s (fp32-equivalent)")
ops.set_option("gemm_x3", 1)
