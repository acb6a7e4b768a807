#!/usr/bin/env python3
"""Per-shape throughput of dctae_model_linear (the patch14-l GEMMs, M = 4 x 3072
tokens): TFLOP/s of each epilogue / shape, HIP-event timed, 20 launches each."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkgload  # noqa: E402

_pkgload.load()
from importlib import import_module  # noqa: E402

L = import_module("dct_autoencoder_amd._lib")
dev = torch.device("cuda", 0)
ctx = L.context(dev)
M = 12288
out = {}
for name, n, k, epi in [("qkv", 3072, 1024, 1), ("out_proj", 1024, 1024, 3), ("fc1", 4096, 1024, 2),
                        ("fc2", 1024, 4096, 3), ("fc1_f32out", 4096, 1024, 0)]:
    x = torch.randn(M, k, device=dev).to(torch.bfloat16).view(torch.int16)
    w = torch.randn(n, k, device=dev).to(torch.bfloat16).view(torch.int16)
    b = torch.randn(n, device=dev)
    o = torch.zeros(M, n, device=dev) if epi in (0, 3) else torch.zeros(M, n, dtype=torch.int16, device=dev)
    st = L.stream_ptr(dev)

    def go():
        ctx.check(ctx.lib.dctae_model_linear(ctx.h, M, n, k, L.ptr(x), k, L.ptr(w), n, k, L.ptr(b), epi, L.ptr(o), n,
                                             st), "linear")
    for _ in range(3):
        go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        go()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    out[name] = {"M": M, "N": n, "K": k, "ms": round(ms, 4), "tflops": round(2 * M * n * k / ms / 1e9, 1)}
print(json.dumps(out))
