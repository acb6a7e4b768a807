"""Times VectorQuantize.forward (eval) at the model's widths on the GPU:
feature_dim D, 8 heads, 4096 codes, codebook_dim 16 (configuration_dct_autoencoder.py:13-15,
modeling_dct_autoencoder.py:77).  Prints per-kernel times (dctae timing) and the rate."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkgload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=int, default=32 * 3072)
ap.add_argument("--dim", type=int, default=768)
ap.add_argument("--heads", type=int, default=8)
ap.add_argument("--codes", type=int, default=4096)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
pkg = _pkgload.load()
from importlib import import_module  # noqa: E402
lib = import_module(pkg.__name__ + "._lib")
vq = pkg.VectorQuantize(a.dim, codebook_size=a.codes, heads=a.heads, kmeans_init=True, codebook_dim=16,
                        learnable_codebook=True, affine_param=True, ema_update=False)
with torch.no_grad():
    vq._codebook.embed.normal_()
    vq._codebook.codebook_mean.zero_()
    vq._codebook.codebook_variance.fill_(1.0)
    vq._codebook.initted.fill_(1.0)
vq = vq.eval().cuda()
x = torch.randn(1, a.tokens, a.dim, device="cuda")
mask = torch.rand(1, a.tokens, device="cuda") > 0.1
for _ in range(3):
    vq(x, mask=mask)
torch.cuda.synchronize()
ctx = lib.context(torch.device("cuda"))
ctx.lib.dctae_set_timing(ctx.h, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    vq(x, mask=mask)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
ctx.lib.dctae_timing_collect(ctx.h)
import ctypes as C  # noqa: E402
kern = {}
i = 0
while True:
    name, tot, n = C.c_char_p(), C.c_double(), C.c_int64()
    if ctx.lib.dctae_timing_get(ctx.h, i, C.byref(name), C.byref(tot), C.byref(n)) != 0:
        break
    kern[name.value.decode()] = round(tot.value / max(1, n.value), 4)
    i += 1
nv = a.tokens * a.heads
flops = 2.0 * nv * a.codes * 16
print(json.dumps({"what": "vq_forward", "tokens": a.tokens, "dim": a.dim, "heads": a.heads, "codes": a.codes,
                  "ms": round(ms, 4), "Mtok_per_s": round(a.tokens / ms / 1e3, 2),
                  "assign_TFLOPs": round(flops / (kern.get("vq_assign", ms) * 1e-3) / 1e12, 2),
                  "kernels_ms": kern}))
