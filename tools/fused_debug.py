"""Fused-kernel diagnostics: encode n images of size^2 with the given library
options, print the launch's XCD queue / per-image counters and (fused_debug=2)
the per-XCD tick profile: wait / row / column ticks per item."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402
from oracle import rng  # noqa: E402

pkg = _pkgload.load()
from importlib import import_module  # noqa: E402
ops = import_module("dct_autoencoder_amd._ops")
lib = import_module("dct_autoencoder_amd._lib")
fe_mod = import_module("dct_autoencoder_amd.feature_extraction")

dev = torch.device("cuda", 0)
tabs = np.load(os.path.join(ROOT, "tests", "golden", "patchnorm_ref.npz"))
pn = pkg.PatchNorm(32, 32, 14, 3).to(dev)
pn.median.data.copy_(torch.from_numpy(tabs["median"]))
pn.b.data.copy_(torch.from_numpy(tabs["b"]))
pn.frozen = True
pn.eval()
lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(dev).eval()
fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
size = int(sys.argv[2]) if len(sys.argv) > 2 else 512
for kv in sys.argv[3:]:
    k, v = kv.split("=")
    ops.set_option(k, int(float(v)), dev)
if n <= 64:
    x = torch.from_numpy(np.stack(rng.synth_images(5, [(size, size)] * n))).to(dev)
else:
    x = ops.synth_images(n, size, size, seed=5, first_index=0, device=dev)
enc = fe_mod.BatchEncoder(fe, n, size, size, pn, lfq, device=dev)
for _ in range(2):
    enc(x)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    enc(x)
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t0) / 5 * 1e3:.3f} ms per encode of {n} x {size}^2")
ctx = lib.context(dev)
m = ctx.lib.dctae_fused_debug_counters(ctx.h, None, 0, lib.stream_ptr(dev))
buf = (C.c_int32 * max(m, 1))()
ctx.lib.dctae_fused_debug_counters(ctx.h, buf, m, lib.stream_ptr(dev))
v = list(buf)[:m]
print("queues", v[:8])
print("rows_done min/max", min(v[24:24 + n]), max(v[24:24 + n]), "cols_done min/max", min(v[24 + n:24 + 2 * n]),
      max(v[24 + n:24 + 2 * n]))
po = (24 + 2 * n + 1) & ~1
prof = np.array(v[po:po + 128], dtype=np.int32).view(np.uint64).reshape(8, 8)
print("prof raw", prof[:, :7].tolist())
if prof.sum():
    for q in range(8):
        w, r, c, nr_, nc_, life, wgs = [int(t) for t in prof[q][:7]]
        print(f"xcd {q}: wgs {wgs} life/wg {life / max(wgs, 1):.0f} | wait {w / max(wgs, 1):.0f}/wg "
              f"| row item {r / max(nr_, 1):.0f} x{nr_} | col item {c / max(nc_, 1):.0f} x{nc_}  (s_memtime ticks)")
try:
    ops.check_device_errors(dev)
    print("no device error")
except Exception as e:  # noqa: BLE001
    print("device error:", e)
