"""Run-to-run stress of the config-4 batch (bench.py's 1024 ragged seed-7
images): encode the same batch N times per option set and report every call
whose codes / raw tokens differ from the first call's, with the images (and
their sizes) that differ.  Usage:
    python tools/c4_stress.py N "opt=v,opt=v" "..."      ("" = defaults)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _pkgload  # noqa: E402

pkg = _pkgload.load()
from importlib import import_module  # noqa: E402

ops = import_module("dct_autoencoder_amd._ops")
DEV = "cuda"
g = np.load(os.path.join(ROOT, "tests", "golden", "patchnorm_ref.npz"))
fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
pn = pkg.PatchNorm(32, 32, 14, 3).to(DEV)
pn.median.data.copy_(torch.from_numpy(g["median"]))
pn.b.data.copy_(torch.from_numpy(g["b"]))
pn.n.data.copy_(torch.from_numpy(g["n"]))
pn.frozen = True
pn.eval()
lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(DEV).eval()
hw = np.random.default_rng(7).integers(14, 1025, size=(1024, 2))
imgs = [ops.synth_images(1, int(h), int(w), seed=7, first_index=i, device=DEV)[0] for i, (h, w) in enumerate(hw)]

n = int(sys.argv[1])
for optset in sys.argv[2:] or [""]:
    kvs = [kv.split("=") for kv in filter(None, optset.split(","))]
    for k, v in kvs:
        ops.set_option(k, int(v))
    ((d0, c0),) = fe.encode_batch(imgs, pn, lfq, return_raw=True)
    ids, kp = d0.batched_image_ids.cpu(), d0.key_pad_mask.cpu()
    bad_calls = 0
    for it in range(n):
        raw = os.environ.get("C4_ALT") != "1" or it % 2 == 0
        ((d1, c1),) = fe.encode_batch(imgs, pn, lfq, return_raw=raw)
        dc = (c1 != c0).any(-1).cpu()
        dr = (d1.patches.view(torch.int32) != d0.patches.view(torch.int32)).any(-1).cpu() if raw else dc & False
        bad = dc | dr
        if bad.any():
            bad_calls += 1
            im = sorted(set(ids[bad & ~kp].tolist()))
            print(f"[{optset}] call {it} raw={raw}: {int(dc.sum())} tokens' codes, {int(dr.sum())} raw differ; "
                  f"images {im[:12]} sizes {[tuple(map(int, hw[i])) for i in im[:12]]}", flush=True)
            if raw and dr.any():   # where: (channel, patch row, patch col) and how much
                pos, ch = d0.patch_positions.cpu(), d0.patch_channels.cpu()
                a, b = d0.patches.cpu()[dr], d1.patches.cpu()[dr]
                rel = ((a - b).abs().amax(-1) / a.abs().amax(-1).clamp_min(1e-30))
                el = (a != b)   # which of the 196 coefficients (14 x 14 within the patch)
                cols = sorted(set((torch.nonzero(el)[:, 1] % 14).tolist()))
                rows_in = sorted(set((torch.nonzero(el)[:, 1] // 14).tolist()))
                pc = sorted(set(pos[dr][:, 1].tolist()))
                pr = sorted(set(pos[dr][:, 0].tolist()))
                print(f"    channels {sorted(set(ch[dr].tolist()))} patch rows {pr[:40]} patch cols {pc} "
                      f"coef cols in patch {cols} coef rows {rows_in}; rel diff max {float(rel.max()):.3e} "
                      f"median {float(rel.median()):.3e}; elements differing per token "
                      f"{sorted(set(el.sum(-1).tolist()))[:10]}", flush=True)
    torch.cuda.synchronize()
    print(f"=== [{optset}] {bad_calls} / {n} calls differ from the first", flush=True)
    for k, _ in kvs:   # back to the defaults
        ops.set_option(k, {"rows_fused": 1, "cols_dma": 1, "gemm_dma": 1, "xcd_order": 1}.get(k, 1))
