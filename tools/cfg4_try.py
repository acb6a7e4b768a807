"""Config 4 (1024 ragged images, (H, W) ~ U{14..1024}^2 seed 7, encode_batch
incl. host packing) timing for an A/B of library builds (DCTAE_LIBRARY) or
options (--opt k=v): ms per call over --steps back-to-back calls (as the
bench's config-4 leg) and the per-kernel device split.  One JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--opt", action="append", default=[])
    args = ap.parse_args()
    import _pkgload
    from bench import kernel_times
    pkg = _pkgload.load()
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    lib = import_module("dct_autoencoder_amd._lib")
    dev = torch.device("cuda", 0)
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    tabs = np.load(os.path.join(ROOT, "tests", "golden", "patchnorm_ref.npz"))
    pn = pkg.PatchNorm(32, 32, 14, 3).to(dev)
    for k in ("median", "b", "n"):
        getattr(pn, k).data.copy_(torch.from_numpy(tabs[k]))
    pn.frozen = True
    pn.eval()
    lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(dev).eval()
    for kv in args.opt:
        k, v = kv.split("=")
        ops.set_option(k, int(float(v)), dev)
    hw = np.random.default_rng(7).integers(14, 1025, size=(1024, 2))
    imgs = [ops.synth_images(1, int(h), int(w), seed=7, first_index=i, device=dev)[0] for i, (h, w) in enumerate(hw)]
    fe.encode_batch(imgs, pn, lfq)
    torch.cuda.synchronize(dev)
    fe.encode_batch(imgs, pn, lfq)   # warm-up call in flight: steady state as bench.config_legs
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        fe.encode_batch(imgs, pn, lfq)
    e1.record()
    torch.cuda.synchronize(dev)
    el = e0.elapsed_time(e1) / 1e3 / args.steps
    kern = kernel_times(lib.context(dev), lambda: fe.encode_batch(imgs, pn, lfq), 2)
    print(json.dumps({"ms": round(el * 1e3, 3), "device_ms": round(sum(v["total_ms"] for v in kern.values()), 3),
                      "kernels": {k: v["total_ms"] for k, v in kern.items()}}))


if __name__ == "__main__":
    main()
