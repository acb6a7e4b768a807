"""Config 2 (256 x 224^2 encode, pre-planned BatchEncoder) timing for an A/B of
library builds (DCTAE_LIBRARY) or options (--opt k=v): ms per call over
--steps back-to-back calls and the per-kernel device split (bench.kernel_times).
One JSON line.  Runs on the GPU box; reads nothing outside the repo."""
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
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--no-kernel-timing", action="store_true")
    args = ap.parse_args()
    import _pkgload
    from bench import kernel_times
    pkg = _pkgload.load()
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
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
    x2 = ops.synth_images(256, 224, 224, seed=1234, device=dev)
    enc2 = fe_mod.BatchEncoder(fe, 256, 224, 224, pn, lfq, device=dev)
    for _ in range(5):
        enc2(x2)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        enc2(x2)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / args.steps
    # host cost of one call: enqueue time of 20 calls on an idle GPU (no sync
    # inside); below the per-call period the GPU, not the host, sets the pace
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(20):
        enc2(x2)
    host = (time.perf_counter() - t0) / 20
    torch.cuda.synchronize(dev)
    kern = {} if args.no_kernel_timing else kernel_times(lib.context(dev), lambda: enc2(x2), 20)
    print(json.dumps({"ms": round(el * 1e3, 4), "host_enqueue_ms": round(host * 1e3, 4),
                      "kernels": {k: v["total_ms"] for k, v in kern.items()}}))


if __name__ == "__main__":
    main()
