"""Config 2: 256 x 224^2 encode through the pre-planned
BatchEncoder, device time per step (HIP events on the encoder's stream) and
per-kernel times.  python tools/cfg2_time.py [--opt key=value ...]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _pkgload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    pkg = _pkgload.load()
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    bench = import_module("bench")
    dev = torch.device("cuda", 0)
    for kv in a.opt:
        k, v = kv.split("=")
        ops.set_option(k, int(v), dev)
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    pn = pkg.PatchNorm(32, 32, 14, 3).to(dev).eval()
    pn.frozen = True
    lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(dev).eval()
    x = ops.synth_images(256, 224, 224, seed=1234, device=dev)
    enc = fe_mod.BatchEncoder(fe, 256, 224, 224, pn, lfq, device=dev)
    for _ in range(5):
        enc(x)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        enc(x)
    e1.record()
    torch.cuda.synchronize(dev)
    lib = import_module("dct_autoencoder_amd._lib")
    k = bench.kernel_times(lib.context(dev), lambda: enc(x), 5)
    print(json.dumps({"ms_per_step": round(e0.elapsed_time(e1) / a.steps, 4), "opts": a.opt,
                      "kernels": {n: v.get("avg_ms", v.get("total_ms")) for n, v in k.items()}}))


if __name__ == "__main__":
    main()
