"""The bench's LFQ-projection leg alone (conf/patch14-l.json LFQ, 16 x 2^13
over 196-element tokens; 1024 x 512^2 through BatchEncoder / BatchDecoder) for
an A/B of library builds (DCTAE_LIBRARY) or options (--opt k=v): ms per call
of the encode and the decode over --steps back-to-back calls, per-kernel
device split.  One JSON line."""
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--opt", action="append", default=[])
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
    for kv in args.opt:
        k, v = kv.split("=")
        ops.set_option(k, int(float(v)), dev)
    torch.manual_seed(0)
    lfq_p = pkg.LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16).to(dev).eval()
    x3 = ops.synth_images(1024, 512, 512, seed=1234, device=dev)
    encp = fe_mod.BatchEncoder(fe, 1024, 512, 512, pn, lfq_p, device=dev)
    res = {}
    encp(x3)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        encp(x3)
    torch.cuda.synchronize(dev)
    res["enc_ms"] = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
    res["enc_kernels"] = {k: v["total_ms"] for k, v in kernel_times(lib.context(dev), lambda: encp(x3), 3).items()}
    packed = encp(x3)
    decp = fe_mod.BatchDecoder(encp, pn, lfq_p)
    decp(packed)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        decp(packed)
    torch.cuda.synchronize(dev)
    res["dec_ms"] = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
    res["dec_kernels"] = {k: v["total_ms"] for k, v in kernel_times(lib.context(dev), lambda: decp(packed), 3).items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
