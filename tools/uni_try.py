"""Uniform-batch encode timing (BatchEncoder of --n images of --h x --w) for
an A/B of options (--opt k=v, applied in order per --case): ms per call over
--steps back-to-back calls for each case, one JSON line.  GPU box only."""
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
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--h", type=int, default=448)
    ap.add_argument("--w", type=int, default=448)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--case", action="append", default=[], help="comma-separated k=v options")
    args = ap.parse_args()
    import _pkgload
    pkg = _pkgload.load()
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    dev = torch.device("cuda", 0)
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    tabs = np.load(os.path.join(ROOT, "tests", "golden", "patchnorm_ref.npz"))
    pn = pkg.PatchNorm(32, 32, 14, 3).to(dev)
    for k in ("median", "b", "n"):
        getattr(pn, k).data.copy_(torch.from_numpy(tabs[k]))
    pn.frozen = True
    pn.eval()
    lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(dev).eval()
    x = ops.synth_images(args.n, args.h, args.w, seed=99, device=dev)
    enc = fe_mod.BatchEncoder(fe, args.n, args.h, args.w, pn, lfq, device=dev)
    res = {"n": args.n, "h": args.h, "w": args.w}
    for case in args.case or [""]:
        for kv in filter(None, case.split(",")):
            k, v = kv.split("=")
            ops.set_option(k, int(v), dev)
        for _ in range(3):
            enc(x)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            enc(x)
        torch.cuda.synchronize(dev)
        res[case or "default"] = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
