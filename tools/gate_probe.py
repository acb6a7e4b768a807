"""VERDICT r5 item 2's gate: can the 512^2 encode's row and column phases hide
each other's latency when they run co-resident with T held in cache?

Needs the profiling build (DCTAE_LIBRARY=_ab/libprof.so, `make PROFILING=1`):
option t_alias=K makes images share K T' slots (T' stays in L2 / MALL, outputs
WRONG), option gate=M launches part of the band path (dctae_api.hip
dctae_ctx::gate).  For every (K, M) the 1024 x 512^2 BatchEncoder call is timed
over --steps back-to-back calls with HIP events on its stream (the side stream
joins it inside the call).  One JSON line per case, then a summary line.
Runs on the GPU box; reads nothing outside the repo."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--alias", default="0,8,64")
    ap.add_argument("--gates", default="0,1,2,5,6,3,4")
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
    x = ops.synth_images(1024, 512, 512, seed=1234, device=dev)
    enc = fe_mod.BatchEncoder(fe, 1024, 512, 512, pn, lfq, device=dev)
    res = {}
    for a in [int(v) for v in args.alias.split(",")]:
        for g in [int(v) for v in args.gates.split(",")]:
            ops.set_option("t_alias", a, dev)
            ops.set_option("gate", g, dev)
            for _ in range(3):
                enc(x)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                enc(x)
            e1.record()
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / args.steps
            res[f"alias{a}_gate{g}"] = round(ms, 4)
            print(json.dumps({"t_alias": a, "gate": g, "ms": round(ms, 4)}), flush=True)
    ops.set_option("gate", 0, dev)
    ops.set_option("t_alias", 0, dev)
    print(json.dumps({"summary": res}))


if __name__ == "__main__":
    main()
