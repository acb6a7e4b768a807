"""Diagnostic: run the persistent 512^2 encode (k_enc512) against the two-kernel
path several times on the same inputs and report which packed rows (= images)
differ and how.  python tools/enc512_diag.py [B] [reps] [opt=v ...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
from importlib import import_module  # noqa: E402
ops = import_module("dct_autoencoder_amd._ops")
fe_mod = import_module("dct_autoencoder_amd.feature_extraction")

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
opts = [a.split("=") for a in sys.argv[3:]]
dev = torch.device("cuda", 0)
tabs = np.load(os.path.join(ROOT, "tests", "golden", "patchnorm_ref.npz"))
fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
pn = pkg.PatchNorm(32, 32, 14, 3).to(dev)
pn.median.data.copy_(torch.from_numpy(tabs["median"]))
pn.b.data.copy_(torch.from_numpy(tabs["b"]))
pn.frozen = True
pn.eval()
lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(dev).eval()
x = ops.synth_images(B, 512, 512, seed=13, first_index=0, device=dev)
enc = fe_mod.BatchEncoder(fe, B, 512, 512, pn, lfq, device=dev)
ops.set_option("enc512", 0, dev)
ref = enc(x)["codes"].clone()
ops.set_option("enc512", 1, dev)
for k, v in opts:
    ops.set_option(k, int(v), dev)
for r in range(reps):
    out = enc(x)["codes"].clone()
    torch.cuda.synchronize()
    err = None
    try:
        ops.check_device_errors(dev)
    except Exception as e:  # noqa: BLE001
        err = str(e)
    bad = (out != ref).any(-1)            # (rows, S): tokens with any code different
    rows = torch.nonzero(bad.any(-1)).flatten().tolist()
    print(f"rep {r}: err={err} bad rows {len(rows)} tokens {int(bad.sum())} "
          f"first rows {rows[:12]} per-row counts {[int(bad[i].sum()) for i in rows[:12]]}", flush=True)
    res = enc.out
    for i in rows[:4]:
        toks = torch.nonzero(bad[i]).flatten()
        ch = res["channels"][i, toks]
        pw = res["positions"][i, toks, 1]
        ph = res["positions"][i, toks, 0]
        items = sorted(set(zip(ch.tolist(), pw.tolist())))
        hs = sorted(set(ph.tolist()))
        print(f"   row {i}: {len(items)} (channel, strip) items bad, e.g. {items[:10]}; tile rows {hs[:12]}...",
              flush=True)
        # do the bad codes of this row equal another image's reference codes at those tokens?
        same = (out[i][None, toks] == ref[:, toks]).all(-1).float().mean(-1)
        best = torch.topk(same, 3)
        print(f"   row {i}: closest reference rows {best.indices.tolist()} match fraction {best.values.tolist()}",
              flush=True)
