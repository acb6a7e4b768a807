"""Config 4 workload alone (1024 ragged images, (H, W) ~ U{14..1024}^2, seed 7),
encode_batch n times: a short target for rocprofv3 kernel traces / PMC passes.
    python tools/cfg4_run.py [n] [key=value ...]   (library options)"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from importlib import import_module
import _pkgload

pkg = _pkgload.load()
ops = import_module("dct_autoencoder_amd._ops")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    ops.set_option(k, int(v))
dev = torch.device("cuda", 0)
fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
pn = pkg.PatchNorm(32, 32, 14, 3).to(dev)
pn.frozen = True
pn.eval()
lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(dev).eval()
hw = np.random.default_rng(7).integers(14, 1025, size=(1024, 2))
imgs = [ops.synth_images(1, int(h), int(w), seed=7, first_index=i, device=dev)[0] for i, (h, w) in enumerate(hw)]
for _ in range(n):
    fe.encode_batch(imgs, pn, lfq)
torch.cuda.synchronize(dev)
print("done", n)
