"""Diagnostic: preprocess tokens on the Bluestein and on the GEMM DCT paths
against the oracle, per shape: max |GPU - oracle| / max|Y| for each path."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from importlib import import_module
from oracle import ref_cpu, rng
import _pkgload
pkg = _pkgload.load()
_ops = import_module("dct_autoencoder_amd._ops")

CFG = ref_cpu.FEConfig()
fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [(97, 1000), (1000, 97), (97, 97)]
for shape in shapes:
    x_np = rng.synth_images(37, [shape])[0]
    x = torch.from_numpy(x_np)
    y = ref_cpu.transform_image_in(x)
    ph, pw = ref_cpu.crop_dims(y.shape[1], y.shape[2], 14)
    toks, pos, ch, _ = ref_cpu.patch_scores(y[:, :ph, :pw], CFG)
    omap = {(int(c), int(p[0]), int(p[1])): i for i, (p, c) in enumerate(zip(pos.tolist(), ch.tolist()))}
    ymax = float(toks.abs().max())
    res = []
    for bs in (1, 0):
        _ops.set_option("bluestein", bs)
        out = fe.preprocess(x.cuda())
        gp, gpos, gch = out["patches"].cpu(), out["positions"].cpu(), out["channels"].cpu()
        idx = torch.tensor([omap[(int(c), int(p[0]), int(p[1]))] for p, c in zip(gpos.tolist(), gch.tolist())])
        err = (gp - toks[idx]).abs()
        worst = int(err.max(1).values.argmax())
        res.append((float(err.max()) / ymax, tuple(gpos[worst].tolist()), int(gch[worst])))
    _ops.set_option("bluestein", 0)
    print(shape, "bluestein", res[0], "gemm", res[1], flush=True)
