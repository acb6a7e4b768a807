"""Calibrate bench.py's CPU baseline: time the oracle port
(oracle/ref_cpu.encode, what bench.py's cpu_baseline leg runs on the GPU box)
against the reference itself (dct_autoencoder loaded from /root/reference via
tests/golden/refload.py) on the same images, thread count and pipeline:
preprocess -> iter_batches(None) (attn_mask built) -> PatchNorm eval -> LFQ eval.

BUILD-CONTAINER ONLY (the GPU box has no /root/reference).  The two are timed
alternately, `--repeats` times each, and the medians are compared; the record
goes to profiles/cpu_calibration_r02.json, which bench.py copies into its
cpu_baseline object.

    python tools/calibrate_cpu_baseline.py [--threads 8] [--images 16] [--size 512] [--repeats 5]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--images", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_calibration_r02.json"))
    args = ap.parse_args()
    import refload
    from oracle import ref_cpu
    if not refload.available():
        sys.exit("the reference is not available here (/root/reference): calibration runs in the build container")
    ref = refload.load()
    torch.set_num_threads(args.threads)
    g = np.load(os.path.join(ROOT, "tests", "golden", "patchnorm_ref.npz"))
    tables = ref_cpu.NormTables(torch.from_numpy(g["n"]), torch.from_numpy(g["median"]), torch.from_numpy(g["b"]))
    P, MAXP, S = 14, 32, 3072
    proc = ref.fe.DCTAutoencoderFeatureExtractor(3, P, 0.0, MAXP, MAXP, S)
    pn = ref.patchnorm.PatchNorm(MAXP, MAXP, P, 3)
    pn.median.data.copy_(torch.from_numpy(g["median"]))
    pn.b.data.copy_(torch.from_numpy(g["b"]))
    pn.n.data.copy_(torch.from_numpy(g["n"]))
    pn.frozen = True
    pn.eval()
    lfq = ref.lfq.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).eval()
    gen = torch.Generator().manual_seed(0)
    imgs = [torch.rand(3, args.size, args.size, generator=gen) for _ in range(args.images)]
    cfg, lcfg = ref_cpu.FEConfig(), ref_cpu.LFQConfig()

    def run_ref():
        with torch.no_grad():
            for k in range(0, len(imgs), 8):
                items = [proc.preprocess(x) for x in imgs[k:k + 8]]
                col = {key: [it[key] for it in items] for key in items[0]}
                (batch,) = list(proc.iter_batches(iter([col]), None))
                nb = batch.shallow_copy()
                nb.patches = pn(nb)
                lfq(nb.patches, mask=~nb.key_pad_mask)

    def run_port():
        for k in range(0, len(imgs), 8):
            ref_cpu.encode(imgs[k:k + 8], cfg, tables, lcfg, batch_size=None, build_attn_mask=True)

    run_ref()
    run_port()   # warm-up
    t_ref, t_port = [], []
    for _ in range(args.repeats):
        t0 = time.perf_counter()
        run_ref()
        t_ref.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        run_port()
        t_port.append(time.perf_counter() - t0)
    mpix = len(imgs) * args.size * args.size / 1e6
    ref_v, port_v = mpix / statistics.median(t_ref), mpix / statistics.median(t_port)
    rec = {"threads": args.threads, "images": len(imgs), "size": args.size, "repeats": args.repeats,
           "reference_mpix_s": round(ref_v, 3), "port_mpix_s": round(port_v, 3),
           "port_over_reference": round(port_v / ref_v, 3),
           "reference_s": [round(t, 3) for t in t_ref], "port_s": [round(t, 3) for t in t_port],
           "pipeline": "preprocess -> iter_batches(None) with attn_mask -> PatchNorm eval -> LFQ eval, 8 images per "
                       "dataloader item, torch.rand RGB",
           "within_10pct": abs(port_v / ref_v - 1.0) <= 0.10}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
