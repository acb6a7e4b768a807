"""Golden vectors for the reference LFQ's index rule at any ``codebook_scale``
(reference dct_autoencoder/lfq.py:174-187: ``quantized = where(x > 0, +s, -s)``,
then ``indices = sum((quantized > 0) * mask)``), produced by running the
REFERENCE's own LFQ class in the build container (refload.py).

    python tests/golden/gen_lfq_scale_golden.py   ->  tests/golden/lfq_scale_ref.npz

Cases: scales {1.0, 0.5, 0.0, -1.0, -0.25}; without projections
LFQ(dim=196, 2**14, 14 codebooks) and with projections LFQ(dim=196, 2**13, 16
codebooks: project_in 196 -> 208, project_out 208 -> 196, seeded weights stored
here).  Inputs hold exact +0 / -0, NaN rows and NaN elements.  Stored: inputs,
weights, indices, quantized outputs and indices_to_codes of every case.  Data
only; no reference source is stored.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import refload  # noqa: E402

SCALES = [1.0, 0.5, 0.0, -1.0, -0.25]


def inputs(n=96, dim=196, seed=11):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(1, n, dim, generator=g)
    x[0, 0] = 0.0                          # an all +0 token
    x[0, 1] = -0.0                         # an all -0 token
    x[0, 2, ::3] = float("nan")            # scattered NaN elements
    x[0, 3] = float("nan")                 # a NaN token
    x[0, 4:12, ::5] = 0.0                  # exact zeros inside ordinary tokens
    x[0, 12:20, 1::7] = -0.0
    return x


def main():
    ref = refload.load()
    LFQ = ref.lfq.LFQ
    out = {}
    x = inputs()
    out["x"] = x.numpy()
    mask = torch.ones(x.shape[:2], dtype=torch.bool)
    for proj in (False, True):
        tag = "p" if proj else "n"
        for si, s in enumerate(SCALES):
            if proj:
                torch.manual_seed(21)
                m = LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16, codebook_scale=s).eval()
                if si == 0:
                    out["w_in"] = m.project_in.weight.detach().numpy()
                    out["b_in"] = m.project_in.bias.detach().numpy()
                    out["w_out"] = m.project_out.weight.detach().numpy()
                    out["b_out"] = m.project_out.bias.detach().numpy()
                else:   # one set of projection weights for every scale
                    with torch.no_grad():
                        m.project_in.weight.copy_(torch.from_numpy(out["w_in"]))
                        m.project_in.bias.copy_(torch.from_numpy(out["b_in"]))
                        m.project_out.weight.copy_(torch.from_numpy(out["w_out"]))
                        m.project_out.bias.copy_(torch.from_numpy(out["b_out"]))
            else:
                m = LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14, codebook_scale=s).eval()
            with torch.no_grad():
                q, idx, _, _ = m(x, mask=mask)
                codes = m.indices_to_codes(idx)
                if proj:
                    h = m.project_in(x)   # the projected features (rounding-band checks)
                    out[f"{tag}{si}_h"] = h.numpy()
            out[f"{tag}{si}_idx"] = idx.numpy().astype(np.int64)
            out[f"{tag}{si}_q"] = q.numpy()
            out[f"{tag}{si}_codes"] = codes.numpy()
    out["scales"] = np.array(SCALES, dtype=np.float64)
    path = os.path.join(HERE, "lfq_scale_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
