"""Golden vectors for the VectorQuantize inference path, made by
running the reference's own vector_quantize.py (read-only, /root/reference)
in the build container — BUILD-CONTAINER ONLY, never run on the GPU box.

The module is built exactly as the model builds it
(modeling_dct_autoencoder.py:76-77: heads, kmeans_init=True,
sample_codebook_temp=20, codebook_dim=16, learnable_codebook=True,
affine_param=True, ema_update=False, threshold_ema_dead_code=15) at a small
size, its parameters set from a seeded generator (the codebook marked as
k-means-initialised, the codebook affine statistics set as training leaves
them), then run in eval mode on two consecutive masked batches (the batch
affine statistics start at None and are EMA-updated by every forward).

    python tests/golden/gen_vq_golden.py   ->  tests/golden/vq_ref.npz
"""
import importlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import refload  # noqa: E402

DIM, HEADS, CB, CBDIM = 40, 3, 96, 16


def main():
    refload.load()
    vqm = importlib.import_module("dct_autoencoder.vector_quantize")
    torch.manual_seed(0)
    vq = vqm.VectorQuantize(DIM, codebook_size=CB, heads=HEADS, kmeans_init=True, sample_codebook_temp=20.0,
                            codebook_dim=CBDIM, learnable_codebook=True, affine_param=True, ema_update=False,
                            threshold_ema_dead_code=15)
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        vq.project_in.weight.copy_(torch.randn(vq.project_in.weight.shape, generator=g) * 0.3)
        vq.project_in.bias.copy_(torch.randn(vq.project_in.bias.shape, generator=g) * 0.1)
        vq.project_out.weight.copy_(torch.randn(vq.project_out.weight.shape, generator=g) * 0.3)
        vq.project_out.bias.copy_(torch.randn(vq.project_out.bias.shape, generator=g) * 0.1)
        cb = vq._codebook
        cb.embed.copy_(torch.randn(cb.embed.shape, generator=g))
        cb.initted.copy_(torch.Tensor([True]))
        cb.codebook_mean.copy_(torch.randn(cb.codebook_mean.shape, generator=g) * 0.1)
        cb.codebook_variance.copy_(torch.rand(cb.codebook_variance.shape, generator=g) + 0.5)
    vq.eval()
    out = {"w_in": vq.project_in.weight.detach().numpy(), "b_in": vq.project_in.bias.detach().numpy(),
           "w_out": vq.project_out.weight.detach().numpy(), "b_out": vq.project_out.bias.detach().numpy(),
           "embed": vq._codebook.embed.detach().numpy(),
           "codebook_mean": vq._codebook.codebook_mean.numpy(),
           "codebook_variance": vq._codebook.codebook_variance.numpy(),
           "heads": np.int64(HEADS)}
    for step, (b, n) in enumerate([(3, 40), (2, 57)]):
        x = torch.randn(b, n, DIM, generator=g) * 1.5
        mask = torch.rand(b, n, generator=g) > 0.25
        with torch.no_grad():
            q, ind, loss = vq(x, mask=mask)
        out[f"x{step}"] = x.numpy()
        out[f"mask{step}"] = mask.numpy()
        out[f"quantize{step}"] = q.numpy()
        out[f"indices{step}"] = ind.numpy()
        out[f"batch_mean{step}"] = vq._codebook.batch_mean.numpy()
        out[f"batch_variance{step}"] = vq._codebook.batch_variance.numpy()
        out[f"loss{step}"] = loss.numpy()
    ind0 = torch.from_numpy(out["indices0"])
    out["codes_from_indices0"] = vq.get_codes_from_indices(ind0).detach().numpy()
    out["output_from_indices0"] = vq.get_output_from_indices(ind0).detach().numpy()
    np.savez_compressed(os.path.join(HERE, "vq_ref.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
