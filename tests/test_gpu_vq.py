"""GPU parity of the VectorQuantize inference path (SURVEY §8(f)1,
vector_quantize.py:675-1050) through dctae_vq_forward / dctae_vq_*_from_indices,
against the reference's golden vectors (tests/golden/vq_ref.npz) and the CPU
oracle (oracle/ref_cpu.vq_forward_eval) at larger sizes.

Tolerances:
  * indices: equal, except where the oracle's distance to the GPU's code is
    within 2e-5 * (1 + |d|) of its best distance (near-ties: the GPU sums the
    16-term dot products in another order than torch's cdist einsum);
  * quantize / project_out results: 2e-5 absolute + 2e-5 relative where the
    indices agree (fp32 GEMMs with different summation order);
  * batch statistics: 1e-6 absolute + 1e-5 relative (GPU sums in fp64);
  * codes from indices: bit-exact (a gather).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref_cpu

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _make(pkg, dim, heads, C, g=None, seed=0):
    """VectorQuantize in the model's configuration (modeling_dct_autoencoder.py:77)."""
    vq = pkg.VectorQuantize(dim, codebook_size=C, heads=heads, kmeans_init=True, sample_codebook_temp=20.0,
                            codebook_dim=16, learnable_codebook=True, affine_param=True, ema_update=False,
                            threshold_ema_dead_code=15)
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        cb = vq._codebook
        if g is not None:
            if vq.has_projections:
                vq.project_in.weight.copy_(torch.from_numpy(g["w_in"]))
                vq.project_in.bias.copy_(torch.from_numpy(g["b_in"]))
                vq.project_out.weight.copy_(torch.from_numpy(g["w_out"]))
                vq.project_out.bias.copy_(torch.from_numpy(g["b_out"]))
            cb.embed.copy_(torch.from_numpy(g["embed"]))
            cb.codebook_mean.copy_(torch.from_numpy(g["codebook_mean"]))
            cb.codebook_variance.copy_(torch.from_numpy(g["codebook_variance"]))
        else:
            if vq.has_projections:
                for lin in (vq.project_in, vq.project_out):
                    lin.weight.copy_(torch.randn(lin.weight.shape, generator=gen) / lin.weight.shape[1] ** 0.5)
                    lin.bias.copy_(torch.randn(lin.bias.shape, generator=gen) * 0.1)
            cb.embed.copy_(torch.randn(cb.embed.shape, generator=gen))
            cb.codebook_mean.copy_(torch.randn(cb.codebook_mean.shape, generator=gen) * 0.1)
            cb.codebook_variance.copy_(torch.rand(cb.codebook_variance.shape, generator=gen) + 0.5)
        cb.initted.fill_(1.0)
    vq.eval()
    return vq.to(DEV)


def _state(vq):
    cb = vq._codebook
    c = lambda t: t.detach().cpu() if t is not None else None  # noqa: E731
    w = (c(vq.project_in.weight), c(vq.project_in.bias), c(vq.project_out.weight), c(vq.project_out.bias)) \
        if vq.has_projections else (None, None, None, None)
    return ref_cpu.VQState(*w, c(cb.embed), c(cb.codebook_mean), c(cb.codebook_variance),
                           c(cb.batch_mean), c(cb.batch_variance), vq.heads)


def _oracle(st, x, mask):
    if st.w_in is None:   # project_in / out = Identity
        eye = torch.eye(x.shape[-1])
        st = ref_cpu.VQState(eye, torch.zeros(x.shape[-1]), eye, torch.zeros(x.shape[-1]), st.embed,
                             st.codebook_mean, st.codebook_variance, st.batch_mean, st.batch_variance, st.heads,
                             st.decay)
    return ref_cpu.vq_forward_eval(st, x, mask)


def _check_indices(ind_gpu, ind_ref, dist, b, n, heads):
    """dist: oracle distances (1, b*h*n, C) (negated), order '(b h) n'."""
    gi = ind_gpu.cpu().reshape(b, n, heads).permute(0, 2, 1).reshape(-1)
    ri = ind_ref.reshape(b, n, heads).permute(0, 2, 1).reshape(-1)
    d = dist[0]
    bad = (gi != ri).nonzero().flatten()
    for v in bad.tolist():
        best, got = d[v, ri[v]].item(), d[v, gi[v]].item()
        assert abs(best - got) <= 2e-5 * (1 + abs(best)), (v, ri[v].item(), gi[v].item(), best, got)
    return (gi == ri).reshape(b, heads, n).permute(0, 2, 1), bad.numel()


def _close(a, b, atol=2e-5, rtol=2e-5):
    assert torch.allclose(a.cpu(), b, atol=atol, rtol=rtol), (a.cpu() - b).abs().max()


def test_vq_golden_two_steps(pkg):
    """The reference's own outputs (gen_vq_golden.py): two consecutive masked
    eval batches, the batch statistics carried between them."""
    g = golden("vq_ref.npz")
    vq = _make(pkg, 40, int(g["heads"]), g["embed"].shape[1], g)
    for step in range(2):
        x = torch.from_numpy(g[f"x{step}"]).to(DEV)
        mask = torch.from_numpy(g[f"mask{step}"]).to(DEV)
        q, ind, loss = vq(x, mask=mask)
        assert ind.dtype == torch.long and ind.shape == g[f"indices{step}"].shape
        assert torch.equal(ind.cpu(), torch.from_numpy(g[f"indices{step}"]))
        _close(q, torch.from_numpy(g[f"quantize{step}"]))
        _close(vq._codebook.batch_mean, torch.from_numpy(g[f"batch_mean{step}"]), 1e-6, 1e-5)
        _close(vq._codebook.batch_variance, torch.from_numpy(g[f"batch_variance{step}"]), 1e-6, 1e-5)
        assert loss.shape == (1,) and float(loss) == 0.0
    ind0 = torch.from_numpy(g["indices0"]).to(DEV)
    assert torch.equal(vq.get_codes_from_indices(ind0).cpu(), torch.from_numpy(g["codes_from_indices0"]))
    _close(vq.get_output_from_indices(ind0), torch.from_numpy(g["output_from_indices0"]))


@pytest.mark.parametrize("dim,heads,C,b,n,masked", [
    (256, 8, 1024, 4, 700, True),     # projected, model-like widths
    (48, 3, 4096, 2, 513, False),     # dim == heads * 16: Identity projections, no mask
    (16, 1, 333, 3, 129, True),       # one head (embed_ind (b, n)), ragged codebook chunk
])
def test_vq_vs_oracle(pkg, dim, heads, C, b, n, masked):
    vq = _make(pkg, dim, heads, C, seed=dim + C)
    gen = torch.Generator().manual_seed(7)
    st = _state(vq)
    total_bad = 0
    for step in range(3):
        x = torch.randn(b, n, dim, generator=gen) * (1.0 + step)
        mask = (torch.rand(b, n, generator=gen) > 0.3) if masked else None
        q, ind, _ = vq(x.to(DEV), mask=mask.to(DEV) if masked else None)
        rq, rind, st, dist = _oracle(st, x, mask)
        if heads == 1:
            assert ind.shape == (b, n)
            ind = ind[..., None]
        agree, nbad = _check_indices(ind, rind, dist, b, n, heads)
        total_bad += nbad
        rows = agree.all(-1)
        if masked:
            rows = rows | ~mask
            # masked-out tokens are the input, exactly (vector_quantize.py:1044-1048)
            assert torch.equal(q.cpu()[~mask], x[~mask])
        _close(q.cpu()[rows], rq[rows], 5e-5, 5e-5)
        _close(vq._codebook.batch_mean, st.batch_mean.reshape(1, 1, -1), 1e-6, 1e-5)
        _close(vq._codebook.batch_variance, st.batch_variance.reshape(1, 1, -1), 1e-6, 1e-5)
    assert total_bad <= max(2, b * n * heads * 3 // 1000), total_bad


def test_vq_only_one_and_codes(pkg):
    """(b, d) input (vector_quantize.py:846-850) and the index gathers."""
    vq = _make(pkg, 72, 4, 256, seed=3)
    x = torch.randn(10, 72, generator=torch.Generator().manual_seed(1))
    q, ind, _ = vq(x.to(DEV))
    assert q.shape == (10, 72) and ind.shape == (10, 4)
    codes = vq.get_codes_from_indices(ind)
    ref = vq._codebook.embed.detach()[0][ind].reshape(10, 64)
    assert torch.equal(codes, ref)
    out = vq.get_output_from_indices(ind)
    _close(out, torch.nn.functional.linear(ref, vq.project_out.weight, vq.project_out.bias).cpu(), 2e-5, 2e-5)


def test_vq_index_out_of_range_raises(pkg):
    vq = _make(pkg, 64, 4, 256, seed=3)
    bad = torch.tensor([[0, 1, 2, 256]], device=DEV)
    with pytest.raises(AssertionError):
        vq.get_codes_from_indices(bad)


def test_vq_training_raises(pkg):
    vq = _make(pkg, 64, 4, 256, seed=3)
    vq.train()
    with pytest.raises(NotImplementedError):
        vq(torch.randn(2, 3, 64, device=DEV))
