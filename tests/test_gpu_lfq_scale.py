"""The reference LFQ's index rule at any codebook_scale (lfq.py:174-187:
quantized = where(x > 0, +s, -s); index bit = quantized > 0), on every HIP
index producer, against the reference's own LFQ outputs
(tests/golden/lfq_scale_ref.npz, gen_lfq_scale_golden.py) at s = 1, 0.5, 0,
-1, -0.25, inputs with +0 / -0 / NaN elements and NaN tokens.

Producers covered:
  * dctae_lfq_forward (LFQ.forward without projections): bit-exact indices and
    quantized values;
  * dctae_lfq_project_in (LFQ.forward with projections, fused MFMA projection):
    indices equal outside the fp32 GEMM rounding band of the reference's
    projected value h (|h| <= 4e-6 (|W||x| + |b|)); NaN tokens exact;
  * the fused encode (threshold epilogue -> u16 staging -> k_sort_pack2 /
    k_pad_fill mapping) and dctae_encode_lfq_proj (staged projection): the
    codes at scale s equal the scale-1 codes of the same images mapped by the
    reference rule, bit for bit (the scale-1 codes are pinned against the
    oracle by test_gpu_parity / test_gpu_lfq_proj);
  * dctae_model_lfq (the transformer's LFQ): bit-exact indices.
Run on an MI355X.
"""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from oracle import rng

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = golden("lfq_scale_ref.npz")
SCALES = [float(s) for s in G["scales"]]


def _map(codes1, s, cd):
    """the reference rule applied to sign-bit codes (= the scale-1 codes)"""
    full = (1 << cd) - 1
    if s > 0:
        return codes1
    if -s > 0:
        return codes1 ^ full
    return torch.zeros_like(codes1)


@pytest.mark.parametrize("si", range(len(SCALES)))
def test_lfq_forward_scale(pkg, si):
    s = SCALES[si]
    m = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14, codebook_scale=s).to(DEV).eval()
    x = torch.from_numpy(G["x"]).to(DEV)
    q, idx, _, _ = m(x, mask=torch.ones(x.shape[:2], dtype=torch.bool, device=DEV))
    assert torch.equal(idx.cpu(), torch.from_numpy(G[f"n{si}_idx"])), s
    assert torch.equal(q.cpu(), torch.from_numpy(G[f"n{si}_q"])), s
    codes = m.indices_to_codes(idx)
    assert torch.equal(codes.cpu(), torch.from_numpy(G[f"n{si}_codes"])), s


@pytest.mark.parametrize("si", range(len(SCALES)))
def test_lfq_project_in_scale(pkg, si):
    s = SCALES[si]
    m = pkg.LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16, codebook_scale=s)
    with torch.no_grad():
        m.project_in.weight.copy_(torch.from_numpy(G["w_in"]))
        m.project_in.bias.copy_(torch.from_numpy(G["b_in"]))
        m.project_out.weight.copy_(torch.from_numpy(G["w_out"]))
        m.project_out.bias.copy_(torch.from_numpy(G["b_out"]))
    m = m.to(DEV).eval()
    assert m._fused_proj()
    xc = torch.from_numpy(G["x"])
    q, idx, _, _ = m(xc.to(DEV), mask=torch.ones(xc.shape[:2], dtype=torch.bool, device=DEV))
    ref = torch.from_numpy(G[f"p{si}_idx"])
    h = torch.from_numpy(G[f"p{si}_h"])
    band = 4e-6 * F.linear(xc.abs(), torch.from_numpy(G["w_in"]).abs(), torch.from_numpy(G["b_in"]).abs())
    near = (h.abs() <= band).view(*ref.shape, 13).any(-1)
    diff = idx.cpu() != ref
    assert not torch.any(diff & ~near), f"scale {s}: index mismatch outside the rounding band"
    nan_tok = torch.isnan(xc).any(-1)   # NaN tokens project to NaN: every bit is the rule's NaN bit
    assert torch.equal(idx.cpu()[nan_tok], ref[nan_tok])
    assert int(diff.sum()) <= 2
    # q = project_out(where(h > 0, s, -s)) (lfq.py:174-212) on the tokens whose
    # indices agree, within the fp32 GEMM band 2e-5 (|W_out| |s| + |b_out|)
    same = ~diff.any(-1)
    q_ref = torch.from_numpy(G[f"p{si}_q"])
    w_out, b_out = torch.from_numpy(G["w_out"]), torch.from_numpy(G["b_out"])
    qband = 2e-5 * (w_out.abs().sum(-1) * abs(s) + b_out.abs()) + 1e-7
    assert torch.all(((q.cpu() - q_ref).abs() <= qband)[same]), f"scale {s}: project_out(quantized) differs"


def _encode_codes(pkg, fe, pn, imgs, s, batch_encoder=False, proj=None):
    kw = dict(codebook_scale=s)
    if proj is None:
        lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14, **kw)
    else:
        lfq = pkg.LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16, **kw)
        lfq.load_state_dict(proj, strict=False)
    lfq = lfq.to(DEV).eval()
    if batch_encoder:
        from importlib import import_module
        fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
        H = imgs[0].shape[-1]
        enc = fe_mod.BatchEncoder(fe, len(imgs), H, H, pn, lfq, device=DEV)
        return enc(torch.stack(imgs).contiguous())["codes"].clone()
    ((dp, codes),) = fe.encode_batch(imgs, pn, lfq)
    return codes


@pytest.fixture(scope="module")
def fe(pkg):
    return pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)


@pytest.fixture(scope="module")
def pn(pkg, ref_tables):
    m = pkg.PatchNorm(32, 32, 14, 3).to(DEV)
    m.median.data.copy_(ref_tables.median)
    m.b.data.copy_(ref_tables.b)
    m.frozen = True
    return m.eval()


@pytest.mark.parametrize("sizes", [[(224, 224), (100, 140), (300, 500)], [(512, 512), (512, 512)]])
def test_fused_encode_scale(pkg, fe, pn, sizes):
    """threshold epilogue + sort_pack2 (+ pad_fill for the rows with pads)"""
    imgs = [torch.from_numpy(x).to(DEV) for x in rng.synth_images(91, sizes)]
    c1 = _encode_codes(pkg, fe, pn, imgs, 1.0)
    for s in SCALES[1:]:
        assert torch.equal(_encode_codes(pkg, fe, pn, imgs, s), _map(c1, s, 14)), s


def test_batch_encoder_scale(pkg, fe, pn):
    imgs = [torch.from_numpy(x).to(DEV) for x in rng.synth_images(92, [(512, 512)] * 2)]
    c1 = _encode_codes(pkg, fe, pn, imgs, 1.0, batch_encoder=True)
    for s in SCALES[1:]:
        assert torch.equal(_encode_codes(pkg, fe, pn, imgs, s, batch_encoder=True), _map(c1, s, 14)), s


@pytest.mark.parametrize("H", [224, 512])
def test_projected_encode_scale(pkg, fe, pn, H):
    """staged projection (dctae_encode_lfq_proj, 512^2: full rows) and the
    packed path + dctae_lfq_project_in (224^2: rows with pads)"""
    imgs = [torch.from_numpy(x).to(DEV) for x in rng.synth_images(93, [(H, H)] * 2)]
    proj = {k: torch.from_numpy(G[n]) for k, n in (("project_in.weight", "w_in"), ("project_in.bias", "b_in"),
                                                    ("project_out.weight", "w_out"), ("project_out.bias", "b_out"))}
    c1 = _encode_codes(pkg, fe, pn, imgs, 1.0, batch_encoder=True, proj=proj)
    for s in SCALES[1:]:
        assert torch.equal(_encode_codes(pkg, fe, pn, imgs, s, batch_encoder=True, proj=proj), _map(c1, s, 13)), s


@pytest.mark.parametrize("si", range(len(SCALES)))
def test_model_lfq_scale(pkg, si):
    from dct_autoencoder_amd import _lib
    s = SCALES[si]
    x = torch.from_numpy(G["x"]).reshape(-1, 196).to(DEV).contiguous()
    m = x.shape[0]
    codes = torch.empty(m, 14, dtype=torch.long, device=DEV)
    xq = torch.empty(m, 196, device=DEV)
    ctx = _lib.context(torch.device(DEV, torch.cuda.current_device()))
    ctx.check(ctx.lib.dctae_model_lfq(ctx.h, m, 14, 14, C.c_float(s), _lib.ptr(x), 196, _lib.ptr(codes), None,
                                      _lib.ptr(xq), 196, _lib.stream_ptr(x.device)), "lfq")
    torch.cuda.synchronize()
    assert torch.equal(codes.cpu().view(1, m, 14), torch.from_numpy(G[f"n{si}_idx"])), s
    assert torch.equal(xq.cpu().view(1, m, 196), torch.from_numpy(G[f"n{si}_q"])), s


@pytest.mark.parametrize("dim", [None, 24])
def test_large_codebook_codes_are_float(pkg, dim):
    """codebook_size > 2**16 (no materialised codebook buffer): indices_to_codes
    keeps the float codebook dtype (lfq.py:101-124), so a non-integer scale
    survives and project_out (dim 24 != 17) gets a float tensor."""
    m = pkg.LFQ(dim=dim, codebook_size=2 ** 17, codebook_scale=0.5).to(DEV).eval()
    assert not hasattr(m, "codebook") and m.dtype == torch.float32
    idx = torch.tensor([[0, 1, 2 ** 17 - 1, 12345]], device=DEV)
    codes = m.indices_to_codes(idx, project_out=False)
    assert codes.dtype == torch.float32
    bits = ((idx[..., None] & (2 ** torch.arange(16, -1, -1, device=DEV))) != 0).float()
    assert torch.equal(codes, bits * 0.5 * 2 - 0.5)
    if dim is not None:
        out = m.indices_to_codes(idx)
        assert out.dtype == torch.float32 and out.shape == (1, 4, dim)
