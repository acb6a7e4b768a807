"""GPU tests of the reference's stage hooks: callers replace
DCTAutoencoderFeatureExtractor._transform_image_in / _transform_image_out /
_patch_image / _group_patches_by_max_seq_len (reference decode_gif.py:86-91,
dct_autoencoder/tests/testpatching.py:42-43), and preprocess / postprocess /
iter_batches then run the reference's stage sequence through them.  Each
default stage is still a HIP kernel (dctae_dct2, dctae_patch_spectrum).

Tolerances: DCT coefficients 2e-6 * max|Y| vs the oracle; RGB round trips
1e-5 absolute + 1e-5 relative; identity-transform patch -> unpatch exact.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu, rng

pytestmark = pytest.mark.gpu
CFG = ref_cpu.FEConfig()
DEV = "cuda"


def _fe(pkg):
    return pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)


@pytest.mark.parametrize("shape", [(224, 224), (100, 77), (512, 512), (333, 517)])
def test_transform_image_in_out_vs_oracle(pkg, shape):
    """_transform_image_in (rgb_to_ipt + whole-image dct2, FE:129-142) and
    _transform_image_out (idct2 + ipt_to_rgb, FE:144-152) on dctae_dct2."""
    fe = _fe(pkg)
    x = torch.from_numpy(rng.synth_image(5, 0, *shape))
    y = fe._transform_image_in(x.to(DEV))
    y_o = ref_cpu.transform_image_in(x)
    assert y.shape == y_o.shape and y.device.type == "cuda"
    d = (y.cpu() - y_o).abs().max().item()
    assert d <= 2e-6 * y_o.abs().max().item(), d
    back = fe._transform_image_out(y)
    diff = (back.cpu() - x).abs()
    assert torch.all(diff <= 1e-5 + 1e-5 * x.abs()), diff.max().item()
    # a CPU input comes back on the CPU (the reference returns on the input's device)
    assert fe._transform_image_in(x).device.type == "cpu"


def test_decode_gif_spectrum_override(pkg):
    """decode_gif.py:86-91: with _transform_image_out = identity, postprocess
    returns the zero-padded spectrum (3, H, W) of the kept tokens."""
    fe = _fe(pkg)
    x = torch.from_numpy(rng.synth_image(9, 0, 300, 500))
    item = fe.preprocess(x.to(DEV))
    (batch,) = list(fe.iter_batches(iter([{k: [v] for k, v in item.items()}]), None))
    fe._transform_image_out = lambda t: t
    (spec,) = fe.postprocess(batch)
    assert spec.shape == (3, 300, 500)
    y_o = ref_cpu.transform_image_in(x)
    kh, kw = 14 * min(300 // 14, 32), 14 * min(500 // 14, 32)
    want = torch.zeros_like(y_o)
    want[:, :kh, :kw] = y_o[:, :kh, :kw]
    d = (spec.cpu() - want).abs().max().item()
    assert d <= 2e-6 * y_o.abs().max().item(), d
    assert torch.all(spec.cpu()[:, kh:, :] == 0) and torch.all(spec.cpu()[:, :, kw:] == 0)
    del fe._transform_image_out
    (img,) = fe.postprocess(batch)     # the default (fused) path again: RGB
    assert (img.cpu() - ref_cpu.transform_image_out(want)).abs().max().item() < 1e-4


@pytest.mark.parametrize("shape", [(224, 224), (98, 140), (700, 560)])
def test_identity_transforms_lossless_unpatch(pkg, shape):
    """testpatching.py:42-43 / 67-71: identity transforms make preprocess ->
    iter_batches -> postprocess a patch -> unpatch round trip of the pixels
    themselves, exact on the kept tiles (<= 32 x 32 of them), zero beyond."""
    fe = _fe(pkg)
    fe._transform_image_in = lambda t: t
    fe._transform_image_out = lambda t: t
    x = torch.from_numpy(rng.synth_image(11, 0, *shape)).to(DEV)
    item = fe.preprocess(x)
    (batch,) = list(fe.iter_batches(iter([{k: [v] for k, v in item.items()}]), None))
    (y,) = fe.postprocess(batch)
    kh, kw = 14 * min(shape[0] // 14, 32), 14 * min(shape[1] // 14, 32)
    assert torch.equal(y[:, :kh, :kw], x[:, :kh, :kw])
    assert torch.all(y[:, kh:, :] == 0) and torch.all(y[:, :, kw:] == 0)


def test_patch_image_matches_fused_preprocess(pkg):
    """A subclass wrapping _patch_image runs the staged path (dctae_dct2 +
    dctae_patch_spectrum); its tokens equal the fused preprocess's (FFT DCT)
    within the coefficient tolerance, same keys and order up to ties."""
    calls = []

    class Spy(pkg.DCTAutoencoderFeatureExtractor):
        def _patch_image(self, x):
            calls.append(tuple(x.shape))
            return super()._patch_image(x)

    fe, spy = _fe(pkg), Spy(3, 14, 0.0, 32, 32, 3072)
    x = torch.from_numpy(rng.synth_image(13, 0, 512, 512)).to(DEV)
    a = fe.preprocess(x)
    b = spy.preprocess(x)
    assert calls == [(3, 504, 504)]
    ka = {(int(c), int(p[0]), int(p[1])): i for i, (p, c) in enumerate(zip(a["positions"].tolist(), a["channels"].tolist()))}
    kb = [(int(c), int(p[0]), int(p[1])) for p, c in zip(b["positions"].tolist(), b["channels"].tolist())]
    assert sorted(ka) == sorted(kb)
    ia = torch.tensor([ka[k] for k in kb])
    ta, tb = a["patches"].cpu()[ia], b["patches"].cpu()
    assert (ta - tb).abs().max().item() <= 2e-6 * ta.abs().max().item()
    assert b["original_sizes"] == (512, 512) and b["patch_sizes"] == (36, 36)


def test_group_override_and_staged_encode(pkg, ref_tables):
    """An overridden _group_patches_by_max_seq_len drives iter_batches
    (FE:216-218); encode_batch with an overridden stage runs preprocess ->
    iter_batches -> PatchNorm -> LFQ through the hooks and agrees with the
    fused encode (same packing metadata; codes inside the guard band)."""
    fe = _fe(pkg)
    seen = []
    default_group = fe._group_patches_by_max_seq_len

    def group(*a, **k):
        seen.append(len(a[0]))
        return default_group(*a, **k)

    fe._group_patches_by_max_seq_len = group
    pn = pkg.PatchNorm(32, 32, 14, 3).to(DEV)
    pn.median.data.copy_(ref_tables.median)
    pn.b.data.copy_(ref_tables.b)
    pn.n.data.copy_(ref_tables.n)
    pn.frozen = True
    pn.eval()
    lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(DEV).eval()
    xs = [torch.from_numpy(a).to(DEV) for a in rng.synth_images(17, [(224, 224), (100, 300), (224, 224)])]
    ((dp_s, c_s),) = fe.encode_batch(xs, pn, lfq)
    assert seen == [3]
    ((dp_f, c_f),) = _fe(pkg).encode_batch(xs, pn, lfq)
    assert torch.equal(dp_s.key_pad_mask.cpu(), dp_f.key_pad_mask.cpu())
    assert torch.equal(dp_s.batched_image_ids.cpu(), dp_f.batched_image_ids.cpu())
    assert (c_s.cpu() != c_f.cpu()).sum().item() <= 4
