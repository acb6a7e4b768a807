"""FE._transform_image_in on fp16 / bf16 images (FE:135-141: the reference runs
rgb_to_ipt in the input dtype before x.float()): the HIP path (dctae_dct2
color 2 / 3: dtype-rounded matrices and exponent, fp32-accumulated einsums
rounded once, fp32 pow rounded) against the reference's own outputs
(tests/golden/color_dtype_ref.npz, gen_color_dtype_golden.py).

Tolerances: the IPT stage may differ from the reference only where the fp32
power (GPU powf vs the CPU's) straddles a rounding boundary of the dtype:
at most 0.2 % of values, by one dtype ulp.  The spectrum (fp32 DCT of that
IPT, cast to the dtype) within 2 dtype ulps of the value + 1e-3 x max|Y| x
(one ulp's share of the IPT differences).  Run on an MI355X.
"""
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ulp(v: torch.Tensor, dt) -> torch.Tensor:
    eps = torch.finfo(dt).eps
    return v.abs().clamp_min(torch.finfo(dt).tiny) * eps


@pytest.mark.parametrize("tag,dt,color", [("f16", torch.float16, 2), ("bf16", torch.bfloat16, 3)])
def test_low_precision_transform_in(pkg, tag, dt, color):
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    g = golden("color_dtype_ref.npz")
    for i in range(2):
        x = torch.from_numpy(g[f"{tag}_{i}_x"]).to(dt).to(DEV)
        ref_ipt = torch.from_numpy(g[f"{tag}_{i}_ipt"])
        ref_spec = torch.from_numpy(g[f"{tag}_{i}_spec"])
        # IPT stage: the fp32 spectrum of the HIP dtype-rounded IPT, inverted
        # by the fp32 IDCT, gives that IPT back to ~1e-6; it must be the
        # reference's IPT except at rare one-ulp rounding-boundary cases
        spec32 = ops.dct2(x.float(), inverse=False, color=color)
        back = ops.dct2(spec32, inverse=True, color=False).cpu()
        dd = (back - ref_ipt).abs()
        tol = 1e-5 * float(ref_ipt.abs().max())
        off = dd > tol
        assert bool(torch.all(dd[off] <= 1.01 * _ulp(ref_ipt, dt)[off] + tol)), float(dd.max())
        assert int(off.sum()) <= max(2, ref_ipt.numel() // 500), int(off.sum())
        ipt = spec32
        y = fe._transform_image_in(x)
        assert y.dtype == dt and y.shape == ref_spec.shape
        d = (y.float().cpu() - ref_spec).abs()
        lim = 2 * _ulp(ref_spec, dt) + 1e-3 * float(ref_spec.abs().max()) * torch.finfo(dt).eps
        assert bool(torch.all(d <= lim)), (tag, i, float(d.max()))
        assert torch.equal(ipt.to(dt).cpu(), y.cpu())
        # the spectrum of the reference's own IPT through the HIP fp32 DCT is
        # the reference spectrum to fp32 rounding (pins the DCT half separately)
        y2 = ops.dct2(ref_ipt.to(DEV), inverse=False, color=False).to(dt).float().cpu()
        d2 = (y2 - ref_spec).abs()
        assert bool(torch.all(d2 <= _ulp(ref_spec, dt) + 1e-6 * float(ref_spec.abs().max()))), float(d2.max())
