"""The split-bf16 MFMA GEMM (k_gemm_x3, dctae_kernels.hip) against float64.

dctae_dct2 runs two DCT GEMMs per image (util.py:333-338 on the whole image);
its shapes cover every operand layout the GEMM stages (k-contiguous and
m/n-contiguous A and B, shared and per-channel operands, K and M/N edges).
The bar: the orthonormal DCT computed with k_gemm_x3 is within 2e-6 of
max |Y| of the float64 DCT (scipy.fft.dctn, norm="ortho") -- the fp32 GEMM's
own error at these sizes is ~1e-6 -- and no worse than 2x the fp32 MFMA
kernel's error on the same input.
"""
import numpy as np
import pytest
import scipy.fft

import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(pkg):
    from importlib import import_module
    return import_module("dct_autoencoder_amd._ops")

SHAPES = [(1, 5), (37, 61), (64, 64), (65, 130), (100, 203), (256, 256), (333, 97)]


def _dct(ops, x, inverse, x3):
    ops.set_option("gemm_x3", int(x3))
    try:
        return ops.dct2(x, inverse=inverse, color=False).cpu().double().numpy()
    finally:
        ops.set_option("gemm_x3", 1)


@pytest.mark.parametrize("hw", SHAPES)
@pytest.mark.parametrize("inverse", [False, True])
def test_gemm_x3_dct2_vs_float64(ops, hw, inverse):
    H, W = hw
    g = np.random.default_rng(H * 1000 + W)
    x64 = g.standard_normal((2, 3, H, W))
    x = torch.tensor(x64, dtype=torch.float32, device="cuda")
    xr = x.cpu().double().numpy()
    fn = scipy.fft.idctn if inverse else scipy.fft.dctn
    ref = fn(xr, type=2, axes=(-2, -1), norm="ortho")
    scale = np.abs(ref).max()
    e3 = np.abs(_dct(ops, x, inverse, True) - ref).max() / scale
    e1 = np.abs(_dct(ops, x, inverse, False) - ref).max() / scale
    assert e3 < 2e-6, (hw, inverse, e3, e1)
    assert e3 <= 2 * e1 + 1e-7, (hw, inverse, e3, e1)


def test_gemm_x3_is_default_and_loaded(ops):
    """the default context runs k_gemm_x3 (option 1): switching it off and on
    changes the bits of a DCT whose K is not a multiple of the k step"""
    x = torch.randn(1, 3, 45, 77, device="cuda")
    a = ops.dct2(x, inverse=False, color=False)
    ops.set_option("gemm_x3", 0)
    try:
        b = ops.dct2(x, inverse=False, color=False)
    finally:
        ops.set_option("gemm_x3", 1)
    c = ops.dct2(x, inverse=False, color=False)
    assert torch.equal(a, c)
    assert not torch.equal(a, b)
