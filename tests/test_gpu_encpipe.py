"""The pipelined 512^2 encode (k_enc_pipe, dctae_encpipe.hip: launch L runs
the row items of image chunk L beside the column items of chunk L - 1, T in a
two-chunk ring) against the two-kernel path (k_rows512 + k_fft_cols7) it
replaces: every packed output bit-identical (the same item bodies run), for
chunk sizes that divide the batch, leave a ragged last chunk, exceed it, and
hold one image; with the scalar (rows_kernel 3) and packed-f32 (rows_kernel 4)
row items.  The two-kernel path itself is pinned against the oracle by
test_gpu_parity.  Run on an MI355X.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def setup(pkg, ref_tables):
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    pn = pkg.PatchNorm(32, 32, 14, 3).to(DEV)
    pn.median.data.copy_(ref_tables.median)
    pn.b.data.copy_(ref_tables.b)
    pn.frozen = True
    pn.eval()
    lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(DEV).eval()
    return ops, fe_mod, fe, pn, lfq


def _run(setup, B, opts, seed):
    ops, fe_mod, fe, pn, lfq = setup
    dev = torch.device(DEV, torch.cuda.current_device())
    x = ops.synth_images(B, 512, 512, seed=seed, device=dev)
    saved = {"enc_pipe": 0, "rows_kernel": 4, "rows_p1": 0}
    for k, v in opts.items():
        ops.set_option(k, v, dev)
    try:
        enc = fe_mod.BatchEncoder(fe, B, 512, 512, pn, lfq, device=dev)
        out = {k: v.clone() for k, v in enc(x).items()}
        torch.cuda.synchronize()
        ops.check_device_errors(dev)
    finally:
        for k, v in saved.items():
            ops.set_option(k, v, dev)
    return out


def _same(a, b):
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("rows_kernel", [3, 4])
@pytest.mark.parametrize("B,C", [(1, 1), (7, 3), (16, 4), (37, 16), (20, 64)])
def test_enc_pipe_matches_two_kernel_path(setup, rows_kernel, B, C):
    ref = _run(setup, B, {"rows_kernel": rows_kernel}, seed=21)
    _same(_run(setup, B, {"rows_kernel": rows_kernel, "enc_pipe": C}, seed=21), ref)


def test_enc_pipe_full_batch(setup):
    """the bench geometry (1024 images, 32-image chunks), twice back to back"""
    ref = _run(setup, 1024, {"rows_kernel": 4}, seed=22)
    _same(_run(setup, 1024, {"rows_kernel": 4, "enc_pipe": 32}, seed=22), ref)
    _same(_run(setup, 1024, {"rows_kernel": 4, "enc_pipe": 32}, seed=22), ref)


def test_packed_rows_close_to_scalar_rows(setup):
    """rows_kernel 4 (packed f32) against 3 (scalar): the same transform with a
    different FFT operation order -> codes may differ only where a token value
    sits within rounding of its threshold; bound the count"""
    a = _run(setup, 8, {"rows_kernel": 3}, seed=23)
    b = _run(setup, 8, {"rows_kernel": 4}, seed=23)
    for k in a:
        if k != "codes":
            assert torch.equal(a[k], b[k]), k
    diff = (a["codes"] != b["codes"]).sum().item()
    assert diff <= 8, diff


@pytest.mark.parametrize("grid", [1, 7, 256])
def test_sort_grid_stride_matches(setup, grid):
    """k_sort_pack2 with fewer blocks than images (grid-stride loop, option
    sort_grid) writes the same packed rows as one block per image"""
    ops = setup[0]
    dev = torch.device(DEV, torch.cuda.current_device())
    ref = _run(setup, 40, {}, seed=24)
    ops.set_option("sort_grid", grid, dev)
    try:
        got = _run(setup, 40, {}, seed=24)
    finally:
        ops.set_option("sort_grid", 0, dev)
    _same(got, ref)


@pytest.mark.parametrize("B", [1, 7, 64, 1024])
def test_rows_p1_matches_two_kernel_path(setup, B):
    """k_rows512p1 (row pass + the column FFT's pass 1) + k_fft_cols7p2 (pass
    2 onwards): the same arithmetic as k_rows512pk + k_fft_cols7, so every
    packed output is bit-identical"""
    ref = _run(setup, B, {}, seed=25)
    _same(_run(setup, B, {"rows_p1": 1}, seed=25), ref)
