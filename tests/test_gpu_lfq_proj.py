"""LFQ with projections through the fused encode_batch / decode_batch
(lfq.py:54-62: dim != codebook_dim * num_codebooks inserts Linear project_in /
project_out; conf/patch14-l.json's 16 codebooks of 2^13 over 196-element
tokens: 196 -> 208 -> 196), against the CPU oracle.  Run on an MI355X.

Tolerances (stated per test):
  * codes: given the GPU's own PatchNorm output y (bit-exact PatchNorm of
    tokens test_gpu_parity already pins), a bit may differ from the oracle's
    LFQ(project_in(y)) only where the oracle's projected value h lies inside
    the fp32 GEMM rounding band |h| <= 4e-6 * (|W| |y| + |b|);
  * decode: RGB within 1e-5 of the image range (+2e-5 relative) of the
    oracle's decode of the same codes (project_out -> inverse PatchNorm ->
    revert_patching -> IDCT -> IPT -> RGB).
"""
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_cpu, rng

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = ref_cpu.FEConfig()
LCFG = ref_cpu.LFQConfig(dim=196, codebook_size=2 ** 13, num_codebooks=16)
LFQ_WS_DEFAULT = 1   # dctae_api.hip: ctx->lfq_ws


@pytest.fixture(scope="module")
def fe(pkg):
    return pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)


@pytest.fixture(scope="module")
def pn(pkg, ref_tables):
    m = pkg.PatchNorm(32, 32, 14, 3).to(DEV)
    m.median.data.copy_(ref_tables.median)
    m.b.data.copy_(ref_tables.b)
    m.n.data.copy_(ref_tables.n)
    m.frozen = True
    return m.eval()


@pytest.fixture(scope="module")
def lfq_p(pkg):
    torch.manual_seed(5)
    m = pkg.LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16)
    assert m.has_projections and LCFG.has_projections
    return m.to(DEV).eval()


def _w(lin):
    return lin.weight.detach().cpu(), lin.bias.detach().cpu()


def _images(seed, sizes):
    return [torch.from_numpy(x).to(DEV) for x in rng.synth_images(seed, sizes)]


@pytest.mark.parametrize("sizes", [[(224, 224), (300, 500), (97, 1000)], [(512, 512)]])
def test_encode_batch_with_projections(fe, pn, lfq_p, sizes):
    imgs = _images(77, sizes)
    ((dp, codes),) = fe.encode_batch(imgs, pn, lfq_p, return_patches=True)
    R, S = dp.key_pad_mask.shape
    assert codes.shape == (R, S, 16) and codes.dtype == torch.long
    y = dp.patches.cpu()                       # PatchNorm output, pads included
    W, b = _w(lfq_p.project_in)
    h = F.linear(y, W, b)
    _, oidx = ref_cpu.lfq_forward(y, LCFG, project_in=lambda t: F.linear(t, W, b))
    g = codes.cpu()
    diff = g != oidx
    band = 4e-6 * F.linear(y.abs(), W.abs(), b.abs())
    near = (h.abs() <= band).view(R, S, 16, 13).any(-1)
    assert torch.all(near[diff]), "code mismatch outside the GEMM rounding band"
    flips, n = int(diff.sum()), g.numel()
    print(f"[{sizes}] projected-code mismatches inside the band: {flips} / {n}")
    assert flips <= max(2, n // 1000)
    # the codes do not depend on whether the normalised tokens are returned
    ((dp2, codes2),) = fe.encode_batch(imgs, pn, lfq_p)
    assert torch.equal(codes2.cpu(), g) and dp2.patches.shape[-1] == 0
    assert torch.equal(dp2.key_pad_mask, dp.key_pad_mask) and torch.equal(dp2.patch_positions, dp.patch_positions)


def test_decode_batch_with_projections(fe, pn, lfq_p, ref_tables):
    imgs = _images(78, [(224, 224), (300, 500), (512, 512)])
    ((dp, codes),) = fe.encode_batch(imgs, pn, lfq_p)
    out = fe.decode_batch(dp, codes, pn, lfq_p)
    Wo, bo = _w(lfq_p.project_out)
    q = ref_cpu.lfq_indices_to_codes(codes.cpu(), LCFG, project_out=lambda t: F.linear(t, Wo, bo))
    kp, ids, pos, ch = (dp.key_pad_mask.cpu(), dp.batched_image_ids.cpu(), dp.patch_positions.cpu(),
                        dp.patch_channels.cpu())
    x = ref_cpu.norm_inverse(ref_tables, q, ch, pos[..., 0], pos[..., 1])
    batch = ref_cpu.Batch(x, kp, None, ids, ch, pos, list(dp.patch_sizes), list(dp.original_sizes))
    ref = ref_cpu.postprocess(batch, CFG)
    assert len(out) == len(ref) == len(imgs)
    for a, r in zip(out, ref):
        assert a.shape == r.shape
        scale = max(1.0, float(r.abs().max()))
        d = (a.cpu() - r).abs()
        assert torch.all(d <= 1e-5 * scale + 2e-5 * r.abs()), (float(d.max()), scale)


@pytest.mark.parametrize("B,H", [(3, 224), (2, 512)])
def test_batch_encoder_with_projections(pkg, fe, pn, lfq_p, B, H):
    """The pre-planned BatchEncoder (bench path) with projections equals
    encode_batch bit for bit (same kernels, same plan)."""
    from importlib import import_module
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    enc = fe_mod.BatchEncoder(fe, B, H, H, pn, lfq_p, device=DEV)
    # 512^2 rows are full (3072 tokens): dctae_encode_lfq_proj (projection on the
    # staged tokens before the sort / pack); 224^2 rows hold pads: the packed path
    assert enc.proj_staged == (H == 512)
    imgs = _images(79, [(H, H)] * B)
    out = enc(torch.stack(imgs).contiguous())
    ((dp, codes),) = fe.encode_batch(imgs, pn, lfq_p, return_patches=True)
    assert torch.equal(out["codes"], codes) and torch.equal(out["key_pad_mask"], dp.key_pad_mask)
    assert torch.equal(out["positions"], dp.patch_positions)
    assert torch.equal(out["image_ids"], dp.batched_image_ids)


@pytest.mark.parametrize("dim,cd,ncb,n,bias", [(196, 13, 16, 3072 * 3 + 5, True), (196, 13, 16, 1, True),
                                               (256, 15, 16, 700, True), (64, 5, 4, 130, False),
                                               (196, 14, 12, 257, True), (12, 31, 4, 64, True),
                                               (196, 17, 12, 300, True), (196, 20, 10, 100, True)])
def test_project_kernels_vs_linear(pkg, dim, cd, ncb, n, bias):
    """dctae_lfq_project_in / _out (the fused MFMA kernels) against torch fp32
    nn.Linear on the CPU.  Tolerance: a code bit may differ only where the CPU's
    projected value lies in the fp32 rounding band |h| <= 4e-6 (|W| |x| + |b|);
    project_out within 2e-5 (|W| |codes| + |b|) (the f32 sum over <= 256 terms
    in another order).  codebook_dim 17 / 20 with K = 204 / 200 -> 196: shapes
    k_lfq_ws's project_out must refuse (its code bits are combined in 32 bits,
    cd <= 16), so they run on k_lfq_proj_h2."""
    torch.manual_seed(dim + cd + n)
    m = pkg.LFQ(dim=dim, codebook_size=2 ** cd, num_codebooks=ncb)
    if not bias:
        m.project_in.bias = None
        m.project_out.bias = None
    m = m.to(DEV).eval()
    assert m._fused_proj()
    cfg = ref_cpu.LFQConfig(dim=dim, codebook_size=2 ** cd, num_codebooks=ncb)
    x = torch.randn(n, dim)
    x[0, :3] = float("nan") if n > 1 else x[0, :3]
    W, b = m.project_in.weight.detach().cpu(), m.project_in.bias
    b = None if b is None else b.detach().cpu()
    idx = m.project_codes(x.to(DEV)).cpu()
    h = F.linear(x, W, b)
    _, oidx = ref_cpu.lfq_forward(x[None], cfg, project_in=lambda t: F.linear(t, W, b))
    oidx = oidx[0]
    diff = idx != oidx
    band = 4e-6 * F.linear(x.abs(), W.abs(), None if b is None else b.abs())
    near = (h.abs() <= band).view(n, ncb, cd).any(-1)
    if n > 1:   # the NaN row: every bit of a codebook touching a NaN feature is 0 on both sides
        near[0] = True
    assert torch.all(near[diff]), "code mismatch outside the fp32 rounding band"
    assert int(diff.sum()) <= max(2, idx.numel() // 1000)
    # decode direction, on the oracle's indices
    Wo, bo = m.project_out.weight.detach().cpu(), m.project_out.bias
    bo = None if bo is None else bo.detach().cpu()
    got = m.indices_to_codes(oidx.to(DEV)).cpu()
    codes = ref_cpu.lfq_indices_to_codes(oidx, cfg)
    ref = F.linear(codes, Wo, bo)
    tol = 2e-5 * F.linear(codes.abs(), Wo.abs(), None if bo is None else bo.abs())
    assert got.shape == ref.shape and torch.all((got - ref).abs() <= tol), float((got - ref).abs().max())
    # LFQ.forward = both kernels (eval quantized = +-scale of the index bits)
    q, i2, _, _ = m(x.to(DEV), mask=torch.ones(n, dtype=torch.bool, device=DEV))
    assert torch.equal(i2.cpu(), idx)
    assert torch.equal(q.cpu(), m.indices_to_codes(idx.to(DEV)).cpu())


def test_batch_decoder_with_projections(pkg, fe, pn, lfq_p):
    """BatchDecoder with projections (fused project_out -> inverse PatchNorm ->
    decode from tokens) equals decode_batch on the same codes (same kernels)."""
    from importlib import import_module
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    enc = fe_mod.BatchEncoder(fe, 2, 512, 512, pn, lfq_p, device=DEV)
    imgs = _images(80, [(512, 512)] * 2)
    out = enc(torch.stack(imgs).contiguous())
    got = fe_mod.BatchDecoder(enc, pn, lfq_p)(out)
    ((dp, codes),) = fe.encode_batch(imgs, pn, lfq_p)
    ref = fe.decode_batch(dp, codes, pn, lfq_p)
    assert got.shape == (2, 3, 512, 512)
    for i in range(2):
        assert torch.equal(got[i], ref[i]), float((got[i] - ref[i]).abs().max())


def test_decode_normed_equals_inverse_then_decode(pkg, fe, pn, lfq_p):
    """dctae_decode_normed (PatchNorm-space tokens, the inverse inside the
    decode) == dctae_norm_inverse then dctae_decode, bit for bit: on 512^2
    (the FFT column kernel applies the inverse with per-block tables;
    BatchDecoder's projections path, against its project_out + inverse path)
    and on GEMM-path geometries (the inverse into the staging buffer first)."""
    from importlib import import_module
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    ops = import_module("dct_autoencoder_amd._ops")
    enc = fe_mod.BatchEncoder(fe, 3, 512, 512, pn, lfq_p, device=DEV)
    imgs = _images(82, [(512, 512)] * 3)
    out = enc(torch.stack(imgs).contiguous())
    dec = fe_mod.BatchDecoder(enc, pn, lfq_p)
    assert dec.normed_decode
    a = dec(out).clone()
    dec.normed_decode = False
    b = dec(out).clone()
    assert torch.equal(a, b), float((a - b).abs().max())
    imgs = _images(83, [(224, 224), (300, 500), (97, 1000)])
    ((dp, codes),) = fe.encode_batch(imgs, pn, lfq_p)
    w, bb = lfq_p._proj_w(lfq_p.project_out, codes.device)
    x = ops.lfq_project_out(codes, w, bb, lfq_p.cfg())
    st = pn.state(thresholds=False)
    args = (fe.params(dp.key_pad_mask.shape[1]), dp.batched_image_ids, dp.key_pad_mask, dp.patch_positions,
            dp.patch_channels, dp.patch_sizes, dp.original_sizes)
    got = ops.decode(*args, patches=x, norm=st, normed=True)
    d2 = dp.shallow_copy()
    d2.patches = x
    ref = ops.decode(*args, patches=pn.inverse_norm(d2))
    assert len(got) == len(ref) == 3
    for g, r in zip(got, ref):
        assert torch.equal(g, r), float((g - r).abs().max())


def test_project_out_inverse_norm_fused(pkg, fe, pn, lfq_p):
    """dctae_lfq_project_out_inverse_norm == project_out kernel then the
    dctae_norm_inverse kernel, bit for bit (same fp32 ops, no FMA)."""
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    imgs = _images(81, [(224, 224), (300, 500)])
    ((dp, codes),) = fe.encode_batch(imgs, pn, lfq_p)
    w, b = lfq_p._proj_w(lfq_p.project_out, codes.device)
    fused = ops.lfq_project_out_inverse_norm(codes, w, b, lfq_p.cfg(), pn.state(thresholds=False), fe.params(),
                                             dp.patch_channels, dp.patch_positions)
    d2 = dp.shallow_copy()
    d2.patches = lfq_p.indices_to_codes(codes)
    two = pn.inverse_norm(d2)
    assert torch.equal(fused, two)
    bad = dp.patch_positions.clone()
    bad[0, 0, 0] = 99                                   # out-of-range table row: NaN + device error flag
    out = ops.lfq_project_out_inverse_norm(codes, w, b, lfq_p.cfg(), pn.state(thresholds=False), fe.params(),
                                           dp.patch_channels, bad)
    assert torch.isnan(out[0, 0]).all() and torch.equal(out[0, 1:], fused[0, 1:])
    with pytest.raises(Exception):
        ops.check_device_errors(codes.device)


@pytest.mark.parametrize("sizes", [[(512, 512), (512, 512)], [(224, 224), (97, 1000), (300, 500)]])
def test_w_stationary_kernel_vs_lfq_proj_h2(pkg, fe, pn, lfq_p, sizes):
    """k_lfq_ws (option lfq_ws=1) against k_lfq_proj_h2 (lfq_ws=0):
    the same fp16 pieces and products summed in another order, so the codes
    agree except inside the rounding band (<= 1 in 1000 bits) and the decode
    within 2e-5 (|W| |codes| + |b|) of each other; both directions, fused
    inverse PatchNorm included, ragged tails (n not a multiple of 32)."""
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    dev = torch.device(DEV, 0)
    imgs = _images(82, sizes)
    try:
        ops.set_option("lfq_ws", 0, dev)
        ((dp0, c0),) = fe.encode_batch(imgs, pn, lfq_p, return_patches=True)
        q0 = lfq_p.indices_to_codes(c0)
        o0 = fe.decode_batch(dp0, c0, pn, lfq_p)
        ops.set_option("lfq_ws", 1, dev)
        ((dp1, c1),) = fe.encode_batch(imgs, pn, lfq_p, return_patches=True)
        q1 = lfq_p.indices_to_codes(c0)
        o1 = fe.decode_batch(dp0, c0, pn, lfq_p)
    finally:
        ops.set_option("lfq_ws", LFQ_WS_DEFAULT, dev)
    assert torch.equal(dp1.patches, dp0.patches)
    diff = int((c1 != c0).sum())
    print(f"[{sizes}] codes differing between the two kernels: {diff} / {c1.numel()}")
    assert diff <= max(2, c1.numel() // 1000)
    Wo, bo = _w(lfq_p.project_out)
    codes = ref_cpu.lfq_indices_to_codes(c0.cpu(), LCFG)
    tol = 2e-5 * F.linear(codes.abs(), Wo.abs(), bo.abs())
    assert torch.all((q1.cpu() - q0.cpu()).abs() <= tol)
    for a, r in zip(o1, o0):
        scale = max(1.0, float(r.abs().max()))
        assert torch.all((a - r).abs() <= 1e-5 * scale + 2e-5 * r.abs())


@pytest.mark.parametrize("n", [3072 * 3 + 5, 1, 130, 64, 256 * 64 * 3 + 37])
@pytest.mark.parametrize("ws", [1, 0])
def test_project_in_bounded_vs_linear(pkg, n, ws):
    """dctae_lfq_project_in_bounded (|x| <= 6, the PatchNorm clamp: the fp16
    kernels -- k_lfq_ws with option lfq_ws=1, k_lfq_proj_h2 with 0) against
    torch fp32 nn.Linear on the CPU, conf/patch14-l.json's 196 -> 16 x 13.
    Tolerance: a code bit may differ only where the CPU's projected value lies
    in the band |h| <= 4e-6 (|W| |x| + |b|); ragged n (tiles of 64 / 32).
    n = 256 x 64 x 3 + 37 gives k_lfq_ws four 64-token tiles per block on 256
    CUs: the persistent loop's later tiles (the next tile's loads in flight),
    which the bench's 3.1 M-token leg runs."""
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    dev = torch.device(DEV, 0)
    torch.manual_seed(n + ws)
    m = pkg.LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16).to(DEV).eval()
    x = (torch.rand(n, 196) * 12 - 6)
    x[0, :2] = 6.0
    W, b = m.project_in.weight.detach().cpu(), m.project_in.bias.detach().cpu()
    w_d, b_d = m._proj_w(m.project_in, dev)
    try:
        ops.set_option("lfq_ws", ws, dev)
        idx = ops.lfq_project_in(x.to(DEV), w_d, b_d, m.cfg(m.project_in.weight.dtype), 6.0).cpu()
    finally:
        ops.set_option("lfq_ws", LFQ_WS_DEFAULT, dev)
    h = F.linear(x, W, b)
    _, oidx = ref_cpu.lfq_forward(x[None], LCFG, project_in=lambda t: F.linear(t, W, b))
    diff = idx != oidx[0]
    band = 4e-6 * F.linear(x.abs(), W.abs(), b.abs())
    near = (h.abs() <= band).view(n, 16, 13).any(-1)
    assert torch.all(near[diff]), f"{int((diff & ~near).sum())} codes outside the rounding band"
    assert int(diff.sum()) <= max(2, idx.numel() // 1000)


@pytest.mark.parametrize("proj", [True, False])
def test_decode_batch_honours_out_hooks(pkg, pn, lfq_p, proj):
    """decode_batch with an overridden _transform_image_out (decode_gif.py:86-91:
    identity, so postprocess returns the kept spectrum) runs the staged
    indices_to_codes -> inverse_norm -> postprocess sequence through the hook,
    with and without LFQ projections; without the override the fused decode
    runs again and equals the hook's spectrum put through the default
    _transform_image_out (1e-5 x image range)."""
    fe2 = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    lfq = lfq_p if proj else pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(DEV).eval()
    imgs = _images(84, [(224, 224), (300, 500), (512, 512)])
    ((dp, codes),) = fe2.encode_batch(imgs, pn, lfq)
    fe2._transform_image_out = lambda t: t
    spec = fe2.decode_batch(dp, codes, pn, lfq)
    d2 = dp.shallow_copy()
    d2.patches = lfq.indices_to_codes(codes)
    d2.patches = pn.inverse_norm(d2)
    want = fe2.postprocess(d2)
    assert len(spec) == len(want) == len(imgs)
    for s, w, im in zip(spec, want, imgs):
        assert s.shape == im.shape and torch.equal(s, w)
    del fe2._transform_image_out
    rgb = fe2.decode_batch(dp, codes, pn, lfq)
    for s, r in zip(spec, rgb):
        back = fe2._transform_image_out(s)
        scale = max(1.0, float(r.abs().max()))
        assert torch.all((back - r).abs() <= 1e-5 * scale + 2e-5 * r.abs()), float((back - r).abs().max())
