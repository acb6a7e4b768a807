"""GPU parity of the DCTAutoencoder transformer path.

Operator tests compare each HIP kernel with a plain torch fp32 computation on
the same (bf16-rounded) inputs; the model test runs the reference's own
weights and inputs (tests/golden/model_ref.npz) through the MI355X forward
and compares with the reference's outputs.  Tolerances are bf16-level: the
kernels take bf16 operands (the reference itself runs this model in fp16 /
bf16, main.py:331-347) and accumulate in fp32."""
import ctypes as C
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_model as R

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
HERE = os.path.dirname(os.path.abspath(__file__))


def _lib(pkg):
    from importlib import import_module
    return import_module("dct_autoencoder_amd._lib")


def _bf(x):
    return x.to(torch.bfloat16)


def _bits(x):
    return _bf(x).view(torch.int16).contiguous()


@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("m,n,k", [(300, 200, 192), (256, 384, 1024), (77, 52, 128), (2304, 200, 192), (3000, 384, 64), (4100, 3900, 128)])
def test_linear_epilogues(pkg, epi, m, n, k):
    L = _lib(pkg)
    ctx = L.context(DEV)
    g = torch.Generator(device="cpu").manual_seed(m + n + k)
    x = _bf(torch.randn(m, k, generator=g)).float().to(DEV)
    w = _bf(torch.randn(n, k, generator=g) / k ** 0.5).float().to(DEV)
    b = torch.randn(n, generator=g).to(DEV)
    ref = x @ w.T + b
    if epi == 0:
        out = torch.empty(m, n, device=DEV)
    elif epi == 3:
        base = torch.randn(m, n, generator=g).to(DEV)
        out = base.clone()
        ref = base + ref
    else:
        out = torch.empty(m, n, dtype=torch.int16, device=DEV)
    if epi == 2:
        ref = ref * torch.sigmoid(1.702 * ref)
    xb, wb = _bits(x), _bits(w)   # keep the operands alive until the kernel has run
    ctx.check(ctx.lib.dctae_model_linear(ctx.h, m, n, k, L.ptr(xb), k, L.ptr(wb), n, k, L.ptr(b), epi,
                                         L.ptr(out), n, L.stream_ptr(DEV)), "linear")
    torch.cuda.synchronize()
    got = out.view(torch.bfloat16).float() if epi in (1, 2) else out
    tol = 1e-4 if epi in (0, 3) else 8e-3   # fp32 out: order of summation only; bf16 out: one rounding
    assert (got - ref).abs().max().item() <= tol * ref.abs().max().item() + 1e-5


def test_linear_rejects_bad_k(pkg):
    L = _lib(pkg)
    ctx = L.context(DEV)
    x = torch.zeros(4, 100, dtype=torch.int16, device=DEV)
    with pytest.raises(AssertionError):
        ctx.check(ctx.lib.dctae_model_linear(ctx.h, 4, 8, 100, L.ptr(x), 100, L.ptr(x), 8, 100, None, 0, L.ptr(x), 8,
                                             L.stream_ptr(DEV)), "linear")


def _packing(r, s, seed):
    """ids / key_pad of r rows: a few images per row, then padding."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.zeros(r, s, dtype=torch.long)
    kp = torch.zeros(r, s, dtype=torch.bool)
    for i in range(r):
        n = int(torch.randint(s // 2, s, (1,), generator=g))
        cuts = sorted(torch.randint(1, n, (2,), generator=g).tolist())
        ids[i, cuts[0]:cuts[1]] = 1
        ids[i, cuts[1]:n] = 2
        kp[i, n:] = True
    return ids, kp


@pytest.mark.parametrize("r,s,heads", [(2, 320, 2), (1, 3072, 4), (3, 256, 1)])
def test_attention_vs_torch(pkg, r, s, heads):
    L = _lib(pkg)
    ctx = L.context(DEV)
    d = 64 * heads
    g = torch.Generator().manual_seed(r * s + heads)
    qkv = _bf(torch.randn(r * s, 3 * d, generator=g)).float()
    ids, kp = _packing(r, s, s)
    q, k, v = (qkv[:, i * d:(i + 1) * d].view(r, s, heads, 64).transpose(1, 2) for i in range(3))
    logits = q @ k.transpose(-1, -2) / 8.0 + R.attn_bias(ids, kp)
    ref = (torch.softmax(logits, -1) @ v).transpose(1, 2).reshape(r * s, d)
    out = torch.empty(r * s, d, dtype=torch.int16, device=DEV)
    qb, idd, kpd = _bits(qkv).to(DEV), ids.to(DEV), kp.to(torch.uint8).to(DEV)
    ctx.check(ctx.lib.dctae_model_attention(ctx.h, r, s, heads, 64, L.ptr(qb), L.ptr(idd), L.ptr(kpd), L.ptr(out), d,
                                            L.stream_ptr(DEV)), "attention")
    torch.cuda.synchronize()
    got = out.view(torch.bfloat16).float().cpu()
    # P is rounded to bf16 before P.V: ~2^-8 relative per term
    assert (got - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("d", [128, 1024])
def test_layernorm_and_embed_norm(pkg, d):
    L = _lib(pkg)
    ctx = L.context(DEV)
    m = 333
    g = torch.Generator().manual_seed(d)
    x = (torch.randn(m, d, generator=g) * 3 + 1).to(DEV)
    gam, bet = torch.randn(d, generator=g).to(DEV), torch.randn(d, generator=g).to(DEV)
    out = torch.empty(m, d, dtype=torch.int16, device=DEV)
    ctx.check(ctx.lib.dctae_model_layernorm(ctx.h, m, d, L.ptr(x), d, L.ptr(gam), L.ptr(bet), C.c_float(1e-5),
                                            L.ptr(out), d, L.stream_ptr(DEV)), "ln")
    ref = F.layer_norm(x, (d,), gam, bet, 1e-5)
    torch.cuda.synchronize()
    assert (out.view(torch.bfloat16).float() - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    ph, pw, pc = (torch.randn(n, d, generator=g).to(DEV) for n in (32, 32, 3))
    ch = torch.randint(0, 3, (m,), generator=g).to(DEV)
    pos = torch.randint(0, 32, (m, 2), generator=g).to(DEV)
    o2 = torch.empty(m, d, device=DEV)
    ctx.check(ctx.lib.dctae_model_embed_norm(ctx.h, m, d, L.ptr(x), d, L.ptr(gam), L.ptr(bet), C.c_float(1e-4),
                                             L.ptr(ph), L.ptr(pw), L.ptr(pc), L.ptr(ch), L.ptr(pos), L.ptr(o2), d,
                                             L.stream_ptr(DEV)), "embed_norm")
    ref2 = F.layer_norm(x, (d,), gam, bet, 1e-4) + ph[pos[:, 0]] + pw[pos[:, 1]] + pc[ch]
    torch.cuda.synchronize()
    assert (o2 - ref2).abs().max().item() <= 1e-4 * ref2.abs().max().item()


@pytest.fixture(scope="module")
def golden_model(pkg):
    d = np.load(os.path.join(HERE, "golden", "model_ref.npz"))
    w = {k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")}
    hid, heads, inter, layers, ncb, cbs, s = [int(v) for v in d["cfg"]]
    enc = dict(hidden_size=hid, intermediate_size=inter, num_attention_heads=heads, num_hidden_layers=layers)
    cfg = pkg.DCTAutoencoderConfig(image_channels=3, patch_size=14, max_patch_h=32, max_patch_w=32,
                                   vq_codebook_size=cbs, vq_num_codebooks=ncb, vq_type="lfq", encoder_config=enc,
                                   decoder_config=enc)
    m = pkg.DCTAutoencoder(cfg)
    m.load_state_dict(w, strict=False)
    m = m.to(DEV).eval()
    t = {k: torch.from_numpy(d[k]) for k in d.files if not k.startswith("w.")}
    return m, w, t, dict(heads=heads, layers=layers, ncb=ncb, cbd=int(np.log2(cbs)))


def _dp(pkg, t, patches):
    return pkg.DCTPatches(patches=patches, key_pad_mask=t["key_pad_mask"].to(DEV),
                          batched_image_ids=t["batched_image_ids"].to(DEV),
                          patch_channels=t["patch_channels"].to(DEV), patch_positions=t["patch_positions"].to(DEV),
                          patch_sizes=[], original_sizes=[])


def test_model_encode_codes_vs_reference(pkg, golden_model):
    """Encoder + LFQ on the reference's inputs: every code bit whose projected
    feature is clear of zero (|x| > 2 % of the feature scale, fp32 oracle)
    equals the reference's; the reported disagreement rate is small."""
    m, w, t, c = golden_model
    dp, codes, _, _ = m.encode(_dp(pkg, t, t["patches_in"].to(DEV)))
    torch.cuda.synchronize()
    codes = codes.cpu()
    args = (t["batched_image_ids"], t["key_pad_mask"], t["patch_channels"], t["patch_positions"])
    hid, _, _ = R.encode(w, t["patches_in"], *args, c["heads"], c["layers"], c["ncb"], c["cbd"])
    feat = F.linear(hid, w["vq_model.project_in.weight"], w["vq_model.project_in.bias"])
    feat = feat.view(*feat.shape[:-1], c["ncb"], c["cbd"])
    mask = 2 ** torch.arange(c["cbd"] - 1, -1, -1)
    bit_ours = (codes[..., None] & mask) != 0
    bit_ref = (t["codes"][..., None] & mask) != 0
    clear = feat.abs() > 0.02 * feat.abs().mean() * 4
    assert torch.equal(bit_ours[clear], bit_ref[clear])
    rate = (bit_ours != bit_ref).float().mean().item()
    print(f"code bits differing from the reference: {rate:.5f}")
    assert rate < 0.01


def test_model_decode_from_reference_codes(pkg, golden_model):
    """Decoder on the reference's codes (decode_from_codes): output within
    bf16 tolerance of the reference's decoded patches."""
    m, w, t, c = golden_model
    kw = dict(key_pad_mask=t["key_pad_mask"].to(DEV), batched_image_ids=t["batched_image_ids"].to(DEV),
              patch_channels=t["patch_channels"].to(DEV), patch_positions=t["patch_positions"].to(DEV),
              patch_sizes=[], original_sizes=[])
    out = m.decode_from_codes(t["codes"].to(DEV), **kw)
    torch.cuda.synchronize()
    got, ref = out.patches.cpu(), t["decoded"]
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    print(f"decoded max rel err {err:.4g}")
    assert err <= 3e-2


def test_model_forward_roundtrip_shapes(pkg, golden_model):
    m, w, t, c = golden_model
    out = m(_dp(pkg, t, t["patches_in"].to(DEV)))
    torch.cuda.synchronize()
    assert out["dct_patches"].patches.shape == t["decoded"].shape
    assert out["codes"].shape == t["codes"].shape and out["codes"].dtype == torch.long
    assert torch.isfinite(out["dct_patches"].patches).all()


def test_model_half_and_device_checks(pkg, golden_model):
    """The reference's loader casts the model to fp16 (factory.py:36-64,
    prepare_autoregressive_dataset.py): the kernels then get fp32 copies of
    the LayerNorm / position / bias operands, so the forward stays sane and
    its codes match the fp32 model's except near zero; a model left on the CPU
    is refused instead of handing host pointers to the kernels."""
    import copy
    m, w, t, c = golden_model
    mh = copy.deepcopy(m).half()
    ref_codes = m.encode(_dp(pkg, t, t["patches_in"].to(DEV)))[1]
    dp, codes, _, _ = mh.encode(_dp(pkg, t, t["patches_in"].to(DEV)))
    torch.cuda.synchronize()
    assert torch.isfinite(dp.patches.float()).all()
    mask = 2 ** torch.arange(c["cbd"] - 1, -1, -1, device=DEV)
    differ = (((codes[..., None] & mask) != 0) != ((ref_codes[..., None] & mask) != 0)).float().mean().item()
    assert differ < 0.02, differ
    cpu_model = copy.deepcopy(m).cpu()
    with pytest.raises(RuntimeError):
        cpu_model.encode(_dp(pkg, t, t["patches_in"].to(DEV)))
