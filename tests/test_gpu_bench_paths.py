"""The bench's own pre-planned paths at the bench's full geometry (SURVEY §8(d)
config 3: 1024 x 512^2, one image per 3072-token row), through the C ABI.

* BatchEncoder (the timed encode of bench.py) -> BatchDecoder (the timed
  decode: codes -> LFQ.indices_to_codes -> PatchNorm.inverse_norm ->
  revert_patching -> IDCT -> RGB, FE:289-310, lfq.py:105-134,
  patchnorm.py:167-177) on all 1024 images;
* the decoder's images of sampled rows equal decode_batch (the general
  decode entry) of the same packed rows bit for bit;
* 2 of them equal the CPU oracle's decode of the same codes within
  1e-5 x image range (+2e-5 relative), the tolerance of north_star's
  round-trip bound;
* size-independent properties over all 1024 images: every pixel finite, and
  the decode is deterministic (a second call is bit-identical).
Run on an MI355X.
"""
import pytest
import torch

from oracle import ref_cpu

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = ref_cpu.FEConfig()


@pytest.fixture(scope="module")
def setup(pkg, ref_tables):
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    pn = pkg.PatchNorm(32, 32, 14, 3).to(DEV)
    pn.median.data.copy_(ref_tables.median)
    pn.b.data.copy_(ref_tables.b)
    pn.n.data.copy_(ref_tables.n)
    pn.frozen = True
    pn.eval()
    lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(DEV).eval()
    return ops, fe_mod, fe, pn, lfq


def test_batch_decoder_full_geometry(pkg, setup, ref_tables):
    ops, fe_mod, fe, pn, lfq = setup
    B, H = 1024, 512
    x = ops.synth_images(B, H, H, seed=1234, first_index=0, device=DEV)
    enc = fe_mod.BatchEncoder(fe, B, H, H, pn, lfq, device=DEV)
    packed = {k: v.clone() for k, v in enc(x).items()}
    del x
    dec = fe_mod.BatchDecoder(enc, pn, lfq)
    out = dec(packed).clone()
    ops.check_device_errors(out.device)
    assert out.shape == (B, 3, H, H)
    assert bool(torch.isfinite(out).all())
    again = dec(packed)
    assert torch.equal(again, out), "decode is not deterministic"
    del again

    # one image per packed row: BatchDecoder image n = row n
    rows = [0, 1, 377, 1023]
    sel = torch.tensor(rows, device=DEV)
    dp = pkg.DCTPatches(patches=torch.empty(len(rows), 3072, 0, device=DEV),
                        key_pad_mask=packed["key_pad_mask"][sel], batched_image_ids=packed["image_ids"][sel],
                        patch_channels=packed["channels"][sel], patch_positions=packed["positions"][sel],
                        patch_sizes=[(H // 14, H // 14)] * len(rows), original_sizes=[(H, H)] * len(rows))
    codes = packed["codes"][sel]
    sub = fe.decode_batch(dp, codes, pn, lfq)
    assert len(sub) == len(rows)
    for r, img in zip(rows, sub):
        assert torch.equal(img, out[r]), f"BatchDecoder row {r} != decode_batch"

    # oracle decode of two of them (codes -> +-1 -> inverse PatchNorm -> revert -> IDCT -> RGB)
    two = [0, 3]
    kp = dp.key_pad_mask.cpu()[two]
    pos = dp.patch_positions.cpu()[two]
    chs = dp.patch_channels.cpu()[two]
    y = ref_cpu.lfq_indices_to_codes(codes.cpu()[two], ref_cpu.LFQConfig())
    xin = ref_cpu.norm_inverse(ref_tables, y, chs, pos[..., 0], pos[..., 1])
    batch = ref_cpu.Batch(xin, kp, None, dp.batched_image_ids.cpu()[two], chs, pos, [(H // 14, H // 14)] * 2,
                          [(H, H)] * 2)
    refs = ref_cpu.postprocess(batch, CFG)
    for i, r in zip(two, refs):
        a = out[rows[i]].cpu()
        scale = max(1.0, float(r.abs().max()))
        d = (a - r).abs()
        assert bool(torch.all(d <= 1e-5 * scale + 2e-5 * r.abs())), (rows[i], float(d.max()), scale)
