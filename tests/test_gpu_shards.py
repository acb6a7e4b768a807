"""GPU preprocessed-shard writer (preproc_dataset.py:59-84):
tokens from the HIP feature path -> shards -> reader -> iter_batches gives the
same batches as feeding preprocess() directly (bit-exact: the same kernels
produced both), and the tokens match the CPU oracle's preprocess."""
import pytest
import torch

from oracle import ref_cpu, rng

pytestmark = pytest.mark.gpu
SIZES = [(224, 224), (100, 100), (30, 700), (300, 500), (512, 512), (57, 91), (224, 224)]


def test_write_read_iter_batches(pkg, tmp_path):
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    imgs = [torch.from_numpy(a) for a in rng.synth_images(1234, SIZES)]
    names = pkg.shards.write_preprocessed(fe, (im.cuda() for im in imgs), str(tmp_path), batch=3)
    assert len(names) == 1
    back = list(pkg.shards.load_preprocessed_dataset(str(tmp_path)))
    direct = fe.preprocess_many([im.cuda() for im in imgs])
    assert len(back) == len(SIZES)
    for i, (b, d) in enumerate(zip(back, direct)):
        assert torch.equal(b["patches"], d["patches"].cpu())
        assert torch.equal(b["positions"], d["positions"].cpu())
        assert torch.equal(b["channels"], d["channels"].cpu())
        assert b["original_sizes"] == SIZES[i]
        assert b["patch_sizes"] == (SIZES[i][0] // 14, SIZES[i][1] // 14)
        # the oracle's tokens, matched by (channel, h, w) (the order may swap at score
        # near-ties: test_gpu_parity.test_preprocess_tokens_and_order), DCT tolerance
        o = ref_cpu.preprocess(imgs[i], ref_cpu.FEConfig())
        omap = {(c, h, w): j for j, ((h, w), c) in enumerate(zip(o["positions"].tolist(), o["channels"].tolist()))}
        idx = torch.tensor([omap[(c, h, w)] for (h, w), c in zip(b["positions"].tolist(), b["channels"].tolist())])
        assert len(set(idx.tolist())) == len(idx) == o["patches"].shape[0]
        tol = 2e-6 * float(o["patches"].abs().max())
        assert float((b["patches"] - o["patches"][idx]).abs().max()) <= tol
    # the reader's dicts feed iter_batches exactly like preprocess()'s
    a = list(fe.iter_batches(pkg.shards.batched(iter(back), 3), 2))
    b = list(fe.iter_batches(pkg.shards.batched(iter(direct), 3), 2))
    assert len(a) == len(b) > 0
    for x, y in zip(a, b):
        assert torch.equal(x.patches.cpu(), y.patches.cpu())
        assert torch.equal(x.key_pad_mask.cpu(), y.key_pad_mask.cpu())
        assert torch.equal(x.batched_image_ids.cpu(), y.batched_image_ids.cpu())
        assert x.original_sizes == y.original_sizes and x.patch_sizes == y.patch_sizes


def test_write_fp16(pkg, tmp_path):
    """preproc_dataset.py's dtype argument (float16 tokens on disk)."""
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    imgs = [torch.from_numpy(a).cuda() for a in rng.synth_images(5, [(224, 224), (140, 98)])]
    pkg.shards.write_preprocessed(fe, iter(imgs), str(tmp_path), dtype=torch.float16)
    back = list(pkg.shards.load_preprocessed_dataset(str(tmp_path)))
    direct = fe.preprocess_many(imgs)
    for b, d in zip(back, direct):
        assert b["patches"].dtype == torch.float16
        assert torch.equal(b["patches"], d["patches"].half().cpu())
