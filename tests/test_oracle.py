"""Pin the CPU oracle (oracle/ref_cpu.py) against the golden vectors produced by
running the reference itself (tests/golden/gen_golden.py) and against an
independent float64 DCT (scipy).  CPU only."""
import json
import random

import numpy as np
import pytest
import scipy.fft
import torch

from conftest import golden
from oracle import ref_cpu, rng

CFG = ref_cpu.FEConfig()
META = json.load(open(__import__("conftest").GOLDEN + "/meta.json"))


def _items(seed, sizes, first=0, cfg=CFG):
    return [ref_cpu.preprocess(torch.from_numpy(x), cfg) for x in rng.synth_images(seed, sizes, first)]


def _tok_map(pos, ch):
    return {(int(c), int(p[0]), int(p[1])): i for i, (p, c) in enumerate(zip(pos, ch))}


def test_rng_is_uniform_and_deterministic():
    a = rng.synth_image(1234, 3, 20, 30)
    b = rng.synth_image(1234, 3, 20, 30)
    assert a.dtype == np.float32 and a.shape == (3, 20, 30)
    assert np.array_equal(a, b)
    assert 0.0 <= a.min() and a.max() < 1.0
    assert abs(a.mean() - 0.5) < 0.05
    assert not np.array_equal(a, rng.synth_image(1234, 4, 20, 30))


def test_color_matrices_match_reference_bits():
    g = golden("colors.npz")
    m = ref_cpu.color_matrices()
    for k in ("rgb2lms", "lms2rgb", "lms2ipt", "ipt2lms"):
        assert np.array_equal(m[k].numpy(), g[k]), k


@pytest.mark.parametrize("shape", [(14, 14), (30, 700), (224, 224), (100, 77), (512, 512)])
def test_dct2_matches_float64_dctn(shape):
    x = torch.from_numpy(rng.synth_image(3, 0, *shape))
    y = ref_cpu.dct2(x).double().numpy()
    ref = scipy.fft.dctn(x.double().numpy(), type=2, norm="ortho", axes=(-2, -1))
    err = np.abs(y - ref).max()
    assert err <= 2e-6 * max(1.0, np.abs(ref).max()), err
    back = ref_cpu.idct2(torch.from_numpy(ref.astype(np.float32))).double().numpy()
    assert np.abs(back - x.double().numpy()).max() < 1e-5


@pytest.mark.parametrize("case", ["sq224", "ragged", "real"])
def test_preprocess_matches_reference(case):
    g = golden(f"case_{case}.npz")
    if case == "real":
        r = golden("real_inputs.npz")
        imgs = [r[f"img{i}"].astype(np.float32) / 255.0 for i in range(len(r.files))]
    else:
        c = META[case]
        imgs = rng.synth_images(c["seed"], [tuple(s) for s in c["sizes"]], c["first"])
    for i, x in enumerate(imgs):
        it = ref_cpu.preprocess(torch.from_numpy(x), CFG)
        assert tuple(it["original_sizes"]) == tuple(g[f"img{i}_original_size"])
        assert tuple(it["patch_sizes"]) == tuple(g[f"img{i}_patch_size"])
        ref_pos, ref_ch = g[f"img{i}_positions"], g[f"img{i}_channels"]
        mine = _tok_map(it["positions"].numpy(), it["channels"].numpy())
        theirs = _tok_map(ref_pos, ref_ch)
        assert mine.keys() == theirs.keys()
        ref_patches = g[f"img{i}_patches"]
        mp = it["patches"].numpy()
        idx_m = np.array([mine[k] for k in theirs])
        idx_t = np.array([theirs[k] for k in theirs])
        np.testing.assert_allclose(mp[idx_m], ref_patches[idx_t], rtol=0, atol=1e-6 * np.abs(ref_patches).max())
        # the reference's order is non-increasing in the oracle's scores
        toks, pos, ch, scores = ref_cpu.patch_scores(
            ref_cpu.transform_image_in(torch.from_numpy(x))[:, : 14 * it["patch_sizes"][0], : 14 * it["patch_sizes"][1]], CFG)
        fmap = _tok_map(pos.numpy(), ch.numpy())
        s_ref_order = np.array([scores[fmap[(int(c), int(p[0]), int(p[1]))]].item() for p, c in zip(ref_pos, ref_ch)])
        assert np.all(np.diff(s_ref_order) <= 0)


def test_sq512_head_and_order():
    g = golden("case_sq512.npz")
    c = META["sq512"]
    x = rng.synth_images(c["seed"], [tuple(s) for s in c["sizes"]], c["first"])[0]
    it = ref_cpu.preprocess(torch.from_numpy(x), CFG)
    assert it["patches"].shape == (3072, 196)
    mine = _tok_map(it["positions"].numpy(), it["channels"].numpy())
    theirs = _tok_map(g["img0_positions"], g["img0_channels"])
    assert mine.keys() == theirs.keys()
    head = g["img0_patches_head"]
    for j in range(head.shape[0]):
        k = (int(g["img0_channels"][j]), int(g["img0_positions"][j][0]), int(g["img0_positions"][j][1]))
        np.testing.assert_allclose(it["patches"][mine[k]].numpy(), head[j], atol=1e-6 * np.abs(head).max())


def test_patchnorm_training_is_bit_exact(ref_tables):
    cal = [tuple(s) for s in META["patchnorm"]["cal_sizes"]]
    items = _items(99, cal)
    loader = [{k: [it[k] for it in items[i:i + 4]] for k in items[0]} for i in range(0, len(items), 4)]
    t = ref_cpu.NormTables.fresh()
    steps = 0
    for batch in ref_cpu.iter_batches(iter(loader), CFG, 4, build_attn_mask=False):
        t = ref_cpu.norm_train_step(t, batch.patches, batch.patch_channels, batch.h_indices, batch.w_indices,
                                    batch.key_pad_mask)
        steps += 1
    assert steps == META["patchnorm"]["steps"]
    assert torch.equal(t.n, ref_tables.n)
    # bit-exact given bit-identical DCT input on this host
    np.testing.assert_array_equal(t.median.numpy(), ref_tables.median.numpy())
    np.testing.assert_array_equal(t.b.numpy(), ref_tables.b.numpy())


@pytest.mark.parametrize("case", ["sq224", "ragged", "real"])
def test_norm_lfq_and_decode_match_reference(case, ref_tables):
    g = golden(f"case_{case}.npz")
    n_img = len([k for k in g.files if k.endswith("_positions") and k.startswith("img")])
    lcfg = ref_cpu.LFQConfig()
    # rebuild the reference's own batch from its stored tokens (identical fp32 inputs)
    items = [dict(patches=torch.from_numpy(g[f"img{i}_patches"]),
                  positions=torch.from_numpy(g[f"img{i}_positions"].astype(np.int64)),
                  channels=torch.from_numpy(g[f"img{i}_channels"].astype(np.int64)),
                  original_sizes=tuple(g[f"img{i}_original_size"]),
                  patch_sizes=tuple(g[f"img{i}_patch_size"])) for i in range(n_img)]
    loader = [{k: [it[k] for it in items] for k in items[0]}]
    (batch,) = list(ref_cpu.iter_batches(iter(loader), CFG, None, build_attn_mask=False))
    np.testing.assert_array_equal(batch.key_pad_mask.numpy(), g["key_pad_mask"])
    np.testing.assert_array_equal(batch.batched_image_ids.numpy(), g["batched_image_ids"])
    np.testing.assert_array_equal(batch.patch_positions.numpy(), g["patch_positions"])
    y = ref_cpu.norm_forward_eval(ref_tables, batch.patches, batch.patch_channels, batch.h_indices, batch.w_indices)
    q, idx = ref_cpu.lfq_forward(y, lcfg)
    np.testing.assert_array_equal(idx.numpy(), g["indices"])       # bit-exact codes, pads included
    batch.patches = ref_cpu.norm_inverse(ref_tables, ref_cpu.lfq_indices_to_codes(idx, lcfg),
                                         batch.patch_channels, batch.h_indices, batch.w_indices)
    dec = ref_cpu.postprocess(batch, CFG)
    for i in range(n_img):
        if f"img{i}_decoded_rgb" in g.files:
            r = g[f"img{i}_decoded_rgb"]
            np.testing.assert_allclose(dec[i].numpy(), r, rtol=1e-6, atol=1e-6)


def test_beta_sampling_reproduces_reference_k():
    g = golden("case_beta.npz")
    m = META["beta"]
    cfg = ref_cpu.FEConfig(sample_patches_beta=m["beta"], max_seq_len=m["max_seq_len"])
    random.seed(m["seed_python_random"])
    imgs = rng.synth_images(m["img_seed"], [tuple(s) for s in m["sizes"]])
    for i, x in enumerate(imgs):
        it = ref_cpu.preprocess(torch.from_numpy(x), cfg)
        assert it["patches"].shape[0] == int(g[f"img{i}_k"])
        # same selected set unless a score tie straddles the cut
        mine = set(_tok_map(it["positions"].numpy(), it["channels"].numpy()))
        theirs = set(_tok_map(g[f"img{i}_positions"], g[f"img{i}_channels"]))
        assert len(mine ^ theirs) <= 2


def test_iter_batches_quirks_match_reference():
    g = golden("case_packing.npz")
    m = META["packing"]
    cfg = ref_cpu.FEConfig(max_seq_len=m["max_seq_len"])
    items = _items(m["img_seed"], [tuple(s) for s in m["sizes"]], cfg=cfg)
    scenarios = {
        "one_item_none": ([items], None),
        "two_items_none": ([items[:4], items[4:]], None),
        "items_b2": ([items[:3], items[3:6], items[6:]], 2),
        "items_b1": ([items[:2], items[2:5], items[5:]], 1),
    }
    for name, (chunks, bs) in scenarios.items():
        loader = [{k: [it[k] for it in ch] for k in ch[0]} | {"tag": [f"t{j}" for j in range(len(ch))]}
                  for ch in chunks]
        got = list(ref_cpu.iter_batches(iter(loader), cfg, bs))
        assert len(got) == int(g[name + "_nbatches"]), name
        for bi, b in enumerate(got):
            pre = f"{name}_b{bi}_"
            np.testing.assert_array_equal(b.key_pad_mask.numpy(), g[pre + "key_pad_mask"])
            np.testing.assert_array_equal(b.batched_image_ids.numpy(), g[pre + "ids"])
            assert np.array_equal(np.array(b.original_sizes).reshape(-1, 2), g[pre + "original_sizes"])
            assert np.array_equal(np.array(b.patch_sizes).reshape(-1, 2), g[pre + "patch_sizes"])
            assert list(b._data.get("tag", [])) == list(g[pre + "data_tag"])
            # positions: equal as per-image sets (tie order may differ)
            for r in range(b.key_pad_mask.shape[0]):
                valid = ~b.key_pad_mask[r].numpy()
                ids = b.batched_image_ids[r].numpy()
                for im in np.unique(ids[valid]):
                    sel = valid & (ids == im)
                    a = _tok_map(b.patch_positions[r].numpy()[sel], b.patch_channels[r].numpy()[sel])
                    t = _tok_map(g[pre + "positions"][r][sel], g[pre + "channels"][r][sel])
                    assert a.keys() == t.keys()


def _vq_state():
    g = golden("vq_ref.npz")
    t = lambda k: torch.from_numpy(g[k])  # noqa: E731
    st = ref_cpu.VQState(t("w_in"), t("b_in"), t("w_out"), t("b_out"), t("embed"), t("codebook_mean"),
                         t("codebook_variance"), heads=int(g["heads"]))
    return g, st


def test_vq_oracle_matches_reference():
    """oracle.vq_forward_eval == the reference VectorQuantize (eval, model
    configuration) on two consecutive masked batches, including the batch
    affine statistics it carries between calls (vector_quantize.py:353-359)."""
    g, st = _vq_state()
    for step in range(2):
        x = torch.from_numpy(g[f"x{step}"])
        mask = torch.from_numpy(g[f"mask{step}"])
        q, ind, st, _ = ref_cpu.vq_forward_eval(st, x, mask)
        assert torch.equal(ind, torch.from_numpy(g[f"indices{step}"]))
        assert torch.allclose(q, torch.from_numpy(g[f"quantize{step}"]), atol=1e-6, rtol=1e-6)
        assert torch.allclose(st.batch_mean, torch.from_numpy(g[f"batch_mean{step}"]), atol=1e-7, rtol=1e-6)
        assert torch.allclose(st.batch_variance, torch.from_numpy(g[f"batch_variance{step}"]), atol=1e-7, rtol=1e-6)
    codes = ref_cpu.vq_codes_from_indices(st, torch.from_numpy(g["indices0"]))
    assert torch.equal(codes, torch.from_numpy(g["codes_from_indices0"]))


@pytest.mark.parametrize("proj", [False, True])
def test_lfq_scale_rule_matches_reference(proj):
    """lfq.py:174-187 at codebook_scale 1, 0.5, 0, -1, -0.25: the index bit is
    that of the QUANTIZED value (s < 0 inverts every bit, NaN inputs included;
    s == 0 gives 0).  Fixture: the reference's own LFQ (gen_lfq_scale_golden.py)."""
    import torch.nn.functional as F
    g = golden("lfq_scale_ref.npz")
    x = torch.from_numpy(g["x"])
    tag = "p" if proj else "n"
    for si, s in enumerate(g["scales"]):
        if proj:
            cfg = ref_cpu.LFQConfig(dim=196, codebook_size=2 ** 13, num_codebooks=16, codebook_scale=float(s))
            win, bin_ = torch.from_numpy(g["w_in"]), torch.from_numpy(g["b_in"])
            wout, bout = torch.from_numpy(g["w_out"]), torch.from_numpy(g["b_out"])
            q, idx = ref_cpu.lfq_forward(x, cfg, project_in=lambda t: F.linear(t, win, bin_),
                                         project_out=lambda t: F.linear(t, wout, bout))
            codes = ref_cpu.lfq_indices_to_codes(idx, cfg, project_out=lambda t: F.linear(t, wout, bout))
        else:
            cfg = ref_cpu.LFQConfig(codebook_scale=float(s))
            q, idx = ref_cpu.lfq_forward(x, cfg)
            codes = ref_cpu.lfq_indices_to_codes(idx, cfg)
        assert torch.equal(idx, torch.from_numpy(g[f"{tag}{si}_idx"])), s
        torch.testing.assert_close(q, torch.from_numpy(g[f"{tag}{si}_q"]), rtol=0, atol=0, equal_nan=True)
        torch.testing.assert_close(codes, torch.from_numpy(g[f"{tag}{si}_codes"]), rtol=0, atol=0)


@pytest.mark.parametrize("tag,dt", [("f16", torch.float16), ("bf16", torch.bfloat16)])
def test_low_precision_colour_matches_reference(tag, dt):
    """FE:135-141 on fp16 / bf16 inputs: rgb_to_ipt in the input dtype, then
    .float() + dct2 + cast back.  The oracle's IPT stage is bit-exact with the
    reference's; the spectrum equals it (same fp32 DCT restatement)."""
    g = golden("color_dtype_ref.npz")
    for i in range(2):
        x = torch.from_numpy(g[f"{tag}_{i}_x"]).to(dt)
        assert torch.equal(ref_cpu.rgb_to_ipt(x).float(), torch.from_numpy(g[f"{tag}_{i}_ipt"]))
        assert torch.equal(ref_cpu.transform_image_in(x).float(), torch.from_numpy(g[f"{tag}_{i}_spec"]))
