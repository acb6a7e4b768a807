"""CPU-only checks of the boundary and the host logic: libdctae.so loads and
exports every symbol include/dctae.h declares (no compute calls), the host
packing mirror reproduces the reference's iter_batches layouts, DCTPatches
API surface, to_dict/from_dict round trip."""
import json
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT, golden
from oracle import ref_cpu, rng


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "dctae.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(dctae_\w+)\(", src, re.M)))


def test_header_declares_entry_points():
    syms = _declared_symbols()
    for s in ["dctae_encode", "dctae_decode", "dctae_norm_forward", "dctae_norm_inverse", "dctae_lfq_forward",
              "dctae_lfq_indices_to_codes", "dctae_ctx_create", "dctae_last_error"]:
        assert s in syms


def test_library_loads_and_exports_every_symbol(pkg):
    lib = pkg.load_library()
    for s in _declared_symbols():
        assert hasattr(lib, s), s
    assert lib.dctae_abi_version() == 1


def test_no_gpu_means_loud_failure(pkg):
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
    with pytest.raises(pkg.DCTAEUnavailable):
        fe.preprocess(torch.rand(3, 28, 28))


def _pack_rows_oracle(items, cfg, chunks, bs):
    loader = [{k: [it[k] for it in ch] for k in ch[0]} for ch in chunks]
    return list(ref_cpu.iter_batches(iter(loader), cfg, bs, build_attn_mask=False))


@pytest.mark.parametrize("bs", [None, 1, 2, 3])
def test_packing_plans_match_oracle(pkg, bs):
    cfg = ref_cpu.FEConfig(max_seq_len=1024)
    sizes = [(224, 224), (100, 300), (512, 140), (64, 64), (300, 300), (28, 28), (150, 420), (90, 90), (14, 700)]
    ks = [min(ref_cpu.num_tokens(h, w, cfg), cfg.max_seq_len) for h, w in sizes]
    # fake items with the right k (tokens are irrelevant to the layout)
    items = [dict(patches=torch.zeros(k, 196), positions=torch.zeros(k, 2, dtype=torch.long),
                  channels=torch.zeros(k, dtype=torch.long), original_sizes=s, patch_sizes=s)
             for k, s in zip(ks, sizes)]
    chunks = [items[:3], items[3:6], items[6:]]
    ref = _pack_rows_oracle(items, cfg, chunks, bs)
    ids = list(range(len(items)))
    plans = list(pkg.packing.iter_batch_plans([(ks[0:3], ids[0:3]), (ks[3:6], ids[3:6]), (ks[6:], ids[6:])],
                                              1024, 3072, bs))
    assert len(plans) == len(ref)
    for rows, b in zip(plans, ref):
        plan = pkg.packing.layout(rows, dict(enumerate(ks)))
        assert plan.n_rows == b.key_pad_mask.shape[0]
        lens = (~b.key_pad_mask).sum(1).tolist()
        assert plan.row_len == lens
        for i, r, c, k, lid in zip(plan.images, plan.row, plan.col, plan.k, plan.local_id):
            assert torch.all(b.batched_image_ids[r, c:c + k] == lid)


def test_choose_k_reproduces_python_random(pkg):
    import random
    random.seed(3)
    a = [pkg.packing.choose_k(768, 0.02, 1024) for _ in range(20)]
    random.seed(3)
    cfg = ref_cpu.FEConfig(sample_patches_beta=0.02, max_seq_len=1024)
    b = [ref_cpu.choose_k(768, cfg) for _ in range(20)]
    assert a == b


def test_dct_patches_surface_and_lazy_attn_mask(pkg):
    ids = torch.tensor([[0, 0, 1, 1, 0], [0, 0, 0, 0, 0]])
    kp = torch.tensor([[False, False, False, False, True], [False, False, False, True, True]])
    dp = pkg.DCTPatches(patches=torch.zeros(2, 5, 196), key_pad_mask=kp, attn_mask=None, batched_image_ids=ids,
                        patch_channels=torch.zeros(2, 5, dtype=torch.long),
                        patch_positions=torch.zeros(2, 5, 2, dtype=torch.long), patch_sizes=[(1, 1)] * 3,
                        original_sizes=[(14, 14)] * 3)
    ref = (ids[:, None, :, None] == ids[:, None, None, :]) & kp[:, None, None, :]
    assert torch.equal(dp.attn_mask, ref)
    assert dp.h_indices.shape == (2, 5) and dp.w_indices.shape == (2, 5)
    c = dp.shallow_copy()
    assert c.patches is dp.patches
    assert dp.to("cpu") is dp


def test_to_dict_matches_reference_json(pkg):
    g = golden("case_ragged.npz")
    ref_objs = json.load(open(os.path.join(GOLDEN, "ragged_to_dict.json")))
    n_img = len(ref_objs)
    dp = pkg.DCTPatches(patches=torch.zeros(g["key_pad_mask"].shape + (196,)),
                        key_pad_mask=torch.from_numpy(g["key_pad_mask"]),
                        batched_image_ids=torch.from_numpy(g["batched_image_ids"].astype(np.int64)),
                        patch_channels=torch.from_numpy(g["patch_channels"].astype(np.int64)),
                        patch_positions=torch.from_numpy(g["patch_positions"].astype(np.int64)),
                        patch_sizes=[tuple(g[f"img{i}_patch_size"].tolist()) for i in range(n_img)],
                        original_sizes=[tuple(g[f"img{i}_original_size"].tolist()) for i in range(n_img)])
    objs = pkg.to_dict(dp, torch.from_numpy(g["indices"].astype(np.int64)))
    assert json.loads(json.dumps(objs)) == json.loads(json.dumps(ref_objs))
    dp1, codes = pkg.from_dict(ref_objs[1])
    assert codes.shape == (len(ref_objs[1]["codes"]), 14)
    assert dp1.patch_sizes == [ref_objs[1]["size"]]
