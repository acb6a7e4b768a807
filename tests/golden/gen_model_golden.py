"""Golden vectors for the DCTAutoencoder transformer forward,
produced by running the reference's own modeling_dct_autoencoder.py (read-only
from /root/reference, loaded by refload.py) in THIS container.  BUILD-CONTAINER
ONLY: the GPU box has no /root/reference; the tests read model_ref.npz.

The reference pins transformers==4.35.2 (requirements.txt), whose CLIPAttention
ADDS the (b, 1, S, S) bool attn_mask of DCTPatches to the attention logits
(True -> +1.0; modeling:131-133 passes DCTPatches.attn_mask as
`attention_mask`).  This container has transformers 5.15, whose eager
attention (`eager_attention_forward`) does the same addition; its SDPA path
would treat the bool mask as a real mask, so the encoder / decoder configs are
forced to the eager implementation here.  That pins the 4.35.2 behaviour.

Small model (hidden 128, 2 heads of 64, 2 + 2 layers, LFQ 4 codebooks x 2^13 over a
128-wide feature: project_in / project_out active), random init (seed 0),
DCTPatches from the reference feature extractor on 4 synthetic images packed
into rows of S = 256, normalised by the reference-fitted PatchNorm tables.

    python tests/golden/gen_model_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import refload  # noqa: E402
from oracle import rng  # noqa: E402

CFG = dict(hidden=128, heads=2, inter=256, layers=2, ncb=4, cb_size=2 ** 13, S=256, patch=14, maxp=32)


def main():
    refload.load()
    import importlib
    m = importlib.import_module("dct_autoencoder.modeling_dct_autoencoder")
    cm = importlib.import_module("dct_autoencoder.configuration_dct_autoencoder")
    fe_mod = importlib.import_module("dct_autoencoder.feature_extraction_dct_autoencoder")
    torch.manual_seed(0)
    enc = dict(hidden_size=CFG["hidden"], intermediate_size=CFG["inter"], num_attention_heads=CFG["heads"],
               num_hidden_layers=CFG["layers"])
    cfg = cm.DCTAutoencoderConfig(image_channels=3, patch_size=CFG["patch"], max_patch_h=CFG["maxp"],
                                  max_patch_w=CFG["maxp"], vq_codebook_size=CFG["cb_size"],
                                  vq_num_codebooks=CFG["ncb"], vq_type="lfq", encoder_config=enc,
                                  decoder_config=enc)
    cfg.encoder_config._attn_implementation = "eager"
    cfg.decoder_config._attn_implementation = "eager"
    model = m.DCTAutoencoder(cfg).eval()
    # non-trivial LayerNorm affine parameters (init is 1 / 0)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if ("layer_norm" in name or "to_patch_embedding.1" in name or "proj_out.0" in name):
                p.add_(0.1 * torch.randn_like(p))
    assert model.encoder.layers[0].self_attn.config._attn_implementation == "eager"
    tabs = np.load(os.path.join(HERE, "patchnorm_ref.npz"))
    model.patchnorm.median.data.copy_(torch.from_numpy(tabs["median"]))
    model.patchnorm.b.data.copy_(torch.from_numpy(tabs["b"]))
    model.patchnorm.n.data.copy_(torch.from_numpy(tabs["n"]))
    model.patchnorm.frozen = True

    fe = fe_mod.DCTAutoencoderFeatureExtractor(channels=3, patch_size=CFG["patch"], sample_patches_beta=0.0,
                                               max_patch_h=CFG["maxp"], max_patch_w=CFG["maxp"],
                                               max_seq_len=CFG["S"])
    shapes = [(112, 112), (42, 70), (98, 140), (56, 84), (70, 70)]   # rows: 192+45, 210, 72+75 tokens
    imgs = [torch.from_numpy(x) for x in rng.synth_images(4242, shapes)]
    items = [fe.preprocess(x) for x in imgs]
    batch = {k: [it[k] for it in items] for k in items[0]}
    (dp,) = list(fe.iter_batches(iter([batch]), batch_size=None))
    with torch.no_grad():
        dp = model.normalize_(dp)
        patches_in = dp.patches.clone()
        out = model(dp)
        # encoder output before the quantiser, for tolerance bookkeeping
        dp2 = fe_mod.DCTPatches(**{k: getattr(out["dct_patches"], k) for k in
                                   ("key_pad_mask", "attn_mask", "batched_image_ids", "patch_channels",
                                    "patch_positions", "patch_sizes", "original_sizes")},
                                patches=patches_in.clone())
        x = model.to_patch_embedding(dp2.patches)
        dp2.patches = x
        dp2 = model.add_pos_embedding_encoder_(dp2)
        hidden = model.encoder(dp2.patches, attention_mask=dp2.attn_mask).last_hidden_state
    res = {"patches_in": patches_in.numpy(), "key_pad_mask": dp.key_pad_mask.numpy(),
           "batched_image_ids": dp.batched_image_ids.numpy(), "patch_channels": dp.patch_channels.numpy(),
           "patch_positions": dp.patch_positions.numpy(), "enc_hidden": hidden.numpy(),
           "codes": out["codes"].numpy(), "decoded": out["dct_patches"].patches.numpy()}
    for k, v in model.state_dict().items():
        if not k.startswith("patchnorm."):   # the tables are patchnorm_ref.npz
            res["w." + k] = v.numpy()
    res["cfg"] = np.array([CFG[k] for k in ("hidden", "heads", "inter", "layers", "ncb", "cb_size", "S")])
    np.savez_compressed(os.path.join(HERE, "model_ref.npz"), **res)
    print({k: v.shape for k, v in res.items() if not k.startswith("w.")})
    print("codes", out["codes"].dtype, "rows", dp.key_pad_mask.shape, "tokens", int((~dp.key_pad_mask).sum()))


if __name__ == "__main__":
    main()
