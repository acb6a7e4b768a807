"""TEST INFRASTRUCTURE ONLY — CPU fp32 restatement of the reference's
DCTAutoencoder forward (dct_autoencoder/modeling_dct_autoencoder.py) with the
CLIPEncoder of transformers==4.35.2 (reference requirements.txt) that it wraps.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product path (dct_autoencoder_amd.model) never does.

Pinned against tests/golden/model_ref.npz, produced by running the reference's
own model in the build container (tests/golden/gen_model_golden.py).

Semantics restated (reference file:line, `M` = modeling_dct_autoencoder.py):
  * to_patch_embedding = Linear(P*P -> D, no bias) + LayerNorm(D, eps=1e-4)   M:57-60
  * encoder position embedding: + pos_c[c] + pos_h[h] + pos_w[w]             M:98-108
  * CLIPEncoder layers (transformers 4.35.2 CLIPEncoderLayer):
        h = h + out_proj(attn(LN1(h)));  h = h + fc2(quick_gelu(fc1(LN2(h))))
    attention logits = (q k^T) / sqrt(d_head) + attn_mask, where attn_mask is
    DCTPatches.attn_mask, a BOOL (b, 1, S, S) tensor = (id_i == id_j) &
    key_pad_mask_j (FE:580-584) that 4.35.2 ADDS (True -> +1.0): no entry is
    masked out (M:131-133, "TODO Should be ~ attn mask?").  LayerNorm eps 1e-5,
    quick_gelu(x) = x * sigmoid(1.702 x) (CLIPVisionConfig defaults).
  * LFQ (lfq.py:136-227, eval): project_in, sign -> +-1, indices MSB-first per
    codebook, project_out                                                     M:137-144
  * decode: + decoder position embedding, CLIPEncoder, LayerNorm(eps=1e-4),
    Linear(D -> P*P, no bias)                                                 M:152-185
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

W = Dict[str, torch.Tensor]


def attn_bias(ids: torch.Tensor, key_pad: torch.Tensor) -> torch.Tensor:
    """(b, 1, S, S) float: the bool attn_mask (FE:580-584) as 4.35.2 adds it."""
    m = (ids[:, None, :, None] == ids[:, None, None, :]) & key_pad[:, None, None, :]
    return m.float()


def clip_layer(h: torch.Tensor, w: W, pre: str, bias: torch.Tensor, heads: int, eps: float = 1e-5) -> torch.Tensor:
    b, s, d = h.shape
    dh = d // heads
    x = F.layer_norm(h, (d,), w[pre + "layer_norm1.weight"], w[pre + "layer_norm1.bias"], eps)

    def proj(name, t):
        return F.linear(t, w[pre + f"self_attn.{name}.weight"], w[pre + f"self_attn.{name}.bias"])

    q = proj("q_proj", x).view(b, s, heads, dh).transpose(1, 2)
    k = proj("k_proj", x).view(b, s, heads, dh).transpose(1, 2)
    v = proj("v_proj", x).view(b, s, heads, dh).transpose(1, 2)
    logits = (q @ k.transpose(-1, -2)) * dh ** -0.5 + bias
    o = torch.softmax(logits, dim=-1) @ v
    o = o.transpose(1, 2).reshape(b, s, d)
    h = h + proj("out_proj", o)
    x = F.layer_norm(h, (d,), w[pre + "layer_norm2.weight"], w[pre + "layer_norm2.bias"], eps)
    x = F.linear(x, w[pre + "mlp.fc1.weight"], w[pre + "mlp.fc1.bias"])
    x = x * torch.sigmoid(1.702 * x)
    return h + F.linear(x, w[pre + "mlp.fc2.weight"], w[pre + "mlp.fc2.bias"])


def clip_encoder(h, w: W, pre: str, bias, heads: int, layers: int):
    for i in range(layers):
        h = clip_layer(h, w, f"{pre}layers.{i}.", bias, heads)
    return h


def pos_embed(w: W, side: str, ch, pos):
    return (w[f"{side}_pos_embed_height"][pos[..., 0]] + w[f"{side}_pos_embed_width"][pos[..., 1]]
            + w[f"{side}_pos_embed_channel"][ch])


def lfq(x: torch.Tensor, w: W, ncb: int, cb_dim: int):
    if "vq_model.project_in.weight" in w:
        x = F.linear(x, w["vq_model.project_in.weight"], w["vq_model.project_in.bias"])
    x = x.view(*x.shape[:-1], ncb, cb_dim)
    q = torch.where(x > 0, torch.ones_like(x), -torch.ones_like(x))
    mask = 2 ** torch.arange(cb_dim - 1, -1, -1)
    idx = ((x > 0).long() * mask).sum(-1)
    q = q.reshape(*q.shape[:-2], ncb * cb_dim)
    if "vq_model.project_out.weight" in w:
        q = F.linear(q, w["vq_model.project_out.weight"], w["vq_model.project_out.bias"])
    return q, idx


def encode(w: W, patches, ids, key_pad, ch, pos, heads: int, layers: int, ncb: int, cb_dim: int):
    """modeling:119-147 (do_normalize=False): returns (hidden, x_q, codes)."""
    d = w["to_patch_embedding.0.weight"].shape[0]
    x = F.linear(patches, w["to_patch_embedding.0.weight"])
    x = F.layer_norm(x, (d,), w["to_patch_embedding.1.weight"], w["to_patch_embedding.1.bias"], 1e-4)
    x = x + pos_embed(w, "encoder", ch, pos)
    hidden = clip_encoder(x, w, "encoder.", attn_bias(ids, key_pad), heads, layers)
    xq, codes = lfq(hidden, w, ncb, cb_dim)
    return hidden, xq, codes


def decode(w: W, x, ids, key_pad, ch, pos, heads: int, layers: int):
    """modeling:160-172 (do_inv_norm=False): patches (b, S, P*P)."""
    d = x.shape[-1]
    x = x + pos_embed(w, "decoder", ch, pos)
    x = clip_encoder(x, w, "decoder.", attn_bias(ids, key_pad), heads, layers)
    x = F.layer_norm(x, (d,), w["proj_out.0.weight"], w["proj_out.0.bias"], 1e-4)
    return F.linear(x, w["proj_out.1.weight"])


def codes_to_features(w: W, codes, ncb: int, cb_dim: int):
    """LFQ.indices_to_codes (lfq.py:105-134) with project_out (decode_from_codes, modeling:149-158)."""
    mask = 2 ** torch.arange(cb_dim - 1, -1, -1)
    bits = ((codes[..., None] & mask) != 0).float()
    q = (bits * 2 - 1).reshape(*codes.shape[:-1], ncb * cb_dim)
    if "vq_model.project_out.weight" in w:
        q = F.linear(q, w["vq_model.project_out.weight"], w["vq_model.project_out.bias"])
    return q
