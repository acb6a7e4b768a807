"""DCTAutoencoder — drop-in for the reference's transformer autoencoder around
the LFQ bottleneck (dct_autoencoder/modeling_dct_autoencoder.py, with the
CLIPEncoder of transformers==4.35.2), inference on MI355X.

Same constructor (a ``DCTAutoencoderConfig``), parameter names / state-dict
keys (a reference checkpoint loads with ``load_state_dict``), and methods
``normalize_`` / ``inv_normalize_`` / ``encode`` / ``decode`` /
``decode_from_codes`` / ``forward`` / ``get_pos_embedding_decoder`` /
``add_pos_embedding_{en,de}coder_`` (modeling:86-200).  Every op of the
forward runs on libdctae's HIP kernels (dctae_model_*: bf16 MFMA linear
layers with fused bias / quick_gelu / residual epilogues, flash attention,
LayerNorm, LFQ codes); weights are kept as fp32 parameters and packed once
into bf16 device copies (K zero-padded to 64).  The residual stream and every
accumulation are fp32; the reference runs this model in fp16 / bf16 autocast
(main.py:331-347, prepare_autoregressive_dataset.py:21).

Attention reproduces the reference exactly as 4.35.2 executes it: the bool
``DCTPatches.attn_mask`` is ADDED to the logits (+1.0 where the query's image
id equals the key's and the key is padding, FE:580-584) and nothing is masked
(modeling:131-133 passes it as ``attention_mask``).  A caller-assigned
``attn_mask`` tensor is not consulted: the kernel derives the mask from
``batched_image_ids`` / ``key_pad_mask``, which is how the feature extractor
defines it.

Training (losses, backward, the VectorQuantize variant's codebook updates) is
not on the MI355X path: ``encode`` / ``decode`` in training mode raise
NotImplementedError.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Optional

import torch
from torch import nn

from . import _lib
from .dct_patches import DCTPatches
from .lfq import LFQ
from .patchnorm import PatchNorm


def _f32(t: torch.Tensor) -> torch.Tensor:
    """fp32 contiguous view / copy of a parameter for a kernel's float* operand."""
    return t.detach().float().contiguous()

LIN_F32, LIN_BF16, LIN_BF16_QGELU, LIN_F32_RESIDUAL = 0, 1, 2, 3


@dataclass
class CLIPEncoderConfig:
    """The CLIPVisionConfig fields the encoder reads (transformers 4.35.2 defaults)."""
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_attention_heads: int = 12
    num_hidden_layers: int = 12
    layer_norm_eps: float = 1e-5
    hidden_act: str = "quick_gelu"
    attention_dropout: float = 0.0
    dropout: float = 0.0

    @classmethod
    def from_any(cls, c):
        if isinstance(c, cls):
            return c
        if c is None:
            return cls()
        if not isinstance(c, dict):
            c = {k: getattr(c, k) for k in cls.__dataclass_fields__ if hasattr(c, k)}
        return cls(**{k: v for k, v in c.items() if k in cls.__dataclass_fields__})


class DCTAutoencoderConfig:
    """configuration_dct_autoencoder.py:5-41: same argument names and defaults;
    sub-configs may be dicts or CLIPVisionConfig-like objects, extra keys
    (e.g. ``transformers_version`` of a saved config.json) are kept as attributes."""

    def __init__(self, image_channels: int = 3, patch_size: int = 16, max_patch_h: int = 32, max_patch_w: int = 32,
                 vq_codebook_size: int = 4096, vq_num_codebooks: int = 8, vq_type: str = "lfq",
                 encoder_config=None, decoder_config=None, **kwargs):
        self.image_channels = image_channels
        self.patch_size = patch_size
        self.max_patch_h = max_patch_h
        self.max_patch_w = max_patch_w
        self.vq_codebook_size = vq_codebook_size
        self.vq_num_codebooks = vq_num_codebooks
        self.vq_type = vq_type
        self.encoder_config = CLIPEncoderConfig.from_any(encoder_config)
        self.decoder_config = CLIPEncoderConfig.from_any(decoder_config)
        for k, v in kwargs.items():
            setattr(self, k, v)


class _Attention(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.k_proj, self.v_proj, self.q_proj, self.out_proj = (nn.Linear(d, d) for _ in range(4))


class _MLP(nn.Module):
    def __init__(self, d, i):
        super().__init__()
        self.fc1 = nn.Linear(d, i)
        self.fc2 = nn.Linear(i, d)


class _Layer(nn.Module):
    def __init__(self, c: CLIPEncoderConfig):
        super().__init__()
        self.self_attn = _Attention(c.hidden_size)
        self.layer_norm1 = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.mlp = _MLP(c.hidden_size, c.intermediate_size)
        self.layer_norm2 = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)


class CLIPEncoder(nn.Module):
    """Parameter container with transformers' CLIPEncoder names (layers.N.*)."""

    def __init__(self, c: CLIPEncoderConfig):
        super().__init__()
        if c.hidden_act != "quick_gelu":
            raise NotImplementedError(f"hidden_act={c.hidden_act!r}: the fused MLP epilogue is quick_gelu")
        if c.hidden_size % c.num_attention_heads or c.hidden_size // c.num_attention_heads != 64:
            raise NotImplementedError("head_dim must be 64 (the attention kernel's tile)")
        self.config = c
        self.layers = nn.ModuleList([_Layer(c) for _ in range(c.num_hidden_layers)])


def _pad64(k: int) -> int:
    return (k + 63) // 64 * 64


def _bf16_padded(w: torch.Tensor, kp: int) -> torch.Tensor:
    """(N, K) fp32 weight -> (N, kp) bf16 bit patterns, zero columns K .. kp."""
    out = torch.zeros(w.shape[0], kp, dtype=torch.bfloat16, device=w.device)
    out[:, :w.shape[1]] = w.detach().to(torch.bfloat16)
    return out.view(torch.int16)


class _Packed:
    """bf16 device copies of the linear weights, built once per parameter version."""

    def __init__(self, model: "DCTAutoencoder"):
        self.w: Dict[str, torch.Tensor] = {}
        self.b: Dict[str, Optional[torch.Tensor]] = {}
        for side in ("encoder", "decoder"):
            for i, L in enumerate(getattr(model, side).layers):
                a = L.self_attn
                self._put(f"{side}.{i}.qkv", torch.cat([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight], 0),
                          torch.cat([a.q_proj.bias, a.k_proj.bias, a.v_proj.bias], 0))
                self._put(f"{side}.{i}.out", a.out_proj.weight, a.out_proj.bias)
                self._put(f"{side}.{i}.fc1", L.mlp.fc1.weight, L.mlp.fc1.bias)
                self._put(f"{side}.{i}.fc2", L.mlp.fc2.weight, L.mlp.fc2.bias)
        self._put("embed", model.to_patch_embedding[0].weight, None)
        vq = model.vq_model
        if vq.has_projections:
            self._put("proj_in", vq.project_in.weight, vq.project_in.bias)
            self._put("proj_out_vq", vq.project_out.weight, vq.project_out.bias)
        self._put("proj_out", model.proj_out[1].weight, None)

    def _put(self, name, w, b):
        self.w[name] = _bf16_padded(w, _pad64(w.shape[1]))
        self.b[name] = b.detach().float().contiguous() if b is not None else None


class DCTAutoencoder(nn.Module):
    def __init__(self, config: DCTAutoencoderConfig):
        super().__init__()
        if not isinstance(config, DCTAutoencoderConfig):
            keys = ("image_channels", "patch_size", "max_patch_h", "max_patch_w", "vq_codebook_size",
                    "vq_num_codebooks", "vq_type", "encoder_config", "decoder_config")
            config = DCTAutoencoderConfig(**{k: getattr(config, k) for k in keys if hasattr(config, k)})
        self.config = config
        d = config.encoder_config.hidden_size
        if config.decoder_config.hidden_size != d:
            raise ValueError("encoder and decoder hidden_size differ")
        self.patchnorm = PatchNorm(max_patch_h=config.max_patch_h, max_patch_w=config.max_patch_w,
                                   patch_size=config.patch_size, channels=config.image_channels)
        pd = config.patch_size ** 2
        c_, h_, w_ = config.image_channels, config.max_patch_h, config.max_patch_w
        self.encoder_pos_embed_channel = nn.Parameter(torch.randn(c_, d))
        self.encoder_pos_embed_height = nn.Parameter(torch.randn(h_, d))
        self.encoder_pos_embed_width = nn.Parameter(torch.randn(w_, d))
        self.decoder_pos_embed_channel = nn.Parameter(torch.randn(c_, d))
        self.decoder_pos_embed_height = nn.Parameter(torch.randn(h_, d))
        self.decoder_pos_embed_width = nn.Parameter(torch.randn(w_, d))
        self.to_patch_embedding = nn.Sequential(nn.Linear(pd, d, bias=False), nn.LayerNorm(d, eps=1e-4))
        self.encoder = CLIPEncoder(config.encoder_config)
        if config.vq_type == "lfq":
            self.vq_model = LFQ(dim=d, num_codebooks=config.vq_num_codebooks, codebook_size=config.vq_codebook_size)
        elif config.vq_type == "vq":
            raise NotImplementedError("vq_type='vq' autoencoder: use the VectorQuantize module directly")
        else:
            raise ValueError(config.vq_type)
        self.decoder = CLIPEncoder(config.decoder_config)
        self.proj_out = nn.Sequential(nn.LayerNorm(d, eps=1e-4), nn.Linear(d, pd, bias=False))
        self._packed: Optional[_Packed] = None
        self._packed_key = None

    # ---- reference helpers (modeling:86-117) ----
    def get_pos_embedding_decoder(self, dct_patches: DCTPatches):
        return (self.decoder_pos_embed_height[dct_patches.h_indices]
                + self.decoder_pos_embed_width[dct_patches.w_indices]
                + self.decoder_pos_embed_channel[dct_patches.patch_channels])

    def add_pos_embedding_decoder_(self, dct_patches: DCTPatches):
        x = dct_patches.patches.float().contiguous().clone()
        self._pos_add(x, "decoder", dct_patches)
        dct_patches.patches = x
        return dct_patches

    def add_pos_embedding_encoder_(self, dct_patches: DCTPatches):
        x = dct_patches.patches.float().contiguous().clone()
        self._pos_add(x, "encoder", dct_patches)
        dct_patches.patches = x
        return dct_patches

    @torch.no_grad()
    def normalize_(self, x: DCTPatches):
        x.patches = self.patchnorm(x)
        return x

    def inv_normalize_(self, x: DCTPatches):
        x.patches = self.patchnorm.inverse_norm(x)
        return x

    # ---- plumbing ----
    @staticmethod
    def _ctx(t):
        return _lib.context(t.device)

    def _weights(self) -> _Packed:
        key = tuple((p.data_ptr(), p._version) for p in self.parameters())
        if self._packed is None or self._packed_key != key:
            self._packed = _Packed(self)
            self._packed_key = key
        return self._packed

    def _check_mode(self, dp: Optional[DCTPatches] = None):
        if self.training:
            raise NotImplementedError("DCTAutoencoder training (losses, backward) is not on the MI355X path: "
                                      "call .eval()")
        if dp is not None:
            dev = dp.patches.device
            # kernels take raw device pointers: a parameter left on another device (or the
            # CPU) would be read as garbage, so refuse it like torch's device mismatch error
            for n, p in self.named_parameters():
                if p.device != dev:
                    raise RuntimeError(f"parameter {n} is on {p.device}, the input on {dev}: move the model with .to()")

    @staticmethod
    def _linear(ctx, x, w, bias, n, epi, out):
        m, kx = x.shape
        rows, kw = w.shape
        ctx.check(ctx.lib.dctae_model_linear(ctx.h, m, n, kw, _lib.ptr(x), kx, _lib.ptr(w), rows, kw, _lib.ptr(bias),
                                             epi, _lib.ptr(out), out.shape[1], _lib.stream_ptr(x.device)),
                  "model_linear")
        return out

    def _pos_tables(self, side):
        return [getattr(self, f"{side}_pos_embed_{k}").detach().float().contiguous()
                for k in ("height", "width", "channel")]

    @staticmethod
    def _meta(dp: DCTPatches):
        return (dp.patch_channels.reshape(-1).long().contiguous(),
                dp.patch_positions.reshape(-1, 2).long().contiguous())

    def _pos_add(self, x, side, dp):
        ctx = self._ctx(x)
        d = x.shape[-1]
        ch, pos = self._meta(dp)
        tabs = self._pos_tables(side)
        ctx.check(ctx.lib.dctae_model_pos_add(ctx.h, x.numel() // d, d, _lib.ptr(x), d, *[_lib.ptr(t) for t in tabs],
                                              _lib.ptr(ch), _lib.ptr(pos), _lib.stream_ptr(x.device)), "model_pos_add")

    @staticmethod
    def _layernorm(ctx, h, ln, out):
        m, d = h.shape
        g, b = _f32(ln.weight), _f32(ln.bias)   # fp32 copies when the model was cast (e.g. .half())
        ctx.check(ctx.lib.dctae_model_layernorm(ctx.h, m, d, _lib.ptr(h), d, _lib.ptr(g), _lib.ptr(b),
                                                C.c_float(ln.eps), _lib.ptr(out), out.shape[1],
                                                _lib.stream_ptr(h.device)), "layer_norm")
        return out

    def _clip(self, side: str, h: torch.Tensor, dp: DCTPatches):
        """CLIPEncoder.forward (transformers 4.35.2 CLIPEncoderLayer) on the f32
        residual stream h (M, D), in place."""
        ctx = self._ctx(h)
        pk = self._weights()
        enc = getattr(self, side)
        c = enc.config
        r, s = dp.key_pad_mask.shape
        m, d = h.shape
        dev = h.device
        st = _lib.stream_ptr(dev)
        ids = dp.batched_image_ids.long().contiguous()
        kp = dp.key_pad_mask.to(torch.uint8).contiguous()
        a = torch.empty(m, d, dtype=torch.int16, device=dev)
        qkv = torch.empty(m, 3 * d, dtype=torch.int16, device=dev)
        o = torch.empty(m, d, dtype=torch.int16, device=dev)
        f = torch.zeros(m, _pad64(c.intermediate_size), dtype=torch.int16, device=dev)
        for i, L in enumerate(enc.layers):
            self._layernorm(ctx, h, L.layer_norm1, a)
            self._linear(ctx, a, pk.w[f"{side}.{i}.qkv"], pk.b[f"{side}.{i}.qkv"], 3 * d, LIN_BF16, qkv)
            ctx.check(ctx.lib.dctae_model_attention(ctx.h, r, s, c.num_attention_heads, 64, _lib.ptr(qkv),
                                                    _lib.ptr(ids), _lib.ptr(kp), _lib.ptr(o), d, st), "self_attn")
            self._linear(ctx, o, pk.w[f"{side}.{i}.out"], pk.b[f"{side}.{i}.out"], d, LIN_F32_RESIDUAL, h)
            self._layernorm(ctx, h, L.layer_norm2, a)
            self._linear(ctx, a, pk.w[f"{side}.{i}.fc1"], pk.b[f"{side}.{i}.fc1"], c.intermediate_size,
                         LIN_BF16_QGELU, f)
            self._linear(ctx, f, pk.w[f"{side}.{i}.fc2"], pk.b[f"{side}.{i}.fc2"], d, LIN_F32_RESIDUAL, h)
        return h

    def _bf16(self, x: torch.Tensor, kp: int) -> torch.Tensor:
        ctx = self._ctx(x)
        m, k = x.shape
        out = torch.empty(m, kp, dtype=torch.int16, device=x.device)
        ctx.check(ctx.lib.dctae_model_to_bf16(ctx.h, m, k, _lib.ptr(x), x.stride(0), kp, _lib.ptr(out),
                                              _lib.stream_ptr(x.device)), "to_bf16")
        return out

    # ---- modeling:119-200 ----
    @torch.no_grad()
    def encode(self, dct_patches: DCTPatches, do_normalize: bool = False):
        self._check_mode(dct_patches)
        if do_normalize:
            dct_patches = self.normalize_(dct_patches)
        pk = self._weights()
        x = dct_patches.patches
        r, s, pd = x.shape
        d = self.config.encoder_config.hidden_size
        dev = x.device
        ctx = self._ctx(x)
        xb = self._bf16(x.reshape(r * s, pd).float().contiguous(), pk.w["embed"].shape[1])
        e = self._linear(ctx, xb, pk.w["embed"], None, d, LIN_F32, torch.empty(r * s, d, device=dev))
        h = torch.empty(r * s, d, device=dev)
        ln = self.to_patch_embedding[1]
        ch, pos = self._meta(dct_patches)
        tabs = self._pos_tables("encoder")
        g, b = _f32(ln.weight), _f32(ln.bias)
        ctx.check(ctx.lib.dctae_model_embed_norm(ctx.h, r * s, d, _lib.ptr(e), d, _lib.ptr(g),
                                                 _lib.ptr(b), C.c_float(ln.eps), *[_lib.ptr(t) for t in tabs],
                                                 _lib.ptr(ch), _lib.ptr(pos), _lib.ptr(h), d, _lib.stream_ptr(dev)),
                  "to_patch_embedding")
        self._clip("encoder", h, dct_patches)
        xq, codes = self._lfq(h)
        dct_patches.patches = xq.view(r, s, d)
        zero = torch.zeros((), device=dev)
        return dct_patches, codes.view(r, s, -1), zero, zero

    def _lfq(self, h: torch.Tensor):
        """LFQ.forward eval (lfq.py:136-227) on (M, D) f32 features."""
        vq = self.vq_model
        pk = self._weights()
        ctx = self._ctx(h)
        m, d = h.shape
        dev = h.device
        st = _lib.stream_ptr(dev)
        ncb, cbd = vq.num_codebooks, vq.codebook_dim
        codes = torch.empty(m, ncb, dtype=torch.long, device=dev)
        if vq.has_projections:
            hb = self._bf16(h, pk.w["proj_in"].shape[1])
            p = self._linear(ctx, hb, pk.w["proj_in"], pk.b["proj_in"], ncb * cbd, LIN_F32,
                             torch.empty(m, ncb * cbd, device=dev))
            kq = pk.w["proj_out_vq"].shape[1]
            q = torch.empty(m, kq, dtype=torch.int16, device=dev)
            ctx.check(ctx.lib.dctae_model_lfq(ctx.h, m, ncb, cbd, C.c_float(vq.codebook_scale), _lib.ptr(p),
                                              ncb * cbd, _lib.ptr(codes), _lib.ptr(q), None, kq, st), "lfq")
            xq = self._linear(ctx, q, pk.w["proj_out_vq"], pk.b["proj_out_vq"], d, LIN_F32,
                              torch.empty(m, d, device=dev))
        else:
            xq = torch.empty(m, d, device=dev)
            ctx.check(ctx.lib.dctae_model_lfq(ctx.h, m, ncb, cbd, C.c_float(vq.codebook_scale), _lib.ptr(h), d,
                                              _lib.ptr(codes), None, _lib.ptr(xq), d, st), "lfq")
        return xq, codes

    @torch.no_grad()
    def decode_from_codes(self, codes: torch.LongTensor, do_inv_norm: bool = False, **dct_patches_kwargs) -> DCTPatches:
        """modeling:149-158: LFQ.indices_to_codes (HIP kernel) + project_out (bf16 MFMA linear)."""
        vq = self.vq_model
        q = vq.indices_to_codes(codes, project_out=False)
        if vq.has_projections:
            pk = self._weights()
            lead = q.shape[:-1]
            qm = q.reshape(-1, q.shape[-1]).float().contiguous()
            ctx = self._ctx(qm)
            qb = self._bf16(qm, pk.w["proj_out_vq"].shape[1])
            q = self._linear(ctx, qb, pk.w["proj_out_vq"], pk.b["proj_out_vq"], vq.dim, LIN_F32,
                             torch.empty(qm.shape[0], vq.dim, device=qm.device)).view(*lead, vq.dim)
        x = DCTPatches(patches=q, **dct_patches_kwargs)
        return self.decode(x, do_inv_norm=do_inv_norm)

    @torch.no_grad()
    def decode(self, x: DCTPatches, do_inv_norm: bool = False) -> DCTPatches:
        self._check_mode(x)
        pk = self._weights()
        r, s, d = x.patches.shape
        dev = x.patches.device
        ctx = self._ctx(x.patches)
        x = self.add_pos_embedding_decoder_(x)
        h = x.patches.view(r * s, d)
        self._clip("decoder", h, x)
        a = self._layernorm(ctx, h, self.proj_out[0], torch.empty(r * s, d, dtype=torch.int16, device=dev))
        pd = self.proj_out[1].weight.shape[0]
        y = self._linear(ctx, a, pk.w["proj_out"], None, pd, LIN_F32, torch.empty(r * s, pd, device=dev))
        x.patches = y.view(r, s, pd)
        if do_inv_norm:
            x = self.inv_normalize_(x)
        return x

    @torch.no_grad()
    def forward(self, dct_patches: DCTPatches, do_normalize: bool = False):
        dct_patches, codes, commit_loss, distances = self.encode(dct_patches, do_normalize=do_normalize)
        dct_patches = self.decode(dct_patches)
        return dict(dct_patches=dct_patches, commit_loss=commit_loss, codes=codes, distances=distances)
