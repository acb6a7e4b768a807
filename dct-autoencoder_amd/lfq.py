"""LFQ — drop-in for the reference's lookup-free quantizer (dct_autoencoder/lfq.py:35-227).

Same constructor arguments, buffers (``mask``, ``zero``, ``codebook``),
``forward(x, mask) -> (x_q, indices, commit_loss, distance)`` and
``indices_to_codes``.  The sign quantisation and index packing run as HIP
kernels (dctae_lfq_forward / dctae_lfq_indices_to_codes).  When
``dim != codebook_dim * num_codebooks`` the reference inserts Linear
projections (lfq.py:54-62); those run fused with the quantiser as MFMA
kernels (dctae_lfq_project_in: project_in + sign + packing, the projected
features never stored; dctae_lfq_project_out: index bits -> +-scale codes ->
project_out).  The module's nn.Linear weights stay the parameters (state dicts
interchange with the reference); the kernels read fp32 copies of them.
The training-only losses (commit / entropy, lfq.py:189-204) are out of scope
of this build.
"""
from __future__ import annotations

import ctypes as C
from math import ceil, log2

import torch
from einops import rearrange
from torch import nn

from . import _ops
from ._lib import LFQCfg


def _exists(v):
    return v is not None


class LFQ(nn.Module):
    def __init__(self, *, dim=None, codebook_size=None, diversity_gamma=2.5,
                 straight_through_activation=nn.Identity(), num_codebooks=1, keep_num_codebooks_dim=None,
                 codebook_scale=1.0):
        super().__init__()
        assert _exists(dim) or _exists(codebook_size), "either dim or codebook_size must be specified for LFQ"
        assert not _exists(codebook_size) or log2(codebook_size).is_integer(), \
            f"your codebook size must be a power of 2 for lookup free quantization (suggested {2 ** ceil(log2(codebook_size))})"
        codebook_size = codebook_size if _exists(codebook_size) else 2 ** dim
        codebook_dim = int(log2(codebook_size))
        codebook_dims = codebook_dim * num_codebooks
        dim = dim if _exists(dim) else codebook_dims
        self.has_projections = dim != codebook_dims
        self.project_in = nn.Linear(dim, codebook_dims) if self.has_projections else nn.Identity()
        self.project_out = nn.Linear(codebook_dims, dim) if self.has_projections else nn.Identity()
        self.dim = dim
        self.codebook_dim = codebook_dim
        self.num_codebooks = num_codebooks
        keep_num_codebooks_dim = keep_num_codebooks_dim if _exists(keep_num_codebooks_dim) else num_codebooks > 1
        assert not (num_codebooks > 1 and not keep_num_codebooks_dim)
        self.keep_num_codebooks_dim = keep_num_codebooks_dim
        self.activation = straight_through_activation
        self.diversity_gamma = diversity_gamma
        self.codebook_scale = codebook_scale
        self.register_buffer("mask", 2 ** torch.arange(codebook_dim - 1, -1, -1))
        self.register_buffer("zero", torch.tensor(0.0), persistent=False)
        # the (codebook_size, codebook_dim) +-scale table; only materialised for
        # small codebooks (it is 2**cd x cd floats and no kernel reads it)
        if codebook_size <= 2 ** 16:
            bits = ((torch.arange(codebook_size)[..., None].int() & self.mask) != 0).float()
            self.register_buffer("codebook", bits * codebook_scale * 2 - codebook_scale, persistent=False)

    def _fused_proj(self) -> bool:
        """The fused MFMA projection kernels compute in fp32: they serve fp32
        projection weights only.  fp16 / bf16 models keep the reference's
        nn.Linear in the model dtype (then the HIP sign / packing kernel), so
        the sign bits are those of the model-dtype projection."""
        cdims = self.codebook_dim * self.num_codebooks
        return (self.has_projections and self.dim % 4 == 0 and 4 <= self.dim <= 256 and cdims % 4 == 0
                and cdims <= 256 and self.codebook_dim <= 31 and self.num_codebooks <= 32
                and self.project_in.weight.dtype == torch.float32
                and self.project_out.weight.dtype == torch.float32)

    @staticmethod
    def _proj_w(lin: nn.Linear, dev):
        """A projection's fp32 weight / bias on ``dev``, contiguous.  No cache:
        the parameters themselves are used when they already are that (the
        usual case), so in-place updates (``weight.data.copy_``) are always
        seen; otherwise a fresh copy is made per call (a few hundred KB)."""
        def f32(t):
            return None if t is None else t.detach().to(device=dev, dtype=torch.float32).contiguous()
        return f32(lin.weight), f32(lin.bias)

    def project_codes(self, x, x_bound=None):
        """Indices only (the encode path): x (..., dim) -> (..., num_codebooks),
        project_in fused with the sign / packing when there are projections.
        x_bound: |x| <= x_bound is known (the PatchNorm clamp in
        encode_batch): the fp16 kernels, as the fused BatchEncoder path."""
        if self._fused_proj():
            w, b = self._proj_w(self.project_in, x.device)
            return _ops.lfq_project_in(x, w, b, self.cfg(self.project_in.weight.dtype), x_bound)
        h = self.project_in(x)
        _, idx = _ops.lfq_forward(h, self.cfg(h.dtype), want_quantized=False)
        return idx

    def cfg(self, dtype=None) -> LFQCfg:
        """Kernel config.  ``dtype``: the dtype the reference forms
        ``ones_like(x) * codebook_scale`` in (lfq.py:174): the index bit is the
        sign of that rounded scale (lfq.py:187), so the scale is rounded to it."""
        s = float(self.codebook_scale)
        if dtype is not None and dtype.is_floating_point and dtype != torch.float64:
            s = float(torch.tensor(s, dtype=dtype))
        return LFQCfg(self.codebook_dim, self.num_codebooks, s)

    @property
    def dtype(self):
        """The codebook's float dtype (lfq.py:101-103).  Codebooks above 2**16
        entries are not materialised; the float buffer ``zero`` follows the same
        module casts (.half(), .to(dtype)), so its dtype stands in."""
        return self.codebook.dtype if hasattr(self, "codebook") else self.zero.dtype

    def bits_to_codes(self, bits):
        return bits * self.codebook_scale * 2 - self.codebook_scale

    def indices_to_codes(self, indices, project_out=True):
        """lfq.py:105-134"""
        is_img_or_video = indices.ndim >= (3 + int(self.keep_num_codebooks_dim))
        if not self.keep_num_codebooks_dim:
            indices = rearrange(indices, "... -> ... 1")
        if project_out and self._fused_proj():
            w, b = self._proj_w(self.project_out, indices.device)
            codes = _ops.lfq_project_out(indices, w, b, self.cfg()).to(self.project_out.weight.dtype)
        else:
            codes = _ops.lfq_codes(indices, self.cfg()).to(self.dtype)
            if project_out:
                codes = self.project_out(codes)
        if is_img_or_video:
            codes = rearrange(codes, "b ... d -> b d ...")
        return codes

    def forward(self, x, mask=None):
        """lfq.py:136-227 (eval).  ``mask`` (False at padding) is required, as
        in the reference, and unused in eval."""
        if mask is None:
            raise NotImplementedError("mask")
        if self.training:
            raise NotImplementedError("LFQ training losses (lfq.py:189-204) are out of scope of the MI355X path")
        is_img_or_video = x.ndim >= 4
        if is_img_or_video:
            x = rearrange(x, "b d ... -> b ... d")
            shape = x.shape
            x = x.reshape(shape[0], -1, shape[-1])
        assert x.shape[-1] == self.dim, f"expected dimension of {self.dim} but received {x.shape[-1]}"
        if self._fused_proj():
            # eval: quantized = where(h > 0, s, -s) (lfq.py:174-175) and the index
            # bit is quantized > 0 (lfq.py:187), so quantized = bit ? |s| : -|s|:
            # project_out(quantized) is the decode kernel on the indices with the
            # scale |s| (for s < 0 the bits are the complemented signs, and
            # indices_to_codes' bit ? s : -s would give -quantized)
            indices = self.project_codes(x)
            w, b = self._proj_w(self.project_out, x.device)
            qc = self.cfg(self.project_in.weight.dtype)
            qc.codebook_scale = abs(qc.codebook_scale)
            q = _ops.lfq_project_out(indices, w, b, qc).to(x.dtype)
        else:
            x = self.project_in(x)
            q, indices = _ops.lfq_forward(x, self.cfg(x.dtype))
            q = self.project_out(q.to(x.dtype))   # the reference keeps the input dtype (fp16 / bf16 models)
        if is_img_or_video:
            q = q.reshape(*shape[:-1], q.shape[-1])
            q = rearrange(q, "b ... d -> b d ...")
            indices = indices.reshape(*shape[:-1], indices.shape[-1])
        if not self.keep_num_codebooks_dim:
            indices = rearrange(indices, "... 1 -> ...")
        return q, indices, self.zero, self.zero
