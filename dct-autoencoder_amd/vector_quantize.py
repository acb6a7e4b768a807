"""VectorQuantize — drop-in for the reference's vector quantizer in inference
(dct_autoencoder/vector_quantize.py:675-1050), SURVEY §8(f)1.

Built for the configuration the model uses (modeling_dct_autoencoder.py:76-77:
euclidean codebook shared by the heads, ``codebook_dim=16``, ``kmeans_init``,
``learnable_codebook``, ``affine_param``, ``ema_update=False``).  Same
constructor arguments, submodule / parameter / buffer names (``project_in``,
``project_out``, ``_codebook.embed``, ``_codebook.codebook_mean`` …, so a
reference ``state_dict`` loads as is), ``forward(x, indices=None, mask=None)
-> (quantize, embed_ind, loss)``, ``get_codes_from_indices`` and
``get_output_from_indices``.

Everything after the caller's tensor runs in libdctae (dctae_vq_forward):
project_in / project_out on the MFMA GEMM, the masked batch statistics and
their EMA (updated even in eval, vector_quantize.py:353-359), the affine
codebook transform, the nearest-code search and the gather.  Training
(k-means init, EMA / learnable codebook updates, commitment and orthogonal
losses) is outside the hot path and raises NotImplementedError.
"""
from __future__ import annotations

from typing import Optional

import torch
from einops import rearrange
from torch import nn

from . import _ops
from ._lib import VQCfg

_CODEBOOK_DIM = 16   # the kernels' vector length (dctae_vq.hip), the model's codebook_dim


def _exists(v):
    return v is not None


class EuclideanCodebook(nn.Module):
    """Parameter / buffer holder of vector_quantize.py:239-316 (shared codebook,
    num_codebooks = 1).  The forward lives in VectorQuantize (one C-ABI call)."""

    def __init__(self, dim, codebook_size, kmeans_init=False, learnable_codebook=False, affine_param=False,
                 affine_param_batch_decay=0.99, affine_param_codebook_decay=0.9, decay=0.8, eps=1e-5,
                 sample_codebook_temp=1.0):
        super().__init__()
        self.codebook_size = codebook_size
        self.num_codebooks = 1
        self.decay = decay
        self.eps = eps
        self.sample_codebook_temp = sample_codebook_temp
        embed = torch.zeros(1, codebook_size, dim) if kmeans_init else \
            nn.init.kaiming_uniform_(torch.empty(1, codebook_size, dim))          # :264-265 uniform_init
        self.register_buffer("initted", torch.Tensor([not kmeans_init]))
        self.register_buffer("cluster_size", torch.zeros(1, codebook_size))
        self.register_buffer("embed_avg", embed.clone())
        self.learnable_codebook = learnable_codebook
        if learnable_codebook:
            self.embed = nn.Parameter(embed)
        else:
            self.register_buffer("embed", embed)
        self.affine_param = affine_param
        if not affine_param:
            return
        self.affine_param_batch_decay = affine_param_batch_decay
        self.affine_param_codebook_decay = affine_param_codebook_decay
        self.register_buffer("batch_mean", None)                                 # :310-311
        self.register_buffer("batch_variance", None)
        self.register_buffer("codebook_mean_needs_init", torch.Tensor([True]))
        self.register_buffer("codebook_mean", torch.empty(1, 1, dim))
        self.register_buffer("codebook_variance_needs_init", torch.Tensor([True]))
        self.register_buffer("codebook_variance", torch.empty(1, 1, dim))


class VectorQuantize(nn.Module):
    def __init__(self, dim, codebook_size, codebook_dim=None, heads=1, separate_codebook_per_head=False,
                 decay=0.8, eps=1e-5, freeze_codebook=False, kmeans_init=False, kmeans_iters=10, sync_kmeans=True,
                 use_cosine_sim=False, threshold_ema_dead_code=0, channel_last=True, accept_image_fmap=False,
                 commitment_weight=1.0, commitment_use_cross_entropy_loss=False, orthogonal_reg_weight=0.0,
                 orthogonal_reg_active_codes_only=False, orthogonal_reg_max_codes=None,
                 stochastic_sample_codes=False, sample_codebook_temp=1.0, straight_through=False, reinmax=False,
                 sync_codebook=None, sync_affine_param=False, ema_update=True, learnable_codebook=False,
                 in_place_codebook_optimizer=None, affine_param=False, affine_param_batch_decay=0.99,
                 affine_param_codebook_decay=0.9, sync_update_v=0.0):
        super().__init__()
        codebook_dim = codebook_dim if _exists(codebook_dim) else dim
        if use_cosine_sim or separate_codebook_per_head or codebook_dim != _CODEBOOK_DIM:
            raise NotImplementedError("the MI355X VectorQuantize covers the model's configuration: euclidean "
                                      "codebook shared by the heads, codebook_dim 16 (modeling_dct_autoencoder.py:77)")
        if accept_image_fmap or not channel_last:
            raise NotImplementedError("channel-last (b, n, d) inputs only")
        if sync_affine_param:
            raise NotImplementedError("sync_affine_param (all-reduced batch statistics)")
        assert not (ema_update and learnable_codebook), "learnable codebook not compatible with EMA update"
        assert 0 <= sync_update_v <= 1.0
        self.dim = dim
        self.heads = heads
        self.separate_codebook_per_head = separate_codebook_per_head
        codebook_input_dim = codebook_dim * heads
        requires_projection = codebook_input_dim != dim                           # :725-728
        self.project_in = nn.Linear(dim, codebook_input_dim) if requires_projection else nn.Identity()
        self.project_out = nn.Linear(codebook_input_dim, dim) if requires_projection else nn.Identity()
        self.has_projections = requires_projection
        self.eps = eps
        self.commitment_weight = commitment_weight
        self.learnable_codebook = learnable_codebook
        self.has_codebook_orthogonal_loss = orthogonal_reg_weight > 0
        self.orthogonal_reg_weight = orthogonal_reg_weight
        self.sync_update_v = sync_update_v
        self._codebook = EuclideanCodebook(codebook_dim, codebook_size, kmeans_init=kmeans_init,
                                           learnable_codebook=self.has_codebook_orthogonal_loss or learnable_codebook,
                                           affine_param=affine_param,
                                           affine_param_batch_decay=affine_param_batch_decay,
                                           affine_param_codebook_decay=affine_param_codebook_decay,
                                           decay=decay, eps=eps, sample_codebook_temp=sample_codebook_temp)
        self.codebook_size = codebook_size
        self.codebook_dim = codebook_dim
        self.accept_image_fmap = accept_image_fmap
        self.channel_last = channel_last
        self._binit = None   # device int32: batch statistics initialised (kernel-side flag)

    @property
    def codebook(self):
        return rearrange(self._codebook.embed, "1 ... -> ...")

    @codebook.setter
    def codebook(self, codes):
        self._codebook.embed.data.copy_(rearrange(codes, "... -> 1 ..."))

    # ---- C-ABI descriptor ------------------------------------------------
    def _cfg(self, dev) -> VQCfg:
        cb = self._codebook
        f = lambda t: t.detach() if t is not None else None  # noqa: E731
        keep = []

        def p(t):
            if t is None:
                return None
            t = f(t)
            if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous():
                raise AssertionError("VectorQuantize parameters must be contiguous fp32 on the input's device")
            keep.append(t)
            return t.data_ptr()

        w_in = b_in = w_out = b_out = None
        if self.has_projections:
            w_in, b_in = self.project_in.weight, self.project_in.bias
            w_out, b_out = self.project_out.weight, self.project_out.bias
        c = VQCfg(self.dim, self.heads, self.codebook_dim, self.codebook_size, int(cb.affine_param),
                  float(getattr(cb, "affine_param_batch_decay", 0.99)),
                  p(w_in), p(b_in), p(w_out), p(b_out), p(cb.embed))
        if cb.affine_param:
            if cb.batch_mean is None or cb.batch_variance is None:
                # vector_quantize.py:350-352: the first forward sets the statistics
                cb.batch_mean = torch.zeros(1, 1, self.codebook_dim, device=dev)
                cb.batch_variance = torch.zeros(1, 1, self.codebook_dim, device=dev)
                self._binit = torch.zeros(1, dtype=torch.int32, device=dev)
            elif self._binit is None or self._binit.device != dev:
                self._binit = torch.ones(1, dtype=torch.int32, device=dev)   # statistics loaded from a state_dict
            c.codebook_mean_dev = p(cb.codebook_mean)
            c.codebook_variance_dev = p(cb.codebook_variance)
            c.batch_mean_dev = p(cb.batch_mean)
            c.batch_variance_dev = p(cb.batch_variance)
            c.batch_initted_dev = self._binit.data_ptr()
        c._keep = keep
        return c

    def get_codes_from_indices(self, indices):
        """vector_quantize.py:814-831 (shared codebook: codebook[indices], '... h d -> ... (h d)')."""
        # the last index axis is taken as 'h' — also for heads == 1, where the
        # reference's rearrange folds the sequence axis into the code axis
        shape = indices.shape
        codes = _ops.vq_from_indices(self._cfg(indices.device), indices.reshape(-1, 1 if self.heads == 1
                                                                                   else self.heads),
                                     project_out=False)
        return codes.reshape(*shape[:-1], shape[-1] * self.codebook_dim)

    def get_output_from_indices(self, indices):
        """vector_quantize.py:833-835."""
        shape = indices.shape
        if shape[-1] != self.heads:
            raise RuntimeError(f"indices (..., {shape[-1]}) do not match project_out's {self.heads} heads")
        out = _ops.vq_from_indices(self._cfg(indices.device), indices.reshape(-1, self.heads), project_out=True)
        return out.reshape(*shape[:-1], self.dim)

    def forward(self, x, indices=None, mask=None, sample_codebook_temp=None, freeze_codebook=False):
        """vector_quantize.py:837-1050, eval.  Returns (quantize, embed_ind, loss = tensor([0.]))."""
        if self.training:
            raise NotImplementedError("VectorQuantize training (k-means init, codebook updates, commitment / "
                                      "orthogonal losses) is outside the MI355X inference path")
        if _exists(indices):
            raise NotImplementedError("cross-entropy loss against given indices (vector_quantize.py:952) is a "
                                      "training path")
        if not bool(self._codebook.initted):
            raise NotImplementedError("codebook not k-means initialised (vector_quantize.py:318-340 runs k-means "
                                      "on the first batch): load a trained state_dict")
        only_one = x.ndim == 2                                                    # :846-850
        if only_one:
            assert not _exists(mask)
            x = rearrange(x, "b d -> b 1 d")
        b, n, d = x.shape
        assert d == self.dim, f"expected dimension of {self.dim} but received {d}"
        xs = x.detach().float().contiguous().reshape(b * n, d)
        m = mask.reshape(b * n) if _exists(mask) else None
        q, ind = _ops.vq_forward(self._cfg(xs.device), xs, m)
        quantize = q.reshape(b, n, d).to(x.dtype)
        embed_ind = ind.reshape(b, n, self.heads)                                 # :989 '1 (b h) n -> b n h'
        if not (self.heads > 1):
            embed_ind = embed_ind[..., 0]
        if only_one:
            quantize = rearrange(quantize, "b 1 d -> b d")
            embed_ind = rearrange(embed_ind, "b 1 ... -> b ...")
        loss = torch.tensor([0.0], device=x.device)                              # :1006
        return quantize, embed_ind, loss
