"""PatchNorm — drop-in for the reference's dct_autoencoder/patchnorm.py:32-177.

Same constructor, buffers (``n``, ``median``, ``b`` as non-trainable
Parameters, so state dicts interchange), ``frozen`` flag, ``forward`` and
``inverse_norm``.  The eval forward and the inverse run as HIP kernels
(dctae_norm_forward / dctae_norm_inverse); the training update (a13) runs as
dctae_stats kernels (see stats.py).
"""
from __future__ import annotations

import torch
from torch import nn

from . import _ops
from ._ops import FEParams, NormState
from .dct_patches import DCTPatches


class PatchNorm(nn.Module):
    def __init__(self, max_patch_h: int, max_patch_w: int, patch_size: int, channels: int, eps: float = 1e-6,
                 max_val: float = 6.0, min_val: float = -6.0):
        super().__init__()
        self.eps = eps
        self.patch_size = patch_size
        self.channels = channels
        self.max_patch_h = max_patch_h
        self.max_patch_w = max_patch_w
        self.n = nn.Parameter(torch.zeros(channels, max_patch_h, max_patch_w), requires_grad=False)
        self.median = nn.Parameter(torch.zeros(channels, max_patch_h, max_patch_w, patch_size ** 2),
                                   requires_grad=False)
        self.b = nn.Parameter(torch.ones(channels, max_patch_h, max_patch_w, patch_size ** 2), requires_grad=False)
        self.frozen = False
        self.max_val = max_val
        self.min_val = min_val

    @property
    def std(self) -> torch.Tensor:
        return self.b * 2 ** 0.5

    def _params(self) -> FEParams:
        return FEParams(channels=self.channels, patch_size=self.patch_size, max_patch_h=self.max_patch_h,
                        max_patch_w=self.max_patch_w)

    def state(self, thresholds: bool = False) -> NormState:
        """Device view of the tables handed to the kernels.  With thresholds,
        the exact LFQ-bit thresholds (one compare per element instead of a
        subtract + divide + two table reads) are attached; they are cached
        and rebuilt whenever median / b / eps / clamp change."""
        med = self.median.data
        b = self.b.data
        if med.dtype != torch.float32 or b.dtype != torch.float32:
            raise AssertionError("PatchNorm tables must be float32 on the MI355X path")
        st = NormState(med.contiguous(), b.contiguous(), float(self.eps), float(self.min_val), float(self.max_val))
        if thresholds and med.is_cuda:
            key = (med.data_ptr(), b.data_ptr(), med._version, b._version, st.eps, st.min_val, st.max_val)
            cache = getattr(self, "_thr_cache", None)
            if cache is None or cache[0] != key:
                cache = (key, _ops.norm_thresholds(st))
                self._thr_cache = cache
            st.thr = cache[1]
        return st

    def forward(self, dct_patches: DCTPatches) -> torch.Tensor:
        """patchnorm.py:81-165.  Training (and not frozen): update n / median /
        b from the non-pad tokens and return the raw patches with pads zeroed;
        otherwise return (x - median) / (b*sqrt(2) + eps) clamped."""
        if self.training and not self.frozen:
            from . import stats
            return stats.train_step(self, dct_patches)
        return _ops.norm_apply(dct_patches.patches, dct_patches.patch_channels, dct_patches.patch_positions,
                               self.state(), self._params(), inverse=False)

    def inverse_norm(self, dct_patches: DCTPatches) -> torch.Tensor:
        """patchnorm.py:167-177"""
        return _ops.norm_apply(dct_patches.patches, dct_patches.patch_channels, dct_patches.patch_positions,
                               self.state(), self._params(), inverse=True)
