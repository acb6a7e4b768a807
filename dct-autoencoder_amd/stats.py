"""PatchNorm training-mode update (reference patchnorm.py:101-155) on the GPU.

The reference updates its running statistics with a Python triple loop over
all C*mh*mw cells (one boolean mask + torch.median per cell) followed by two
scatter_add_ passes.  Here the whole update is one C-ABI call
(``dctae_norm_train_step``) running the dctae_stats.hip kernels:

  cells -> per-cell token lists in batch order (ballot scan, one wave per cell)
        -> lower median per (cell, element) by rank selection in LDS
        -> running-median merge -> sum |x - median| in batch order
        -> running-b merge -> n += batch_n -> pads zeroed

Results are bit-exact with the reference (tests/test_gpu_stats.py::
test_train_step_reproduces_reference_fit / test_train_step_matches_oracle):
the per-cell lists keep batch order, which is the reference's scatter_add_
accumulation order, and every fp32 op is rounded like the reference's
separate torch ops.

Like the reference, the update replaces the tables (``.data = new``) rather
than mutating the tensors a caller may hold.
"""
from __future__ import annotations

import torch

from . import _ops


def train_step(pn, dct_patches) -> torch.Tensor:
    """patchnorm.py:101-155 for ``PatchNorm.forward`` in training mode."""
    n = pn.n.data.float().clone().contiguous()
    median = pn.median.data.float().clone().contiguous()
    b = pn.b.data.float().clone().contiguous()
    out = _ops.norm_train_step(dct_patches.patches, dct_patches.patch_channels, dct_patches.patch_positions,
                               dct_patches.key_pad_mask, n, median, b, pn._params())
    _ops.check_device_errors(n.device)
    pn.n.data = n
    pn.median.data = median
    pn.b.data = b
    pn._thr_cache = None
    return out.view(dct_patches.patches.shape)
