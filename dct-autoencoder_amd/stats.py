"""PatchNorm training-mode update (patchnorm.py:101-155) on the GPU."""
from __future__ import annotations


def train_step(pn, dct_patches):
    raise NotImplementedError("PatchNorm training update: HIP stats kernels not built yet")
