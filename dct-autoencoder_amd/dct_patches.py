"""DCTPatches batch container — same fields and methods as the reference
(dct_autoencoder/dct_patches.py:6-51) — plus the JSON code dump
(to_dict / from_dict, dct_patches.py:54-122).

Difference by design: ``attn_mask`` is materialised lazily.  The reference
builds a (b, 1, S, S) bool tensor ``(id_i == id_j) & key_pad_mask_j``
(feature_extraction_dct_autoencoder.py:580-584) for every batch (9.4 MB per
row at S = 3072); here it is computed on first access, on the device of
``batched_image_ids``, with identical values.  Assigning ``attn_mask`` stores
the given tensor as in the reference.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import torch


def build_attn_mask(batched_image_ids: torch.Tensor, key_pad_mask: torch.Tensor) -> torch.Tensor:
    """(b, 1, S, S) bool = (ids_i == ids_j) & key_pad_mask_j (FE:580-584)."""
    ids = batched_image_ids
    m = ids[:, None, :, None] == ids[:, None, None, :]
    return m & key_pad_mask[:, None, None, :]


class DCTPatches:
    __slots__ = ("patches", "key_pad_mask", "_attn_mask", "batched_image_ids", "patch_channels",
                 "patch_positions", "patch_sizes", "original_sizes", "_data")

    def __init__(self, patches: torch.Tensor, key_pad_mask: torch.Tensor,
                 attn_mask: Optional[torch.Tensor] = None, batched_image_ids: torch.Tensor = None,
                 patch_channels: torch.Tensor = None, patch_positions: torch.Tensor = None,
                 patch_sizes: List[Tuple] = None, original_sizes: List[Tuple] = None,
                 _data: Optional[Dict[str, List[Any]]] = None):
        self.patches = patches
        self.key_pad_mask = key_pad_mask
        self._attn_mask = attn_mask
        self.batched_image_ids = batched_image_ids
        self.patch_channels = patch_channels
        self.patch_positions = patch_positions
        self.patch_sizes = patch_sizes
        self.original_sizes = original_sizes
        self._data = _data

    @property
    def attn_mask(self) -> torch.Tensor:
        if self._attn_mask is None:
            self._attn_mask = build_attn_mask(self.batched_image_ids, self.key_pad_mask)
        return self._attn_mask

    @attn_mask.setter
    def attn_mask(self, v):
        self._attn_mask = v

    @property
    def h_indices(self):
        return self.patch_positions[..., 0]

    @property
    def w_indices(self):
        return self.patch_positions[..., 1]

    def shallow_copy(self) -> "DCTPatches":
        return DCTPatches(patches=self.patches, key_pad_mask=self.key_pad_mask, attn_mask=self._attn_mask,
                          batched_image_ids=self.batched_image_ids, patch_channels=self.patch_channels,
                          patch_positions=self.patch_positions, patch_sizes=self.patch_sizes,
                          original_sizes=self.original_sizes, _data=self._data)

    def to(self, what) -> "DCTPatches":
        """In place, like the reference (dct_patches.py:44-51)."""
        self.patches = self.patches.to(what)
        self.key_pad_mask = self.key_pad_mask.to(what)
        if self._attn_mask is not None:
            self._attn_mask = self._attn_mask.to(what)
        self.batched_image_ids = self.batched_image_ids.to(what)
        self.patch_channels = self.patch_channels.to(what)
        self.patch_positions = self.patch_positions.to(what)
        return self

    def __repr__(self):
        return (f"DCTPatches(patches={tuple(self.patches.shape)}, rows={self.key_pad_mask.shape[0]}, "
                f"images={len(self.patch_sizes or [])}, device={self.patches.device})")


def to_dict(dct_patches: DCTPatches, codes: torch.Tensor) -> List[dict]:
    """JSON-able per-image code dump (dct_patches.py:54-83): one object per
    image with its patch grid size, original size and, per token, the
    channel, position and LFQ codes."""
    b, s, _ = codes.shape
    assert b == dct_patches.patches.shape[0] and s == dct_patches.patches.shape[1]
    ids = dct_patches.batched_image_ids.cpu()
    pad = dct_patches.key_pad_mask.cpu()
    ch = dct_patches.patch_channels.cpu()
    pos = dct_patches.patch_positions.cpu()
    cds = codes.cpu()
    objs = []
    for bi in range(b):
        for im in range(int(ids[bi].max()) + 1):
            sel = (ids[bi] == im) & ~pad[bi]
            c_l, h_l, w_l = ch[bi, sel].tolist(), pos[bi, sel, 0].tolist(), pos[bi, sel, 1].tolist()
            d_l = cds[bi, sel].tolist()
            objs.append({
                "size": dct_patches.patch_sizes[len(objs)],
                "original_size": dct_patches.original_sizes[len(objs)],
                "codes": [{"c": c, "h": h, "w": w, "data": d} for c, h, w, d in zip(c_l, h_l, w_l, d_l)],
            })
    return objs


def from_dict(obj: dict) -> Tuple[DCTPatches, torch.Tensor]:
    """Inverse of to_dict for one image (dct_patches.py:86-122): a one-row
    DCTPatches without padding, plus its (n, num_codebooks) codes."""
    toks = obj["codes"]
    n = len(toks)
    h = torch.tensor([d["h"] for d in toks], dtype=torch.long)
    w = torch.tensor([d["w"] for d in toks], dtype=torch.long)
    c = torch.tensor([d["c"] for d in toks], dtype=torch.long)
    codes = torch.tensor([d["data"] for d in toks], dtype=torch.long)
    dp = DCTPatches(
        patches=torch.zeros(1),
        key_pad_mask=torch.zeros(1, n, dtype=torch.bool),
        attn_mask=torch.ones(1, n, n, dtype=torch.bool),   # reference keeps this (1, n, n) shape
        batched_image_ids=torch.zeros(1, n, dtype=torch.long),
        patch_channels=c.unsqueeze(0),
        patch_positions=torch.stack((h, w), dim=-1).unsqueeze(0),
        patch_sizes=[obj["size"]],
        original_sizes=[obj["original_size"]],
    )
    return dp, codes
