"""Host-side packing plans: the greedy first-fit grouping and the batch
emission rules of the reference, computed on token COUNTS only so the device
never has to wait for them.

Mirrors (FE = dct_autoencoder/feature_extraction_dct_autoencoder.py):
  * FE._group_patches_by_max_seq_len (FE:454-513): a new row starts when
    seq_len + k > max_seq_len, in arrival order;
  * FE.iter_batches (FE:179-287): with batch_size=None every dataloader item
    flushes the current row and emits ALL rows accumulated so far (rows of
    earlier items are re-emitted — a quirk kept for drop-in fidelity); with a
    batch size B a batch of the first B rows is emitted whenever more than B
    rows are complete, and the trailing partial batch is dropped.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple


def crop_dims(h: int, w: int, patch_size: int) -> Tuple[int, int]:
    """FE:312-345"""
    assert h >= patch_size, f"image height {h} < patch_size {patch_size}"
    assert w >= patch_size, f"image width {w} < patch_size {patch_size}"
    ph = max(int(h / patch_size), 1)
    pw = max(int(w / patch_size), 1)
    return ph * patch_size, pw * patch_size


def patch_grid(h: int, w: int, patch_size: int) -> Tuple[int, int]:
    ch, cw = crop_dims(h, w, patch_size)
    return ch // patch_size, cw // patch_size


def tokens_per_image(h: int, w: int, channels: int, patch_size: int, max_patch_h: int, max_patch_w: int) -> int:
    ph, pw = patch_grid(h, w, patch_size)
    return channels * min(ph, max_patch_h) * min(pw, max_patch_w)


def choose_k(total: int, sample_patches_beta: float, max_seq_len: int, rng=random) -> int:
    """FE:429-435 with util.exp_trunc_dist (util.py:167-172): k ~ Exp(beta)
    drawn from python ``random`` in image order, so seeding ``random``
    reproduces the reference's k exactly."""
    k = total
    if sample_patches_beta > 0.0:
        k = min(round(-1 / sample_patches_beta * math.log(rng.random())), k)
        k = max(1, k)
    return min(k, max_seq_len)


@dataclass
class GroupState:
    rows: List[List[int]] = field(default_factory=list)   # complete rows (image ids)
    cur: List[int] = field(default_factory=list)
    seq_len: int = 0


def group(ks: Sequence[int], ids: Sequence[int], max_seq_len: int, max_tokens: int,
          state: Optional[GroupState] = None) -> GroupState:
    """FE:454-513"""
    st = state or GroupState()
    for k, i in zip(ks, ids):
        assert k <= max_tokens and k <= max_seq_len, f"patch with len {k} exceeds maximum sequence length"
        if st.seq_len + k > max_seq_len:
            st.rows.append(st.cur)
            st.cur = []
            st.seq_len = 0
        st.cur.append(i)
        st.seq_len += k
    return st


def iter_batch_plans(items: Iterable[Tuple[Sequence[int], Sequence[int]]], max_seq_len: int,
                     max_tokens: int, batch_size: Optional[int]) -> Iterator[List[List[int]]]:
    """FE:179-287 on counts: items are (ks, image ids) per dataloader item;
    yields the list of rows (each a list of image ids) of every batch."""
    st = None
    for ks, ids in items:
        st = group(ks, ids, max_seq_len, max_tokens, st)
        if batch_size is None and st.cur:
            st.rows.append(st.cur)
            st.cur, st.seq_len = [], 0
        if batch_size is None or len(st.rows) > batch_size:
            emit = st.rows[:batch_size]
            st = GroupState(rows=st.rows[batch_size:], cur=st.cur, seq_len=st.seq_len)
            yield emit


@dataclass
class PackPlan:
    """One emitted batch laid out for the kernels (include/dctae.h dctae_packing)."""
    images: List[int]          # image ids in row-major packing order
    row: List[int]
    col: List[int]
    k: List[int]
    local_id: List[int]
    row_len: List[int]

    @property
    def n_rows(self) -> int:
        return len(self.row_len)


def layout(rows: List[List[int]], k_of: dict) -> PackPlan:
    """FE:540-576: concatenate the images of each row; local ids 0..n-1."""
    plan = PackPlan([], [], [], [], [], [])
    for r, row in enumerate(rows):
        col = 0
        for j, i in enumerate(row):
            plan.images.append(i)
            plan.row.append(r)
            plan.col.append(col)
            plan.k.append(k_of[i])
            plan.local_id.append(j)
            col += k_of[i]
        plan.row_len.append(col)
    return plan
