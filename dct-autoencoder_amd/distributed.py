"""Data-parallel PatchNorm fitting.

Encode shards images across ranks with no collective.  The one exchange step
on the path is the PatchNorm statistics update when the tables are fitted on
a data-parallel batch (reference train.py drives PatchNorm.forward in
training mode on each batch; patchnorm.py:101-155).

Contract: ``train_step(pn, shard)`` on R ranks leaves every rank with tables
bit-identical to the reference's single-process update applied to the R
shards as R consecutive batches in rank order.  The running update is a
chain (the median merge of shard r uses n after shards < r, and shard r's
MAD is taken around the median after shard r), so the exchange is:

  1. each rank: (batch_n_r, batch_median_r) of its shard        [HIP kernels]
  2. all_gather of both (RCCL over xGMI; C*mh*mw*(P*P+1) floats per rank)
  3. every rank replays the median chain r = 0..R-1 locally     [merge kernel]
     and keeps the median after its own shard
  4. each rank: batch_b_r around that median                    [HIP kernel]
  5. all_gather of batch_b, every rank replays the b / n chain  [merge kernel]

Two all_gathers of C*mh*mw*P*P floats (2.4 MB at 3x32x32x196) per rank per
fit step — small next to the encode traffic, so no bucketing is needed.

``ops`` is the statistics backend (default: the HIP kernels of this package).
The CPU multi-process tests inject a backend built on the test oracle to
check the exchange logic over gloo; the product path has no CPU fallback.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist

from . import _ops


@dataclass
class StatsOps:
    """batch_stats(x, ch, pos, key_pad) -> (batch_n, batch_median);
    batch_mad(x, ch, pos, key_pad, median, batch_n) -> batch_b;
    merge_(table, batch, n, batch_n, n_update) in place."""
    batch_stats: Callable
    batch_mad: Callable
    merge_: Callable


def hip_ops(p: _ops.FEParams) -> StatsOps:
    return StatsOps(
        batch_stats=lambda x, ch, pos, kp: _ops.norm_batch_stats(x, ch, pos, kp, p),
        batch_mad=lambda x, ch, pos, kp, med, bn: _ops.norm_batch_mad(x, ch, pos, kp, med, p),
        merge_=_ops.norm_merge_,
    )


def _all_gather(t: torch.Tensor, group) -> list:
    world = dist.get_world_size(group)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t.contiguous(), group=group)
    return out


def fit_tables(n, median, b, x, ch, pos, key_pad, ops: StatsOps, group=None):
    """Steps 1-5 above on plain tensors; returns the new (n, median, b)."""
    rank = dist.get_rank(group)
    bn, bm = ops.batch_stats(x, ch, pos, key_pad)
    all_bn = _all_gather(bn, group)
    all_bm = _all_gather(bm, group)
    med = median.clone()
    nn_ = n.clone()
    mine = None
    for r in range(len(all_bn)):
        ops.merge_(med, all_bm[r], nn_, all_bn[r], True)
        if r == rank:
            mine = med.clone()
    bb = ops.batch_mad(x, ch, pos, key_pad, mine, all_bn[rank])
    all_bb = _all_gather(bb, group)
    bnew = b.clone()
    n2 = n.clone()
    for r in range(len(all_bb)):
        ops.merge_(bnew, all_bb[r], n2, all_bn[r], True)
    return n2, med, bnew


def train_step(pn, dct_patches, group=None, ops: Optional[StatsOps] = None) -> torch.Tensor:
    """Data-parallel PatchNorm.forward in training mode: every rank passes its
    own shard; returns the shard's patches with pads zeroed (patchnorm.py:153-155)."""
    ops = ops or hip_ops(pn._params())
    dp = dct_patches
    n, med, b = fit_tables(pn.n.data.float().contiguous(), pn.median.data.float().contiguous(),
                           pn.b.data.float().contiguous(), dp.patches, dp.patch_channels, dp.patch_positions,
                           dp.key_pad_mask, ops, group)
    pn.n.data, pn.median.data, pn.b.data = n, med, b
    pn._thr_cache = None
    return torch.where(dp.key_pad_mask.unsqueeze(-1), torch.zeros((), dtype=dp.patches.dtype,
                                                                   device=dp.patches.device), dp.patches)
