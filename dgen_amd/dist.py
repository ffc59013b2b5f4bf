"""Multi-GPU: agents shard across ranks with no data-path collective; one
small RCCL all-reduce per model year carries the per-(state, sector) totals
and per-state 8760-h net sums that the diffusion step consumes.

The reference's parallel shape is a spawn Pool over np.array_split chunks of
the agent ids (dgen_model.py:312-339); shard_bounds() keeps that split so a
rank's shard is exactly the chunk the reference's worker `rank` would size.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

TOTAL_FIELDS = ("system_kw", "batt_kw", "batt_kwh", "n_agents")


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of rank's chunk under np.array_split(range(n), world)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    q, r = divmod(int(n), int(world))
    lo = rank * q + min(rank, r)
    hi = lo + q + (1 if rank < r else 0)
    return lo, hi


def group_order(keys: Sequence) -> Tuple[np.ndarray, np.ndarray, List]:
    """Stable order that makes every group contiguous + segment offsets.
    Returns (perm, seg_off[S+1], unique keys in order)."""
    keys = list(keys)
    uniq: Dict = {}
    ids = np.empty(len(keys), dtype=np.int64)
    for i, k in enumerate(keys):
        ids[i] = uniq.setdefault(k, len(uniq))
    perm = np.argsort(ids, kind="stable")
    counts = np.bincount(ids, minlength=len(uniq))
    seg_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return perm, seg_off, list(uniq.keys())


def allreduce_sum(t):
    """SUM all-reduce over the default process group (RCCL on GPU tensors,
    gloo on CPU tensors); identity when not distributed."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def local_totals_device(engine, out, perm_dev, seg_off):
    """Per-group [system_kw, batt_kw, batt_kwh, n_agents] of this rank's shard,
    computed by the device segment-sum kernel on group-ordered outputs."""
    import torch
    cols = [out["system_kw"], out["batt_kw"], out["batt_kwh"],
            torch.ones_like(out["system_kw"])]
    planes = torch.stack([c.index_select(0, perm_dev) for c in cols])
    return engine.segment_sums(planes, seg_off)


def global_totals(engine, out, group_keys: Sequence, all_keys: Sequence):
    """All-reduced per-group totals over every rank, rows in `all_keys` order
    (every rank must pass the same all_keys)."""
    import torch
    perm, seg_off, uniq = group_order(group_keys)
    perm_dev = torch.as_tensor(perm, device=engine.dev)
    loc = local_totals_device(engine, out, perm_dev, seg_off)
    full = torch.zeros((len(all_keys), len(TOTAL_FIELDS)), dtype=torch.float64, device=engine.dev)
    pos = {k: i for i, k in enumerate(all_keys)}
    idx = torch.as_tensor([pos[k] for k in uniq], device=engine.dev, dtype=torch.int64)
    full.index_copy_(0, idx, loc)
    return allreduce_sum(full)
