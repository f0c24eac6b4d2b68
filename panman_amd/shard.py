"""Column sharding across ranks: alignment columns are independent, so
rank r of W owns sites [r*S//W, (r+1)*S//W); the tree is replicated.  The only exchange
is one all-gather of the per-site (score, root code) pair; over RCCL (backend "nccl")
on GPUs, gloo on CPU tensors in the tests.  Mutation records stay per rank and are
merged on the host by (node, site)."""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_range(rank: int, world: int, sites: int) -> tuple[int, int]:
    return rank * sites // world, (rank + 1) * sites // world


def gather_site_results(score_local: torch.Tensor, root_local: torch.Tensor, sites: int,
                        group=None) -> tuple[torch.Tensor, torch.Tensor]:
    """All-gather every rank's (score, root code) shard into full-length vectors."""
    world = dist.get_world_size(group)
    per = (sites + world - 1) // world
    dev = score_local.device
    s_pad = torch.zeros(per, dtype=torch.int32, device=dev)
    r_pad = torch.full((per,), 255, dtype=torch.uint8, device=dev)
    s_pad[: score_local.numel()] = score_local
    r_pad[: root_local.numel()] = root_local
    s_all = torch.empty(per * world, dtype=torch.int32, device=dev)
    r_all = torch.empty(per * world, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(s_all, s_pad, group=group)
    dist.all_gather_into_tensor(r_all, r_pad.view(torch.uint8), group=group)
    keep = torch.cat([torch.arange(r * per, r * per + (shard_range(r, world, sites)[1] - shard_range(r, world, sites)[0]))
                      for r in range(world)]).to(dev)
    return s_all[keep], r_all[keep]


def merge_mut_records(parts: list[np.ndarray], site_offsets: list[int]) -> np.ndarray:
    """Per-rank records in the C-ABI layout (pm_mut: [n, 2] uint32 node, site << 8 | type << 4
    | code, site local to the rank's shard) -> global pm_mut records sorted by (node, site)."""
    rows = []
    for recs, off in zip(parts, site_offsets):
        r = np.ascontiguousarray(recs, dtype=np.uint32).reshape(-1, 2).copy()
        r[:, 1] += np.uint32(off << 8)
        rows.append(r)
    allr = np.concatenate(rows) if rows else np.zeros((0, 2), np.uint32)
    order = np.lexsort((allr[:, 1], allr[:, 0]))
    return allr[order]


def to_pm_mut(recs4: np.ndarray) -> np.ndarray:
    """[n, 4] (node, site, type, code) -> [n, 2] pm_mut."""
    r = np.asarray(recs4, dtype=np.uint32)
    return np.stack([r[:, 0], (r[:, 1] << 8) | (r[:, 2] << 4) | r[:, 3]], axis=1)


def merge_records(parts: list[np.ndarray], site_offsets: list[int]) -> np.ndarray:
    """Per-rank [n,4] (node, local site, type, code) -> global records sorted by (node, site)."""
    rows = []
    for recs, off in zip(parts, site_offsets):
        r = recs.copy()
        r[:, 1] += off
        rows.append(r)
    allr = np.concatenate(rows) if rows else np.zeros((0, 4), np.uint32)
    order = np.lexsort((allr[:, 1], allr[:, 0]))
    return allr[order]
