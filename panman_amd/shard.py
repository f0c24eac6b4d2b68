"""Column sharding across ranks: alignment columns are independent, so
rank r of W owns sites [r*S//W, (r+1)*S//W); the tree is replicated.  The only exchange
is one all-gather of the per-site (score, root code) pair in the library's chunk layout
(include/panman_gpu.h, pm_chunk.h); over RCCL inside the library (pm_run_gather) on GPUs,
or through torch.distributed (gloo on CPU tensors in the tests).  Mutation records stay per rank and are
merged on the host by (node, site)."""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_range(rank: int, world: int, sites: int) -> tuple[int, int]:
    return rank * sites // world, (rank + 1) * sites // world


def gather_chunks(chunk: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather one fixed-size chunk (int64 / u64 entries) per rank, rank order."""
    world = dist.get_world_size(group)
    out = torch.empty(world * chunk.numel(), dtype=chunk.dtype, device=chunk.device)
    dist.all_gather_into_tensor(out, chunk.contiguous(), group=group)
    return out


def gather_site_results(score_local, root_local, site_begin: int, sites: int, group=None):
    """Host tensors (gloo): this rank's (score, root code) shard packed into the library's
    gather chunk (pm_chunk_pack: head site_begin << 32 | count, one score | root << 32 entry
    per site), every rank's chunk all-gathered, and unpacked into full-length vectors
    (pm_chunk_unpack) -- the layout pm_run_gather moves over RCCL."""
    from .engine import chunk_entries, chunk_pack, chunk_unpack
    world = dist.get_world_size(group)
    per = chunk_entries(sites, world)
    chunk = chunk_pack(site_begin, np.asarray(score_local), np.asarray(root_local), per)
    allc = gather_chunks(torch.from_numpy(chunk.view(np.int64)), group)
    s, r = chunk_unpack(allc.numpy().view(np.uint64), per, world, sites)
    return torch.from_numpy(s), torch.from_numpy(r)


def gather_site_results_device(engine, site_begin: int, sites: int, score_all: torch.Tensor,
                               root_all: torch.Tensor, group=None):
    """GPU tensors through a torch.distributed collective: the engine's last run packed on the
    device (pm_pack_site_results), the chunks all-gathered, unpacked on the device
    (pm_unpack_site_results) into score_all [sites] int32 / root_all [sites] u8."""
    from .engine import chunk_entries
    world = dist.get_world_size(group)
    per = chunk_entries(sites, world)
    chunk = torch.empty(per, dtype=torch.int64, device=score_all.device)
    engine.pack_site_results(site_begin, per, chunk.data_ptr())   # returns with the chunk written
    allc = gather_chunks(chunk, group)
    # the collective ran on torch's stream, the unpack runs on the engine's: wait for it here
    # (the unpack itself synchronises its stream before returning)
    if allc.is_cuda:
        torch.cuda.current_stream(allc.device).synchronize()
    engine.unpack_site_results(allc.data_ptr(), per, world, sites, score_all.data_ptr(), root_all.data_ptr())


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
