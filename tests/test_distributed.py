"""N>1 path on CPU: column shards on 2 / 3 / 8 gloo ranks, one all-gather of (score, root code)
carried in the library's gather chunks (pm_chunk_pack -> all_gather -> pm_chunk_unpack, the
layout pm_run_gather moves over RCCL), host merge of the records in the C-ABI layout (pm_mut:
node, site << 8 | type << 4 | code, sites local to the rank's shard, as pm_mutations_fetch
returns them) -- must equal the single-shard result, under both shard rules in use (balanced
and the MSA driver's even-aligned split).  The oracle is the per-shard engine, since this host
has no GPU; the GPU side of the same path (pm_run_gather over RCCL) is tests/test_gpu_multi.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _problem():
    import sys
    sys.path.insert(0, ROOT)
    import panman_amd
    rng = np.random.default_rng(5)
    leaves, sites = 150, 211
    off, idx, root = panman_amd.random_join_tree(leaves, seed=3)
    codes = rng.choice(np.array([1, 2, 4, 8, 0, 15], np.uint8), size=(leaves, sites))
    cons = rng.choice(np.array([1, 2, 4, 8], np.uint8), size=sites)
    node_row = np.full(2 * leaves - 1, -1, np.int32)
    node_row[:leaves] = np.arange(leaves)
    names = [f"s{i}" if i < leaves else f"node_{i}" for i in range(2 * leaves - 1)]
    return off, idx, root, codes, cons, node_row, names


def _ranges(rule, world, sites):
    if rule == "balanced":
        return [(r * sites // world, (r + 1) * sites // world) for r in range(world)]
    lo = [min(sites, (sites * g // world + 1) // 2 * 2) for g in range(world)] + [sites]   # pm_msa.cpp
    return [(lo[g], lo[g + 1]) for g in range(world)]


def _worker(rank, world, port, q, rule):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as orc
    from panman_amd.shard import gather_site_results, to_pm_mut
    off, idx, root, codes, cons, node_row, names = _problem()
    lo, hi = _ranges(rule, world, codes.shape[1])[rank]
    _, recs, rootc = orc.load().csr_columns(off, idx, root, names, codes[:, lo:hi], node_row, cons[lo:hi],
                                           None, algo=0, threads=2, with_root=True)
    score = np.bincount(recs[recs[:, 0] != root][:, 1], minlength=hi - lo).astype(np.int32)
    s_all, r_all = gather_site_results(score, rootc, lo, codes.shape[1])
    objs = [None] * world
    dist.all_gather_object(objs, (lo, to_pm_mut(recs)))
    if rank == 0:
        q.put((s_all.numpy(), r_all.numpy(), objs))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,rule", [(2, "balanced"), (3, "balanced"), (3, "even"), (8, "even")])
def test_sharded_columns_match_single_shard(world, rule):
    import sys
    sys.path.insert(0, ROOT)
    import oracle as orc
    from panman_amd.shard import merge_mut_records, to_pm_mut
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, rule)) for r in range(world)]
    for p in procs:
        p.start()
    s_all, r_all, parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    off, idx, root, codes, cons, node_row, names = _problem()
    _, want, want_root = orc.load().csr_columns(off, idx, root, names, codes, node_row, cons, None, algo=0,
                                                threads=2, with_root=True)
    want_score = np.bincount(want[want[:, 0] != root][:, 1], minlength=codes.shape[1])
    assert (s_all == want_score).all()
    assert (r_all == want_root).all()
    merged = merge_mut_records([p[1] for p in parts], [p[0] for p in parts])
    want_mut = to_pm_mut(want)
    assert merged.shape == want_mut.shape and (merged == want_mut).all()
