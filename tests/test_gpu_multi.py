"""Multi-GPU column-shard path through the C-ABI (pm_rccl.hip): a
single-rank RCCL communicator must reproduce pm_run's per-site results exactly; n = 2, 3, 8
shards run as separate contexts on this one GPU, packed by the device kernel into the gather
chunk (pm_pack_site_results), laid side by side as an all-gather leaves them and unpacked on
the device (pm_unpack_site_results), must reproduce the unsharded run; a record buffer far too
small is settled before the gather; and the measurement helpers behind bench.py's roofline
must be self-consistent.  (RCCL across two or more GPUs needs two GPUs; the gloo tests in
test_distributed.py carry the same chunks through a real all-gather.)"""
import numpy as np
import pytest
import torch

import panman_amd

pytestmark = pytest.mark.gpu


def _engine(leaves=3000, sites=2500, seed=4):
    off, idx, root = panman_amd.random_join_tree(leaves, seed=seed)
    eng = panman_amd.Engine(0)
    eng.tree_upload(off, idx, root)
    eng.synth_columns(0, sites, seed=seed + 1)
    return eng


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_init_all_single_rank_equals_run(mode):
    eng = _engine()
    eng.run(mode)
    want_score, want_root = eng.site_results()
    want_recs = eng.mutations_raw()
    score, root = panman_amd.multi_run([eng], mode, [0], eng.num_sites)
    assert (score == want_score).all() and (root == want_root).all()
    assert (eng.mutations_raw() == want_recs).all()
    eng.close()


def test_init_rank_run_gather_equals_run():
    eng = _engine(sites=4097)
    eng.run(panman_amd.MODE_FITCH)
    want_score, want_root = eng.site_results()
    uid = panman_amd.comm_unique_id()
    assert len(uid) == 128
    eng.comm_init_rank(uid, 1, 0)
    s = torch.full((eng.num_sites,), -7, dtype=torch.int32, device="cuda")
    r = torch.full((eng.num_sites,), 77, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()   # the engine's own (non-blocking) stream does not wait for torch's
    eng.run_gather(panman_amd.MODE_FITCH, eng.num_sites, 0, s.data_ptr(), r.data_ptr())
    torch.cuda.synchronize()
    assert (s.cpu().numpy() == want_score).all() and (r.cpu().numpy() == want_root).all()
    # a shard claiming sites outside the total is refused
    with pytest.raises(panman_amd.PanmanError):
        eng.run_gather(panman_amd.MODE_FITCH, eng.num_sites, 5, s.data_ptr(), r.data_ptr())
    eng.close()


def _ranges(rule, world, sites):
    if rule == "balanced":
        return [panman_amd.shard_range_c(r, world, sites) for r in range(world)]
    lo = [min(sites, (sites * g // world + 1) // 2 * 2) for g in range(world)] + [sites]   # pm_msa.cpp
    return [(lo[g], lo[g + 1]) for g in range(world)]


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
@pytest.mark.parametrize("world,rule", [(2, "balanced"), (3, "even"), (8, "balanced"), (8, "even")])
def test_device_chunks_of_shards_equal_one_run(mode, world, rule):
    leaves, sites, seed = 3000, 4099, 9
    full = _engine(leaves, sites, seed)
    full.run(mode)
    want_score, want_root = full.site_results()
    want_recs = full.mutations()
    full.close()
    per = panman_amd.chunk_entries(sites, world)
    allc = torch.zeros(per * world, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()   # the engines' own (non-blocking) streams do not wait for torch's
    off, idx, root = panman_amd.random_join_tree(leaves, seed=seed)
    parts, offsets = [], []
    for r, (lo, hi) in enumerate(_ranges(rule, world, sites)):
        eng = panman_amd.Engine(0)
        eng.tree_upload(off, idx, root)
        eng.synth_columns(lo, hi - lo, seed=seed + 1)
        eng.run(mode)
        eng.pack_site_results(lo, per, allc[r * per:].data_ptr())
        parts.append(eng.mutations_raw())
        offsets.append(lo)
        torch.cuda.synchronize()
        eng.close()
    s = torch.full((sites,), -7, dtype=torch.int32, device="cuda")
    rt = torch.full((sites,), 77, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    helper = _engine(200, 64, 1)
    helper.unpack_site_results(allc.data_ptr(), per, world, sites, s.data_ptr(), rt.data_ptr())
    assert (s.cpu().numpy() == want_score).all() and (rt.cpu().numpy() == want_root).all()
    # a rank whose chunk head says "failed" fails the unpack on every rank
    allc[per] = 0xffffffff
    torch.cuda.synchronize()
    with pytest.raises(panman_amd.PanmanError, match="failed"):
        helper.unpack_site_results(allc.data_ptr(), per, world, sites, s.data_ptr(), rt.data_ptr())
    helper.close()
    from panman_amd.shard import merge_mut_records
    merged = merge_mut_records(parts, offsets)
    assert merged.shape[0] == want_recs.shape[0]
    from panman_amd.shard import to_pm_mut
    assert (merged == to_pm_mut(want_recs)).all()


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_tiny_record_buffer_settles_before_gather(mode):
    eng = _engine(sites=3001)
    eng.run(mode)
    want_score, want_root = eng.site_results()
    want_n = eng.mutation_count()
    eng.set_record_cap(4)   # 4 records per shard: every run overflows first
    uid = panman_amd.comm_unique_id()
    eng.comm_init_rank(uid, 1, 0)
    s = torch.zeros(eng.num_sites, dtype=torch.int32, device="cuda")
    r = torch.zeros(eng.num_sites, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()   # the engine's own (non-blocking) stream does not wait for torch's
    eng.run_gather(mode, eng.num_sites, 0, s.data_ptr(), r.data_ptr())
    assert (s.cpu().numpy() == want_score).all() and (r.cpu().numpy() == want_root).all()
    assert eng.mutation_count() == want_n
    eng.set_record_cap(4)
    eng.run(mode)
    s.zero_()
    torch.cuda.synchronize()
    eng.site_results_device(s.data_ptr(), r.data_ptr())
    torch.cuda.synchronize()
    assert (s.cpu().numpy() == want_score).all() and (r.cpu().numpy() == want_root).all()
    eng.close()


def test_run_gather_needs_a_communicator():
    eng = _engine(leaves=200, sites=100)
    s = torch.zeros(100, dtype=torch.int32, device="cuda")
    r = torch.zeros(100, dtype=torch.uint8, device="cuda")
    with pytest.raises(panman_amd.PanmanError, match="communicator"):
        eng.run_gather(panman_amd.MODE_FITCH, 100, 0, s.data_ptr(), r.data_ptr())
    eng.close()


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_design_bytes_consistent(mode):
    leaves, sites = 20000, 3000
    eng = _engine(leaves, sites)
    eng.run(mode)
    d = eng.design_bytes()
    n = eng.mutation_count()
    assert d["records"] == n
    # the post-order pass reads every leaf word once (64-word tiles of 16 B per lane)
    tiles = ((sites + 31) // 32 + 63) // 64
    assert d["up"] >= leaves * tiles * 64 * 16
    assert d["floor"] == pytest.approx(0.5 * leaves * sites + 8 * n)
    assert d["down"] >= 8 * n and d["score"] == 8 * n + 4 * sites
    eng.close()


def test_stream_copy_rate_is_physical():
    gbs = panman_amd.stream_copy_rate(0, gib=1, reps=3)
    assert 1000.0 < gbs < 8000.0


@pytest.mark.parametrize("lo,n", [(2049, 2050), (31, 100), (3750, 3750), (1, 1)])
def test_synthetic_columns_are_shard_consistent(lo, n):
    """The on-device generator gives a shard [lo, lo + n) the columns of one unsharded run
    (runs restart at global 32-site blocks; a mid-block shard start replays the block's draws),
    so bench.py --gpus N and the chunk tests see one alignment whatever the shard rule."""
    leaves = 3000
    full = _engine(leaves, lo + n + 40, seed=6)
    want = full.leaf_codes(lo, n, leaves)
    want_c = full.consensus(lo, n)
    full.close()
    off, idx, root = panman_amd.random_join_tree(leaves, seed=6)
    eng = panman_amd.Engine(0)
    eng.tree_upload(off, idx, root)
    eng.synth_columns(lo, n, seed=7)
    got = eng.leaf_codes(0, n, leaves)
    got_c = eng.consensus(0, n)
    eng.close()
    assert (got == want).all() and (got_c == want_c).all()
