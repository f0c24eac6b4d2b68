"""The multi-GPU gather chunk (pm_chunk.h, include/panman_gpu.h) on host memory: every
rank's shard packed with pm_chunk_pack, the ranks' chunks concatenated as an all-gather
leaves them, unpacked with pm_chunk_unpack -- for 2, 3 and 8 ranks under both shard rules
the library uses (the balanced r*S/n split of pm_shard_range / bench.py, and the MSA
driver's even-aligned split, pm_msa.cpp), uneven and empty shards included.  The same
functions run in the device pack / unpack kernels behind pm_run_gather, pm_multi_run and
bench.py --gpus N.  Columns are independent in the reference (src/panman.cpp:1381, :1568),
so the reassembled vectors must equal one unsharded run's."""
import numpy as np
import pytest

import panman_amd


def balanced(world, sites):
    return [panman_amd.shard_range_c(r, world, sites) for r in range(world)]


def even_aligned(world, sites):   # pm_msa.cpp: lo[g] = min(S, (S*g/G + 1) / 2 * 2), lo[G] = S
    lo = [min(sites, (sites * g // world + 1) // 2 * 2) for g in range(world)] + [sites]
    return [(lo[g], lo[g + 1]) for g in range(world)]


def _full(sites, seed):
    rng = np.random.default_rng(seed)
    score = rng.integers(0, 5000, size=sites).astype(np.int32)
    root = rng.choice(np.array([0, 1, 2, 4, 8, 15, 255], np.uint8), size=sites)
    return score, root


@pytest.mark.parametrize("rule", [balanced, even_aligned])
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("sites", [1, 7, 30000, 30001, 3750 * 8 + 5])
def test_pack_unpack_roundtrip(rule, world, sites):
    score, root = _full(sites, world * 1000 + sites)
    per = panman_amd.chunk_entries(sites, world)
    assert per == -(-sites // world) + 3
    chunks = []
    for lo, hi in rule(world, sites):
        assert hi - lo <= per - 1
        chunks.append(panman_amd.chunk_pack(lo, score[lo:hi], root[lo:hi], per))
    s, r = panman_amd.chunk_unpack(np.concatenate(chunks), per, world, sites)
    assert (s == score).all() and (r == root).all()


def test_chunk_layout():
    per = panman_amd.chunk_entries(10, 2)
    c = panman_amd.chunk_pack(5, np.array([7, -1], np.int32), np.array([4, 255], np.uint8), per)
    assert c[0] == (5 << 32 | 2)
    assert c[1] == 7 | (4 << 32)
    assert c[2] == 0xffffffff | (255 << 32)   # int32 -1 in the low half
    assert (c[3:] == 0).all()


def test_failed_rank_is_reported():
    sites, world = 100, 3
    score, root = _full(sites, 1)
    per = panman_amd.chunk_entries(sites, world)
    chunks = [panman_amd.chunk_pack(lo, score[lo:hi], root[lo:hi], per) for lo, hi in balanced(world, sites)]
    chunks[1] = panman_amd.chunk_pack(0, None, None, per)   # rank 1's shard failed
    with pytest.raises(panman_amd.PanmanError, match="failed"):
        panman_amd.chunk_unpack(np.concatenate(chunks), per, world, sites)


@pytest.mark.parametrize("case", ["overlap", "gap", "past_end"])
def test_inconsistent_shards_are_refused(case):
    sites, world = 100, 2
    score, root = _full(sites, 2)
    per = panman_amd.chunk_entries(sites, world)
    ranges = {"overlap": [(0, 51), (50, 100)], "gap": [(0, 49), (50, 100)], "past_end": [(0, 50), (51, 101)]}[case]
    chunks = []
    for lo, hi in ranges:
        n = hi - lo
        chunks.append(panman_amd.chunk_pack(lo, np.resize(score, n), np.resize(root, n), per))
    with pytest.raises(panman_amd.PanmanError):
        panman_amd.chunk_unpack(np.concatenate(chunks), per, world, sites)


def test_shard_wider_than_chunk_is_refused():
    per = panman_amd.chunk_entries(100, 4)
    with pytest.raises(panman_amd.PanmanError):
        panman_amd.chunk_pack(0, np.zeros(per, np.int32), np.zeros(per, np.uint8), per)
