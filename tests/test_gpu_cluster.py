"""PM_OPT_CLUSTER: the post-order above the plan's first level as LDS-staged sweeps (bands of
heights, one workgroup per (cluster, tile), inner sets in LDS slots; pm_cluster.cpp,
k_fitch_up_cluster) gives exactly the records, scores and root codes of the level kernels --
and of the oracle (src/fitchSankoff.cpp:30-171) -- on deep ladder trees (T2: 3-64-child
polytomies, chains hundreds of nodes long), random-join trees and random polytomy trees."""
import numpy as np
import pytest

import panman_amd
from _trees import names_for, random_tree
from panman_amd._lib import phase_report, phase_reset
from test_gpu_fitch import _random_columns

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _run(engine, off, idx, root, cluster, sites=None, codes=None, cons=None, forced=None, seed=5,
         mode=panman_amd.MODE_FITCH):
    engine.set_cluster(cluster)
    phase_reset()
    engine.tree_upload(off, idx, root)
    ph = dict(phase_report())
    if codes is None:
        engine.synth_columns(0, sites, seed=seed)
    else:
        n = off.shape[0] - 1
        leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
        node_row = np.full(n, -1, np.int32)
        node_row[leaf_ids] = np.arange(len(leaf_ids), dtype=np.int32)
        engine.leaves_upload(codes, node_row)
        engine.sites_upload(cons, forced)
    engine.run(mode)
    got = engine.mutations()
    score, rootc = engine.site_results()
    return got, score, rootc, ph


@pytest.mark.parametrize("threshold", [1, 2, 64, 1 << 20])
@pytest.mark.parametrize("tree,leaves,sites", [("sars-like", 3000, 4500), ("sars-like", 20000, 2100),
                                               ("random-join", 6000, 3000)])
def test_cluster_equals_levels(engine, tree, leaves, sites, threshold):
    """Sweeps from the default first level (1), from the top few levels only (2, 64) and over
    the whole post-order (2^20): records, scores and root codes equal to the level kernels'."""
    make = panman_amd.sars_like_tree if tree == "sars-like" else panman_amd.random_join_tree
    off, idx, root = make(leaves, seed=31)
    try:
        want = _run(engine, off, idx, root, 0, sites)
        got = _run(engine, off, idx, root, threshold, sites)
    finally:
        engine.set_cluster(panman_amd.engine.CLUSTER_DEFAULT)
    # (the default plan skips a random-join tree's bushy bands)
    assert got[3]["cluster.bands"] > 0 or (threshold == 1 and tree == "random-join"), got[3]
    assert want[0].shape[0] > 0
    assert got[0].shape == want[0].shape and (got[0] == want[0]).all()
    assert (got[1] == want[1]).all() and (got[2] == want[2]).all()


@pytest.mark.parametrize("seed", range(6))
def test_cluster_vs_oracle_polytomies(engine, oracle, seed):
    """Random trees with polytomies up to 40 children (wide rounds: children dealt to every
    wave, slot and record children mixed), every leaf present (the subtree form), random codes
    incl. gaps / ambiguity codes, a forced root on odd seeds; the whole post-order in sweeps."""
    rng = np.random.default_rng(7100 + seed)
    off, idx, root = random_tree(600, rng, max_children=[2, 3, 5, 9, 40, 64][seed], unary=0.0)
    leaves = int((np.diff(off) == 0).sum())
    sites = [97, 2049, 4100, 65, 2048, 5000][seed]
    codes, _ = _random_columns(rng, leaves, sites, absent_frac=0.0)
    cons = rng.choice(np.array([0, 1, 2, 4, 8], np.uint8), size=sites)
    forced = rng.integers(0, 16, size=sites).astype(np.uint8) if seed % 2 else None
    try:
        got, score, rootc, ph = _run(engine, off, idx, root, 1 << 20, codes=codes, cons=cons, forced=forced)
    finally:
        engine.set_cluster(panman_amd.engine.CLUSTER_DEFAULT)
    assert ph["cluster.bands"] > 0 and ph["cluster.first_level"] == 0, ph
    n = off.shape[0] - 1
    node_row = np.full(n, -1, np.int32)
    node_row[[i for i in range(n) if off[i] == off[i + 1]]] = np.arange(leaves, dtype=np.int32)
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, forced,
                                            algo=0, threads=8, with_root=True)
    assert got.shape == want.shape and (got == want).all()
    assert (rootc == want_root).all()
    nonroot = want[want[:, 0] != root]
    assert (score == np.bincount(nonroot[:, 1], minlength=sites)).all()


def test_cluster_t2_100k_sampled_vs_oracle(engine, oracle):
    """C3's shape (T2 100k leaves, 278 materialised heights) with the default plan, at 24
    sampled columns over every node against the oracle (full columns: test_gpu_fullsize)."""
    off, idx, root = panman_amd.sars_like_tree(100_000, seed=1)
    sites = 6000
    got, score, rootc, ph = _run(engine, off, idx, root, 1, sites)
    assert ph["cluster.bands"] > 0, ph
    runs = [(0, 8), (2044, 8), (sites - 8, 8)]
    codes = np.hstack([engine.leaf_codes(s0, ns, 100_000) for s0, ns in runs])
    cons = np.concatenate([engine.consensus(s0, ns) for s0, ns in runs])
    cols = np.concatenate([np.arange(s0, s0 + ns) for s0, ns in runs]).astype(np.uint32)
    n = off.shape[0] - 1
    node_row = np.full(n, -1, np.int32)
    node_row[:100_000] = np.arange(100_000)
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, None,
                                            algo=0, threads=8, with_root=True)
    want[:, 1] = cols[want[:, 1]]
    sel = got[np.isin(got[:, 1], cols)]
    assert sel.shape == want.shape and (sel == want).all()
    assert (rootc[cols] == want_root).all()
    assert (score == np.bincount(got[got[:, 0] != root][:, 1], minlength=sites)).all()


@pytest.mark.parametrize("threshold", [1, 1 << 20])
@pytest.mark.parametrize("leaves,sites", [(3000, 4500), (20000, 2100)])
def test_cluster_sankoff_equals_levels(engine, leaves, sites, threshold):
    """Sankoff runs the pre-order over the same clusters (k_down_cluster<Sankoff>: Z0 / Z1 of
    the node's record, the parent's final through LDS, src/fitchSankoff.cpp:487-531, :676-703)
    whenever the plan sweeps every height: records, scores and root codes equal to the level
    kernels'."""
    off, idx, root = panman_amd.sars_like_tree(leaves, seed=31)
    try:
        want = _run(engine, off, idx, root, 0, sites, mode=panman_amd.MODE_SANKOFF)
        got = _run(engine, off, idx, root, threshold, sites, mode=panman_amd.MODE_SANKOFF)
    finally:
        engine.set_cluster(panman_amd.engine.CLUSTER_DEFAULT)
    assert got[3]["cluster.bands"] > 0 and got[3]["cluster.down"] == 1, got[3]
    assert want[0].shape[0] > 0
    assert got[0].shape == want[0].shape and (got[0] == want[0]).all()
    assert (got[1] == want[1]).all() and (got[2] == want[2]).all()


@pytest.mark.parametrize("seed", range(4))
def test_cluster_sankoff_vs_oracle_polytomies(engine, oracle, seed):
    """Sankoff with the pre-order sweeps on random polytomy trees (every leaf present, random
    codes incl. gaps / ambiguity codes, a forced root on odd seeds) against the oracle."""
    rng = np.random.default_rng(7300 + seed)
    off, idx, root = random_tree(600, rng, max_children=[2, 3, 9, 40][seed], unary=0.0)
    leaves = int((np.diff(off) == 0).sum())
    sites = [97, 2049, 4100, 2048][seed]
    codes, _ = _random_columns(rng, leaves, sites, absent_frac=0.0)
    cons = rng.choice(np.array([0, 1, 2, 4, 8], np.uint8), size=sites)
    forced = rng.integers(0, 16, size=sites).astype(np.uint8) if seed % 2 else None
    try:
        got, score, rootc, ph = _run(engine, off, idx, root, 1 << 20, codes=codes, cons=cons, forced=forced,
                                     mode=panman_amd.MODE_SANKOFF)
    finally:
        engine.set_cluster(panman_amd.engine.CLUSTER_DEFAULT)
    assert ph["cluster.bands"] > 0 and ph["cluster.down"] == 1, ph
    n = off.shape[0] - 1
    node_row = np.full(n, -1, np.int32)
    node_row[[i for i in range(n) if off[i] == off[i + 1]]] = np.arange(leaves, dtype=np.int32)
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, forced,
                                            algo=1, threads=8, with_root=True)
    assert got.shape == want.shape and (got == want).all()
    assert (rootc == want_root).all()
    nonroot = want[want[:, 0] != root]
    assert (score == np.bincount(nonroot[:, 1], minlength=sites)).all()


def test_cluster_count_rule_leaves_wide_bands_to_levels(engine):
    """Bands of more than 16384 clusters stay level kernels (PM_CL_MAX_CLUSTERS: their waves fill
    the GPU as well): a 1M-leaf SARS-like tree's bottom bands are that wide, so its sweeps start
    above height 0 -- and then the pre-order and the Sankoff post-order stay level kernels."""
    off, idx, root = panman_amd.sars_like_tree(1_000_000, seed=1)
    engine.set_cluster(1)
    phase_reset()
    engine.tree_upload(off, idx, root)
    ph = dict(phase_report())
    assert ph["cluster.bands"] > 0 and ph["cluster.first_level"] > 0 and ph["cluster.down"] == 0, ph


def test_design_line_reads_cover_design_bytes(engine):
    """pm_design_bytes out[14..19] (the pre-order's reads at 128-B line granularity) is at least
    the 16-B-granular design of the same reads, class by class, and every class is counted."""
    off, idx, root = panman_amd.sars_like_tree(20000, seed=4)
    _run(engine, off, idx, root, 1, 4100)
    d = engine.design_bytes()
    parts, lines = d["parts"], d["line_reads"]["parts"]
    assert all(v > 0 for v in lines.values()), lines
    assert lines["levels_dirty_leaf_words"] >= parts["down_dirty_leaf_words"]
    assert lines["tail_dirty_leaf_words"] >= parts["down_tail_leaf_words"]
    assert lines["levels_own_records"] >= parts["down_own_records"]
    assert d["line_reads"]["levels"] + d["line_reads"]["tail"] > 0
