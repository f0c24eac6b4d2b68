"""GPU parity for FASTA replay and reroot on DEEP trees (root->leaf paths longer than 64 nodes):
the replay kernel walks such a path in 64-node chunks (pm_replay.hip, chunk_edits), with an
overriding edit's order kept across chunks.  The reference: printFASTAUltraFastHelper applies
each node's mutations root first along the path (src/fasta.cpp:1753-1764, 1789-1979), so the
deepest edit of a column wins.  Every case also asserts, through the phase log, that the
tree really is deeper than one chunk."""
import numpy as np
import pytest

import panman_amd
from _panmat import random_panmat, tree_dump
from _trees import names_for, parse_newick, to_newick
from panman_amd._lib import phase_report, phase_reset
from panman_amd.engine import sars_like_tree
from panman_amd.synth import c5_panmat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _records(text):
    return sorted(">" + r for r in text.split(">")[1:])


def caterpillar(leaves: int):
    """((((s0,s1),s2),s3)...): leaf k hangs off spine node k; depth = leaves - 1."""
    n = 2 * leaves - 1
    kids = {}
    cur = 0
    nxt = leaves
    for k in range(1, leaves):
        kids[nxt] = [cur, k]
        cur = nxt
        nxt += 1
    off = np.zeros(n + 1, np.int32)
    idx = []
    for v in range(n):
        idx += kids.get(v, [])
        off[v + 1] = len(idx)
    return off, np.array(idx, np.int32), cur


def _fasta_checked(engine, pm, aligned, min_chunks=2):
    phase_reset()
    text = engine.fasta(pm, aligned)
    ph = dict(phase_report())
    assert ph["replay.max_depth"] > 64 and ph["replay.path_chunks"] >= min_chunks, ph
    return text


# paths over kDfsUnionCap (128) nodes take k_replay: 200 leaves (path bounds in the LDS ring),
# 600 (deeper than the ring's 512 nodes: bounds of the deeper path nodes from HBM)
@pytest.mark.parametrize("leaves", [200, 600])
@pytest.mark.parametrize("aligned", [True, False])
def test_caterpillar_vs_oracle(engine, oracle, aligned, leaves):
    rng = np.random.default_rng(4242)
    off, idx, root = caterpillar(leaves)
    pm = random_panmat(rng, off, idx, root, names_for(off), blocks=6, block_len=(40, 300), mut_rate=0.03)
    text = _fasta_checked(engine, pm, aligned, min_chunks=(leaves - 1 + 63) // 64)
    assert _records(text) == _records(oracle.fasta(pm, aligned))


@pytest.mark.parametrize("leaves", [200, 600])
def test_caterpillar_override_chain_across_chunks(engine, oracle, leaves):
    """Every spine node rewrites the SAME columns (each edit overrides its ancestor's, up to
    599 deep, crossing every chunk boundary); every leaf must end with its deepest ancestor's
    characters.  Also a second column set edited only by every 63rd / 64th / 65th node."""
    off, idx, root = caterpillar(leaves)
    names = names_for(off)
    pm = random_panmat(np.random.default_rng(7), off, idx, root, names, blocks=3, block_len=(30, 60),
                       mut_rate=0.0, block_rate=0.0, options=False)
    n = len(names)
    spine = [v for v in range(n) if off[v] != off[v + 1]]
    for k, v in enumerate(spine):
        code = [1, 2, 4, 8][k % 4]
        pm.add_nuc_mut(v, 0, 3, -1, 0, [code, [2, 4, 8, 1][k % 4]])   # MNP of 2 over columns 3-4
        if k % 63 == 0 or k % 64 == 0 or k % 65 == 0:
            pm.add_nuc_mut(v, 1, 5, -1, 3, [[8, 4, 2, 1][k % 4]])
    for v in range(leaves):                                           # leaves: some override again
        if v % 3 == 0:
            pm.add_nuc_mut(v, 0, 4, -1, 3, [15])
    for aligned in (True, False):
        text = _fasta_checked(engine, pm, aligned, min_chunks=(leaves - 1 + 63) // 64)
        assert _records(text) == _records(oracle.fasta(pm, aligned))


@pytest.mark.parametrize("aligned", [True, False])
def test_sars_like_2000_c5_style_vs_oracle(engine, oracle, aligned):
    """A C5-style PanMAT (blocks with gap slots, block insertions / deletions / inversions,
    SNPs, MNPs, gap-slot insertions, overriding edits) on the deep T2 tree family."""
    tree = sars_like_tree(2000, seed=3)
    pm = c5_panmat(blocks=12, mean_len=2500, mu=2e-3, block_rate=2e-2, seed=21, tree=tree)
    text = _fasta_checked(engine, pm, aligned)
    assert _records(text) == _records(oracle.fasta(pm, aligned))


def test_deep_multi_tile_many_edits_vs_oracle(engine, oracle):
    """Many column tiles (> one 8-tile workgroup group) and dense edits on a 150-deep path:
    more than one super-round per chunk and per tile."""
    off, idx, root = caterpillar(150)
    pm = c5_panmat(blocks=30, mean_len=6000, mu=4e-3, block_rate=1e-2, seed=8, tree=(off, idx, root))
    text = _fasta_checked(engine, pm, True, min_chunks=3)
    assert _records(text) == _records(oracle.fasta(pm, True))


@pytest.mark.parametrize("which", ["caterpillar", "sars_like"])
def test_reroot_deep_tree_vs_oracle(engine, oracle, which):
    """Reroot (M4) reads every leaf's replayed row (R4): on a deep tree that is the chunked
    replay; the dump must equal the oracle's restatement."""
    rng = np.random.default_rng(55)
    if which == "caterpillar":
        off, idx, root = caterpillar(120)
    else:
        off, idx, root = sars_like_tree(800, seed=5)
    names, off, idx, root = parse_newick(to_newick(off, idx, root, names_for(off)))
    pm = random_panmat(rng, off, idx, root, names, blocks=4, block_len=(20, 120), mut_rate=0.02)
    pm.branch_length = rng.integers(1, 50, size=len(names)).astype(np.float32) / 8
    leaves = pm.leaves()
    for leaf in (names[leaves[0]], names[leaves[len(leaves) // 2]]):
        phase_reset()
        f = engine.reroot(pm, leaf)
        try:
            assert dict(phase_report())["replay.max_depth"] > 64
            assert tree_dump(f) == oracle.reroot(pm, leaf)
        finally:
            f.close()


@pytest.mark.parametrize("leaves", [60, 200])
def test_override_fallback_more_than_cap(engine, oracle, leaves):
    """More overriding edits in one tile than the kernel's parallel resolver holds (kOvrCap =
    1024): every spine node rewrites the same 24 columns, so the tile's overriding edits are
    applied in path order by the fallback; 60 leaves = one chunk, 200 = four."""
    off, idx, root = caterpillar(leaves)
    names = names_for(off)
    pm = random_panmat(np.random.default_rng(17), off, idx, root, names, blocks=2, block_len=(80, 90),
                       mut_rate=0.0, block_rate=0.0, options=False)
    spine = [v for v in range(len(names)) if off[v] != off[v + 1]]
    for k, v in enumerate(spine):
        for start in (0, 6, 20, 40):
            pm.add_nuc_mut(v, 0, start, -1, 0, [[1, 2, 4, 8][(k + i) % 4] for i in range(6)])
    for aligned in (True, False):
        assert _records(engine.fasta(pm, aligned)) == _records(oracle.fasta(pm, aligned))


@pytest.mark.parametrize("dense", [True, False])
def test_dfs_stack_overflow_rebuild_vs_oracle(engine, oracle, dense):
    """k_replay_dfs (every path <= 128 nodes) on a 100-leaf caterpillar (paths of 65-99 nodes,
    one long stem shared by each 16-leaf group): dense edits in one 4 KiB column tile overflow
    the group-specific undo stacks (kDfsPCap / kDfsOCap), so the leaf that would overflow and the
    group's later leaves rebuild their rows from the consensus (pm_replay.hip dfs_leaf); sparse
    edits never do.  The phase log says which kernel ran and how many (leaf, tile) rows were
    rebuilt; the text must equal the oracle's printFASTAUltraFast (src/fasta.cpp:1789-1979)."""
    off, idx, root = caterpillar(100)
    pm = random_panmat(np.random.default_rng(91), off, idx, root, names_for(off), blocks=2,
                       block_len=(1500, 1800), mut_rate=0.02 if dense else 0.0005, block_rate=0.0)
    for aligned in (True, False):
        phase_reset()
        text = engine.fasta(pm, aligned)
        ph = dict(phase_report())
        assert 64 < ph["replay.max_depth"] <= 128 and ph["replay.dfs_groups"] > 0, ph
        if dense:
            assert ph["replay.dfs_rebuilds"] > 0, ph
        else:
            assert ph["replay.dfs_rebuilds"] == 0, ph
        assert _records(text) == _records(oracle.fasta(pm, aligned))
