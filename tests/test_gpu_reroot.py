"""GPU reroot (M4 + R4, src/reroot.cpp:4-262): pm_reroot vs the oracle restatement, dump
for dump (Newick with lengths and names, block mutations, NucMut records in list order),
plus the size-independent property that rerooting leaves every FASTA record unchanged."""
import numpy as np
import pytest

import panman_amd
from _panmat import random_panmat, tree_dump
from _trees import names_for, parse_newick, random_tree, to_newick
from panman_amd.panmat import PanmanFile

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _case(seed, leaves=40, blocks=5, **kw):
    rng = np.random.default_rng(seed)
    off, idx, root = random_tree(leaves, rng, max_children=4, unary=0.0)
    names, off, idx, root = parse_newick(to_newick(off, idx, root, names_for(off)))
    pm = random_panmat(rng, off, idx, root, names, blocks=blocks, **kw)
    pm.branch_length = rng.integers(1, 50, size=len(names)).astype(np.float32) / 8
    leaf_names = [names[v] for v in pm.leaves()]
    return rng, pm, leaf_names


def _records(text):
    return sorted(">" + r for r in text.split(">")[1:])


@pytest.mark.parametrize("seed", range(8))
def test_reroot_matches_oracle(engine, oracle, seed):
    rng, pm, leaf_names = _case(700 + seed)
    leaf = leaf_names[int(rng.integers(len(leaf_names)))]
    f = engine.reroot(pm, leaf)
    try:
        assert tree_dump(f) == oracle.reroot(pm, leaf)
    finally:
        f.close()


@pytest.mark.parametrize("seed", range(3))
def test_reroot_preserves_fasta_through_file(engine, tmp_path, seed):
    rng, pm, leaf_names = _case(800 + seed, leaves=120, blocks=12, block_len=(50, 400))
    leaf = leaf_names[int(rng.integers(len(leaf_names)))]
    f = engine.reroot(pm, leaf)
    path = str(tmp_path / "r.panman")
    f.write(path)
    f.close()
    g = PanmanFile(path)
    try:
        for aligned in (True, False):
            assert _records(engine.fasta(g.view(0), aligned)) == _records(engine.fasta(pm, aligned))
    finally:
        g.close()


def test_reroot_twice_and_at_child_of_root(engine, oracle, tmp_path):
    """Rerooting an already rerooted tree (written, reloaded: internal nodes renamed in
    pre-order as the reference's loader does) still matches the oracle."""
    rng, pm, leaf_names = _case(901)
    f = engine.reroot(pm, leaf_names[3])
    path = str(tmp_path / "once.panman")
    f.write(path)
    f.close()
    h = PanmanFile(path)
    pm2 = h.to_panmat(0)
    h.close()
    root_kids = pm2.child_index[pm2.child_offsets[pm2.root]:pm2.child_offsets[pm2.root + 1]]
    under_root = [pm2.names[c] for c in root_kids if pm2.child_offsets[c] == pm2.child_offsets[c + 1]]
    for leaf in (leaf_names[11], under_root[0]):
        g = engine.reroot(pm2, leaf)
        try:
            assert tree_dump(g) == oracle.reroot(pm2, leaf)
        finally:
            g.close()


def test_reroot_errors(engine):
    _, pm, _ = _case(5)
    with pytest.raises(panman_amd.PanmanError, match="not found"):
        engine.reroot(pm, "nope")
    with pytest.raises(panman_amd.PanmanError, match="not a tip"):
        engine.reroot(pm, pm.names[pm.root])
