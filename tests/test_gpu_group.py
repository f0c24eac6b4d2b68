"""PM_OPT_GROUP_*: two to four consecutive pre-order levels in one k_down launch, the lower
levels' waves recomputing their ancestors' finals from the ancestors' intact sets and the
last stored final, give exactly the records, scores and root codes of one launch per level
-- and of the oracle."""
import numpy as np
import pytest

import panman_amd
from _trees import random_tree
from test_gpu_fitch import _compare, _random_columns, _variant

pytestmark = pytest.mark.gpu

ALL = 1 << 40   # every level grouped


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _run(engine, waves, narrow, levels=4, mode=panman_amd.MODE_FITCH):
    engine.set_group(waves, levels)
    engine.set_narrow(narrow)
    engine.run(mode)
    got = engine.mutations()
    score, rootc = engine.site_results()
    return got, score, rootc


@pytest.mark.parametrize("variant", ["virtual", "leafparent", "plain"])
@pytest.mark.parametrize("narrow", [0, 16])
@pytest.mark.parametrize("levels", [2, 3, 4])
@pytest.mark.parametrize("tree", ["sars-like", "random-join"])
def test_groups_equal_levels(engine, variant, narrow, levels, tree):
    """T2 (deep ladder, polytomies) and T1 trees, with and without narrow bands between
    the groups: identical records to one launch per level."""
    if tree == "sars-like":
        off, idx, root = panman_amd.sars_like_tree(5000, seed=21)
    else:
        off, idx, root = panman_amd.random_join_tree(6000, seed=22)
    _variant(engine, variant)
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, 4500, seed=5)
    try:
        want = _run(engine, 0, 0)
        got = _run(engine, ALL, narrow, levels)
    finally:
        engine.set_group(32768, 4)
        engine.set_narrow(16)
    assert want[0].shape[0] > 0
    assert got[0].shape == want[0].shape and (got[0] == want[0]).all()
    assert (got[1] == want[1]).all() and (got[2] == want[2]).all()


@pytest.mark.parametrize("variant", ["virtual", "leafparent", "plain"])
@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("levels", [2, 3, 4])
def test_groups_vs_oracle_absent_and_polytomies(engine, oracle, variant, seed, levels):
    """Absent leaves (the non-AP kernels), unary nodes, polytomies, forced root; every
    level grouped, no bands."""
    rng = np.random.default_rng(5000 + seed)
    off, idx, root = random_tree(500, rng, max_children=[2, 5, 9, 40][seed], unary=[0.0, 0.2, 0.0, 0.1][seed])
    leaves = int((np.diff(off) == 0).sum())
    sites = [97, 2049, 4100, 65][seed]
    codes, present = _random_columns(rng, leaves, sites, absent_frac=[0.0, 0.1, 0.3, 0.0][seed])
    cons = rng.choice(np.array([0, 1, 2, 4, 8], np.uint8), size=sites)
    forced = rng.integers(0, 16, size=sites).astype(np.uint8) if seed % 2 else None
    engine.set_group(ALL, levels)
    engine.set_narrow(0)
    try:
        _compare(engine, oracle, off, idx, root, codes, present, cons, forced, variant)
    finally:
        engine.set_group(32768, 4)
        engine.set_narrow(16)


def test_group_option_range(engine):
    with pytest.raises(panman_amd.PanmanError):
        engine.set_group(-1)
    with pytest.raises(panman_amd.PanmanError):
        engine.set_group(32768, 5)
    engine.set_group(32768, 4)


@pytest.mark.parametrize("narrow", [0, 16, 1024])
@pytest.mark.parametrize("tree", ["sars-like", "random-join", "polytomy", "wide"])
@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_up_groups_equal_heights(engine, narrow, tree, mode):
    """PM_OPT_UP_GROUP: post-order launches where nodes of out-degree <= 3 recompute their
    same-launch children (subtree form; Sankoff: binary children only) -- identical records
    to one launch per height, with and without narrow bands over the grouped launches, and
    (wide) with Sankoff nodes of more than 255 children, whose parts index the grouped array."""
    if tree == "sars-like":
        off, idx, root = panman_amd.sars_like_tree(6000, seed=31)
    elif tree == "random-join":
        off, idx, root = panman_amd.random_join_tree(6000, seed=32)
    elif tree == "polytomy":
        off, idx, root = random_tree(3000, np.random.default_rng(33), max_children=4, unary=0.0)
    else:
        off, idx, root = random_tree(3000, np.random.default_rng(34), max_children=300, unary=0.0)
    _variant(engine, "virtual")
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, 4500, seed=6)
    res = []
    try:
        for grp in (False, True):
            engine.set_up_group(grp)
            res.append(_run(engine, 32768, narrow, mode=mode))
    finally:
        engine.set_up_group(True)
        engine.set_narrow(16)
    (w, ws, wr), (g, gs, gr) = res
    assert w.shape[0] > 0
    assert g.shape == w.shape and (g == w).all()
    assert (gs == ws).all() and (gr == wr).all()


@pytest.mark.parametrize("narrow", [0, 16])
@pytest.mark.parametrize("tree", ["sars-like", "random-join", "polytomy"])
@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_plain_up_equals_general_kernel(engine, narrow, tree, mode):
    """PM_OPT_PLAIN_UP: the grouped post-order's plain prefix (binary, no S2 / S3 child,
    nothing recomputed) in the lean kernel gives the general kernel's records (Fitch and
    Sankoff)."""
    if tree == "sars-like":
        off, idx, root = panman_amd.sars_like_tree(6000, seed=41)
    elif tree == "random-join":
        off, idx, root = panman_amd.random_join_tree(6000, seed=42)
    else:
        off, idx, root = random_tree(3000, np.random.default_rng(43), max_children=3, unary=0.05)
    _variant(engine, "virtual")
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, 4500, seed=7)
    res = []
    try:
        for on in (False, True):
            engine.set_plain_up(on, min_waves=2)   # (every plain prefix split off, small trees too)
            res.append(_run(engine, 32768, narrow, mode=mode))
    finally:
        engine.set_plain_up(True)
        engine.set_narrow(16)
    (w, ws, wr), (g, gs, gr) = res
    assert w.shape[0] > 0
    assert g.shape == w.shape and (g == w).all()
    assert (gs == ws).all() and (gr == wr).all()


@pytest.mark.parametrize("mode", [panman_amd.MODE_SANKOFF, panman_amd.MODE_BLOCK_SANKOFF])
@pytest.mark.parametrize("levels", [2, 3, 4])
@pytest.mark.parametrize("narrow", [0, 16])
def test_sankoff_groups_equal_levels(engine, mode, levels, narrow):
    """Sankoff pre-order level groups (Z0 / Z1 of the ancestors recomputed), in level launches
    and inside bands: identical records to one launch per level."""
    rng = np.random.default_rng(90 + levels)
    off, idx, root = panman_amd.sars_like_tree(4000, seed=41) if mode == panman_amd.MODE_SANKOFF else \
        random_tree(600, rng, max_children=5, unary=0.1)
    engine.tree_upload(off, idx, root)
    if mode == panman_amd.MODE_SANKOFF:
        engine.synth_columns(0, 3000, seed=7)
    else:
        n = off.shape[0] - 1
        leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
        node_row = np.full(n, -1, np.int32)
        for r, lid in enumerate(leaf_ids):
            if rng.random() > 0.2:
                node_row[lid] = r
        engine.leaves_upload(rng.choice(np.array([0, 1, 1, 1, 2], np.uint8), size=(len(leaf_ids), 400)), node_row)
        engine.sites_upload(np.zeros(400, np.uint8), rng.integers(0, 3, size=400).astype(np.uint8))
    res = []
    try:
        for waves in (0, ALL):
            engine.set_group(waves, levels)
            engine.set_narrow(narrow)
            engine.run(mode)
            recs = engine.mutations() if mode == panman_amd.MODE_SANKOFF else engine.block_mutations()
            res.append((recs,) + tuple(engine.site_results()))
    finally:
        engine.set_group(32768, 4)
        engine.set_narrow(16)
    (w, ws, wr), (g, gs, gr) = res
    assert w.shape[0] > 0
    assert g.shape == w.shape and (g == w).all()
    assert (gs == ws).all() and (gr == wr).all()
