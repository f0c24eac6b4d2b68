"""PM_OPT_NARROW: runs of narrow levels walked by one band launch (k_fitch_up_band /
k_down_band, one workgroup per tile, barriers between levels) and small levels with both
narrow and wide nodes in one mixed launch give exactly the records, scores and root codes
of one launch per level -- and of the oracle."""
import numpy as np
import pytest

import panman_amd
from _trees import names_for, random_tree
from test_gpu_fitch import _compare, _random_columns, _variant

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _run(engine, mode, narrow):
    engine.set_narrow(narrow)
    engine.run(mode)
    got = engine.mutations()
    score, rootc = engine.site_results()
    return got, score, rootc


@pytest.mark.parametrize("narrow", [16, 1024])
@pytest.mark.parametrize("virtual", [True, False])
def test_sankoff_sars_like_bands_equal_levels(engine, oracle, narrow, virtual):
    """Sankoff on T2 trees: pre-order bands and the mixed (narrow + wide) post-order launches
    of small levels give the records of one launch per level and class -- and the oracle's."""
    off, idx, root = panman_amd.sars_like_tree(3000, seed=12)
    engine.set_virtual(virtual)
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, 2200, seed=4)
    want = _run(engine, panman_amd.MODE_SANKOFF, 0)
    got = _run(engine, panman_amd.MODE_SANKOFF, narrow)
    engine.set_narrow(16)
    engine.set_virtual(True)
    assert got[0].shape == want[0].shape and (got[0] == want[0]).all()
    assert (got[1] == want[1]).all() and (got[2] == want[2]).all()
    sample = slice(300, 364)
    codes = engine.leaf_codes(sample.start, sample.stop - sample.start, 3000)
    cons = engine.consensus(sample.start, sample.stop - sample.start)
    n = off.shape[0] - 1
    node_row = np.full(n, -1, np.int32)
    node_row[:3000] = np.arange(3000)
    _, ref = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, None, algo=1, threads=8)
    ref[:, 1] += sample.start
    sel = got[0][(got[0][:, 1] >= sample.start) & (got[0][:, 1] < sample.stop)]
    assert sel.shape == ref.shape and (sel == ref).all()


@pytest.mark.parametrize("variant", ["virtual", "leafparent", "plain"])
@pytest.mark.parametrize("narrow", [4, 16, 64, 1024])
def test_sars_like_bands_equal_levels(engine, variant, narrow):
    """T2 trees (deep ladder, polytomies up to 64 children: wide nodes inside the bands);
    1024 puts almost every level into bands."""
    off, idx, root = panman_amd.sars_like_tree(5000, seed=11)
    _variant(engine, variant)
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, 4500, seed=3)
    want = _run(engine, panman_amd.MODE_FITCH, 0)
    got = _run(engine, panman_amd.MODE_FITCH, narrow)
    engine.set_narrow(16)
    assert got[0].shape == want[0].shape and (got[0] == want[0]).all()
    assert (got[1] == want[1]).all() and (got[2] == want[2]).all()
    assert want[0].shape[0] > 0


@pytest.mark.parametrize("variant", ["virtual", "leafparent", "plain"])
@pytest.mark.parametrize("seed", range(4))
def test_bands_vs_oracle_absent_and_polytomies(engine, oracle, variant, seed):
    """Absent leaves / partial presence (the non-AP kernels), unary nodes, polytomies, forced
    root, every level in a band."""
    rng = np.random.default_rng(4000 + seed)
    off, idx, root = random_tree(400, rng, max_children=[2, 5, 9, 40][seed], unary=[0.0, 0.2, 0.0, 0.1][seed])
    leaves = int((np.diff(off) == 0).sum())
    sites = [97, 2049, 4100, 65][seed]
    codes, present = _random_columns(rng, leaves, sites, absent_frac=[0.0, 0.1, 0.3, 0.0][seed])
    cons = rng.choice(np.array([0, 1, 2, 4, 8], np.uint8), size=sites)
    forced = rng.integers(0, 16, size=sites).astype(np.uint8) if seed % 2 else None
    engine.set_narrow(1024)
    try:
        _compare(engine, oracle, off, idx, root, codes, present, cons, forced, variant)
    finally:
        engine.set_narrow(16)


@pytest.mark.parametrize("mode", [panman_amd.MODE_BLOCK_FITCH, panman_amd.MODE_SANKOFF])
def test_block_and_sankoff_unaffected(engine, mode):
    """Block Fitch walks its narrow levels in bands; Sankoff its narrow pre-order levels."""
    rng = np.random.default_rng(77)
    off, idx, root = random_tree(300, rng, max_children=4, unary=0.1)
    n = off.shape[0] - 1
    leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
    node_row = np.full(n, -1, np.int32)
    for r, lid in enumerate(leaf_ids):
        if rng.random() > 0.2:
            node_row[lid] = r
    sites = 300
    block = mode == panman_amd.MODE_BLOCK_FITCH
    alphabet = np.array([0, 1, 1, 1, 2] if block else [1, 2, 4, 8, 0, 15], np.uint8)
    codes = rng.choice(alphabet, size=(len(leaf_ids), sites))
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(codes, node_row)
    engine.sites_upload(np.zeros(sites, np.uint8) if block else rng.choice(np.array([1, 2, 4, 8], np.uint8), size=sites),
                        rng.integers(0, 3, size=sites).astype(np.uint8) if block else None)
    res = []
    for narrow in (0, 1024):
        engine.set_narrow(narrow)
        engine.run(mode)
        res.append((engine.block_mutations() if block else engine.mutations(),) + tuple(engine.site_results()))
    engine.set_narrow(16)
    (w, ws, wr), (g, gs, gr) = res
    assert g.shape == w.shape and (g == w).all() and w.shape[0] > 0
    assert (gs == ws).all() and (gr == wr).all()
