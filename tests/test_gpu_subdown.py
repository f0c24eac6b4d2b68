"""PM_OPT_SUB_DOWN: the three- and four-leaf subtrees' finals and records from their parent's
pre-order wave (k_down<.., SUB>) give exactly the records, scores and root codes of the tail
path -- and of the oracle -- on T1 / T2 trees, with and without level groups and bands."""
import numpy as np
import pytest

import panman_amd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.set_sub_down(False)
    e.close()


def _run(engine, on):
    engine.set_sub_down(on)
    engine.run(panman_amd.MODE_FITCH)
    got = engine.mutations()
    score, rootc = engine.site_results()
    return got, score, rootc


@pytest.mark.parametrize("group", [0, 32768])
@pytest.mark.parametrize("narrow", [0, 16])
@pytest.mark.parametrize("tree", ["sars-like", "random-join"])
def test_sub_down_equals_tail(engine, tree, narrow, group):
    if tree == "sars-like":
        off, idx, root = panman_amd.sars_like_tree(6000, seed=31)
    else:
        off, idx, root = panman_amd.random_join_tree(8000, seed=32)
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, 4500, seed=7)
    engine.set_narrow(narrow)
    engine.set_group(group, 4)
    try:
        want = _run(engine, False)
        got = _run(engine, True)
    finally:
        engine.set_sub_down(False)
        engine.set_narrow(16)
        engine.set_group(32768, 4)
    assert want[0].shape[0] > 0
    assert got[0].shape == want[0].shape and (got[0] == want[0]).all()
    assert (got[1] == want[1]).all() and (got[2] == want[2]).all()


@pytest.mark.parametrize("seed", range(3))
def test_sub_down_vs_oracle(engine, oracle, seed):
    leaves, sites = [2000, 3001, 777][seed], [777, 2049, 4099][seed]
    off, idx, root = panman_amd.random_join_tree(leaves, seed=40 + seed)
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, sites, seed=9 + seed)
    got = _run(engine, True)[0]
    engine.set_sub_down(False)
    codes = engine.leaf_codes(0, sites, leaves)
    cons = engine.consensus(0, sites)
    n = 2 * leaves - 1
    names = [f"s{i}" if i < leaves else f"node_{i}" for i in range(n)]
    node_row = np.full(n, -1, np.int32)
    node_row[:leaves] = np.arange(leaves)
    _, want = oracle.csr_columns(off, idx, root, names, codes, node_row, cons, None, algo=0, threads=4)
    assert got.shape == want.shape and (got == want).all()
