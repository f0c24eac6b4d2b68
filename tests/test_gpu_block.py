"""GPU parity for block-level parsimony (B1 block Fitch, B2 block Sankoff) vs the oracle."""
import json
import os

import numpy as np
import pytest

import panman_amd
from _trees import names_for, parse_newick, random_tree

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kats.json")


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def test_block_fitch_kat_on_gpu(engine):
    kat = [k for k in json.load(open(GOLDEN))["column"] if k["id"] == "B-K1"][0]
    names, off, idx, root = parse_newick(kat["newick"])
    vals = dict(kv.split("=") for kv in kat["leaves"].split(","))
    node_row = np.full(len(names), -1, np.int32)
    rows = []
    for i, nm in enumerate(names):
        if off[i] == off[i + 1] and nm in vals:
            node_row[i] = len(rows)
            rows.append([int(vals[nm]).bit_length() - 1])   # state {1,2,4} -> code {0,1,2}
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(np.array(rows, np.uint8), node_row)
    engine.sites_upload(np.array([0], np.uint8))
    engine.run(panman_amd.MODE_BLOCK_FITCH)
    got = {names[m[0]]: [int(m[2]), str(int(m[3]))] for m in engine.block_mutations()}
    assert got == {k: list(v) for k, v in kat["expect"]["muts"].items()}


@pytest.mark.parametrize("mode", [panman_amd.MODE_BLOCK_FITCH, panman_amd.MODE_BLOCK_SANKOFF])
@pytest.mark.parametrize("seed", range(4))
def test_block_random_vs_oracle(engine, oracle, mode, seed):
    rng = np.random.default_rng(300 + seed)
    if seed == 0:
        off, idx, root = panman_amd.random_join_tree(120, seed=seed + 1)
    else:
        off, idx, root = random_tree(120, rng, max_children=[2, 4, 30, 3][seed], unary=0.1)
    n = off.shape[0] - 1
    blocks = 150
    codes = rng.choice(np.array([0, 1, 1, 1, 2], np.uint8), size=(120, blocks))
    present = rng.random(120) >= 0.15
    leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
    node_row = np.full(n, -1, np.int32)
    for r, lid in enumerate(leaf_ids):
        if present[r]:
            node_row[lid] = r
    cons = np.zeros(blocks, np.uint8)
    forced = rng.integers(0, 3, size=blocks).astype(np.uint8) if seed % 2 else None
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(codes, node_row)
    engine.sites_upload(cons, forced)
    engine.run(mode)
    got = engine.block_mutations()
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, forced,
                                            algo=mode, threads=8, with_root=True)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert (got == want).all()
    assert (engine.site_results()[1] == want_root).all()
