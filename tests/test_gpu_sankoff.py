"""GPU parity for the Sankoff path (S1-S3 + M2): HIP kernels through the C-ABI vs the
CPU oracle, bit-exact."""
import json
import os

import numpy as np
import pytest

import panman_amd
from _trees import CODE, names_for, parse_newick, random_tree
from test_gpu_fitch import VARIANTS, _random_columns, _random_msa, _variant

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kats.json")


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("kat", [k for k in json.load(open(GOLDEN))["column"] if k["algo"] == "sankoff"],
                         ids=lambda k: k["id"])
def test_sankoff_kats_on_gpu(engine, kat):
    names, off, idx, root = parse_newick(kat["newick"])
    vals = dict(kv.split("=") for kv in kat["leaves"].split(","))
    node_row = np.full(len(names), -1, np.int32)
    rows = []
    for i, nm in enumerate(names):
        if off[i] == off[i + 1] and nm in vals:
            node_row[i] = len(rows)
            rows.append([CODE[vals[nm]]])
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(np.array(rows, np.uint8), node_row)
    forced = None if kat["forced"] == -1 else np.array([kat["forced"]], np.uint8)
    engine.sites_upload(np.array([kat["parent"]], np.uint8), forced)
    engine.run(panman_amd.MODE_SANKOFF)
    got = {names[m[0]]: [int(m[2]), "-ACMGRSVTWYHKDBN"[m[3]] if m[2] != 1 else "-"]
           for m in engine.mutations()}
    assert got == {k: list(v) for k, v in kat["expect"]["muts"].items()}
    _, rootc = engine.site_results()
    r = kat["expect"]["final"][names[root]]
    assert rootc[0] == (255 if r == -1 else r)


def _compare(engine, oracle, off, idx, root, codes, present, cons, forced, variant="virtual"):
    n = off.shape[0] - 1
    _variant(engine, variant)
    leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
    node_row = np.full(n, -1, np.int32)
    for r, lid in enumerate(leaf_ids):
        if present[r]:
            node_row[lid] = r
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(codes, node_row)
    engine.sites_upload(cons, forced)
    engine.run(panman_amd.MODE_SANKOFF)
    got = engine.mutations()
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, forced,
                                            algo=1, threads=8, with_root=True)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert (got == want).all()
    score, rootc = engine.site_results()
    assert (rootc == want_root).all()
    assert (score == np.bincount(want[want[:, 0] != root][:, 1], minlength=codes.shape[1])).all()
    _variant(engine, "virtual")


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("seed", range(4))
def test_sankoff_all_present_random_codes_vs_oracle(engine, oracle, seed, variant):
    """Every leaf present -- the subtree form's condition (S2 / S3 subtrees: Z0 inline in the
    parent's post-order wave, finals and records in the tail) -- with unrelated random codes,
    so cherries and three- / four-leaf subtrees disagree everywhere; binary, unary and
    polytomy trees; forced root (defaultState) on odd seeds."""
    rng = np.random.default_rng(1900 + seed)
    if seed == 0:
        off, idx, root = panman_amd.random_join_tree(1500, seed=seed + 3)
    else:
        off, idx, root = random_tree(700, rng, max_children=[2, 3, 5][seed - 1], unary=[0.0, 0.1, 0.0][seed - 1])
    leaves = int((np.diff(off) == 0).sum())
    sites = [700, 2049, 333, 65][seed]
    codes, present = _random_columns(rng, leaves, sites, absent_frac=0.0, gap=0.1)
    assert present.all()
    cons = rng.choice(np.array([1, 2, 4, 8], np.uint8), size=sites)
    forced = rng.integers(0, 16, size=sites).astype(np.uint8) if seed % 2 else None
    _compare(engine, oracle, off, idx, root, codes, present, cons, forced, variant)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("tree", ["random-join", "sars-like"])
def test_sankoff_synthetic_columns_sample_vs_oracle(engine, oracle, variant, tree):
    """Tree-evolved columns from the on-device generator (the bench workload, reduced):
    every variant gives the oracle's records on a column sample and identical scores."""
    leaves, sites = 20000, 4096
    off, idx, root = (panman_amd.random_join_tree(leaves, seed=1) if tree == "random-join"
                      else panman_amd.sars_like_tree(leaves, seed=1))
    leaves = int((np.diff(off) == 0).sum())
    _variant(engine, variant)
    try:
        engine.tree_upload(off, idx, root)
        engine.synth_columns(0, sites, seed=2)
        engine.run(panman_amd.MODE_SANKOFF)
        got = engine.mutations()
        score, rootc = engine.site_results()
    finally:
        _variant(engine, "virtual")
    assert (score == np.bincount(got[got[:, 0] != root][:, 1], minlength=sites)).all()
    sample = slice(1000, 1096)
    codes = engine.leaf_codes(sample.start, sample.stop - sample.start, leaves)
    cons = engine.consensus(sample.start, sample.stop - sample.start)
    n = off.shape[0] - 1
    node_row = np.full(n, -1, np.int32)
    leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
    node_row[leaf_ids] = np.arange(len(leaf_ids), dtype=np.int32)
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, None, algo=1,
                                            threads=8, with_root=True)
    want[:, 1] += sample.start
    sel = got[(got[:, 1] >= sample.start) & (got[:, 1] < sample.stop)]
    assert sel.shape == want.shape and (sel == want).all()
    assert (rootc[sample] == want_root).all()


@pytest.mark.parametrize("sites", [1, 33, 700, 2049])
def test_sankoff_random_binary_vs_oracle(engine, oracle, sites):
    rng = np.random.default_rng(sites)
    off, idx, root = panman_amd.random_join_tree(200, seed=sites)
    codes, present = _random_columns(rng, 200, sites)
    cons = rng.integers(0, 16, size=sites).astype(np.uint8)
    _compare(engine, oracle, off, idx, root, codes, present, cons, None)


@pytest.mark.parametrize("seed", range(5))
def test_sankoff_random_polytomy_vs_oracle(engine, oracle, seed):
    rng = np.random.default_rng(200 + seed)
    max_children = [3, 6, 15, 40, 300][seed]
    off, idx, root = random_tree(400, rng, max_children=max_children, unary=0.1)
    sites = 257
    codes, present = _random_columns(rng, 400, sites, absent_frac=0.3)
    cons = rng.choice(np.array([0, 1, 2, 4, 8], np.uint8), size=sites)
    forced = rng.integers(0, 16, size=sites).astype(np.uint8) if seed % 2 else None
    _compare(engine, oracle, off, idx, root, codes, present, cons, forced)


@pytest.mark.parametrize("with_ref", [False, True])
def test_msa_driver_m2_vs_oracle(oracle, with_ref):
    rng = np.random.default_rng(17 + with_ref)
    nwk, msa = _random_msa(rng, 60, 150, with_ref)
    ref = "ref" if with_ref else ""
    want = oracle.msa_build(nwk, msa, ref, mode=1)
    got = panman_amd.msa_build(nwk, msa, ref, panman_amd.MODE_SANKOFF)
    assert not want.startswith("#error"), want
    assert got == want


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
@pytest.mark.parametrize("width", [16, 300, 1500, 5000, 20000])
def test_star_polytomy_vs_oracle(engine, oracle, mode, width):
    """One node with `width` children (SARS-like trees have nodes with thousands; the
    reference sums over any number of children, src/fitchSankoff.cpp:371-402)."""
    rng = np.random.default_rng(width)
    n = width + 3
    # root(0) -> [star(1), leaf n-1]; star -> leaves 2..width+1
    off = np.zeros(n + 1, np.int32)
    off[1] = 2
    off[2:] = 2 + width
    idx = np.array([1, n - 1] + list(range(2, 2 + width)), np.int32)
    leaves = width + 1
    codes, present = _random_columns(rng, leaves, 97, absent_frac=0.1)
    codes[rng.random(codes.shape) < 0.6] = 4   # a majority state
    cons = rng.choice(np.array([1, 2, 4, 8], np.uint8), size=97)
    node_row = np.full(n, -1, np.int32)
    leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
    for r, lid in enumerate(leaf_ids):
        if present[r]:
            node_row[lid] = r
    engine.tree_upload(off, idx, 0)
    engine.leaves_upload(codes, node_row)
    engine.sites_upload(cons)
    engine.run(mode)
    got = engine.mutations()
    _, want, want_root = oracle.csr_columns(off, idx, 0, names_for(off), codes, node_row, cons, None,
                                            algo=mode, threads=8, with_root=True)
    assert got.shape == want.shape and (got == want).all()
    assert (engine.site_results()[1] == want_root).all()


def test_sankoff_sars_like_tree_vs_oracle(engine, oracle):
    """SURVEY.md §8d family T2 (deep ladder + polytomies up to 64) with tree-evolved columns."""
    leaves, sites = 6000, 2500
    off, idx, root = panman_amd.sars_like_tree(leaves, seed=6)
    n = off.shape[0] - 1
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, sites, seed=2)
    engine.run(panman_amd.MODE_SANKOFF)
    got = engine.mutations()
    _, rootc = engine.site_results()
    sample = slice(1200, 1456)
    codes = engine.leaf_codes(sample.start, sample.stop - sample.start, leaves)
    cons = engine.consensus(sample.start, sample.stop - sample.start)
    node_row = np.full(n, -1, np.int32)
    node_row[:leaves] = np.arange(leaves)
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, None,
                                            algo=1, threads=8, with_root=True)
    want[:, 1] += sample.start
    sel = got[(got[:, 1] >= sample.start) & (got[:, 1] < sample.stop)]
    assert sel.shape == want.shape and (sel == want).all()
    assert (rootc[sample] == want_root).all()


def _attach_star(off, idx, parent, width):
    """A new internal node with `width` new leaf children hung under `parent`."""
    n0 = off.shape[0] - 1
    kids = [list(idx[off[i]:off[i + 1]]) for i in range(n0)]
    star = n0
    kids[parent].append(star)
    kids.append(list(range(n0 + 1, n0 + 1 + width)))
    kids += [[] for _ in range(width)]
    off2 = np.zeros(len(kids) + 1, np.int32)
    flat = []
    for i, k in enumerate(kids):
        flat += k
        off2[i + 1] = len(flat)
    return off2, np.array(flat, np.int32)


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_sars_like_tree_with_10k_polytomy_vs_oracle(engine, oracle, mode):
    """SURVEY.md §8d T2 tree plus one node with 10 000 children (the node-degree range of
    real SARS-CoV-2 trees), bit-exact against the oracle in both modes."""
    rng = np.random.default_rng(10_000)
    off, idx, root = panman_amd.sars_like_tree(3000, seed=4)
    hang = int(idx[off[root]:off[root + 1]][0])
    hang = hang if off[hang + 1] > off[hang] else root
    off, idx = _attach_star(off, idx, hang, 10_000)
    n = off.shape[0] - 1
    leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
    sites = 161
    codes, present = _random_columns(rng, len(leaf_ids), sites, absent_frac=0.05)
    codes[rng.random(codes.shape) < 0.5] = 2   # a majority state
    cons = rng.choice(np.array([1, 2, 4, 8], np.uint8), size=sites)
    node_row = np.full(n, -1, np.int32)
    for r, lid in enumerate(leaf_ids):
        if present[r]:
            node_row[lid] = r
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(codes, node_row)
    engine.sites_upload(cons)
    engine.run(mode)
    got = engine.mutations()
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, None,
                                            algo=mode, threads=8, with_root=True)
    assert got.shape == want.shape and (got == want).all()
    assert (engine.site_results()[1] == want_root).all()
