"""GPU parity for the Fitch path (F1-F3 + M1): HIP kernels through the C-ABI vs the
CPU oracle, bit-exact."""
import json
import os

import numpy as np
import pytest

import panman_amd
from _trees import CODE, names_for, parse_newick, random_tree, to_newick

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kats.json")


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _log2(state):
    return state.bit_length() - 1


@pytest.mark.parametrize("kat", [k for k in json.load(open(GOLDEN))["column"] if k["algo"] == "fitch"],
                         ids=lambda k: k["id"])
def test_fitch_kats_on_gpu(engine, kat):
    names, off, idx, root = parse_newick(kat["newick"])
    vals = dict(kv.split("=") for kv in kat["leaves"].split(","))
    n = len(names)
    node_row = np.full(n, -1, np.int32)
    rows = []
    for i, nm in enumerate(names):
        if off[i] == off[i + 1] and nm in vals:
            node_row[i] = len(rows)
            rows.append([CODE[vals[nm]]])
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(np.array(rows, np.uint8), node_row)
    forced = None if kat["forced"] == -1 else np.array([_log2(kat["forced"])], np.uint8)
    engine.sites_upload(np.array([_log2(kat["parent"])], np.uint8), forced)
    engine.run(panman_amd.MODE_FITCH)
    got = {names[m[0]]: [int(m[2]), "-ACMGRSVTWYHKDBN"[m[3]] if m[2] != 1 else "-"]
           for m in engine.mutations()}
    assert got == {k: list(v) for k, v in kat["expect"]["muts"].items()}
    score, rootc = engine.site_results()
    assert rootc[0] == _log2(kat["expect"]["final"][names[root]])
    assert score[0] == sum(1 for k in got if k != names[root])


def _random_columns(rng, leaves, sites, absent_frac=0.1, gap=0.2):
    alphabet = np.array([1, 2, 4, 8, 1, 2, 4, 8, 0, 15, 5, 10, 3], np.uint8)
    codes = alphabet[rng.integers(0, alphabet.size, size=(leaves, sites))]
    codes[rng.random((leaves, sites)) < gap] = 0
    present = rng.random(leaves) >= absent_frac
    return codes, present


VARIANTS = ["virtual", "leafparent", "plain"]


def _variant(engine, variant):
    """virtual (default): leaf-parents and, with every leaf present, three- and four-leaf
    subtrees evaluated inline by their parent; leafparent: leaf-parents only; plain: every
    internal node materialised."""
    engine.set_virtual(variant != "plain")
    engine.set_subtree(variant == "virtual")


def _compare(engine, oracle, off, idx, root, codes, present, cons, forced, variant="virtual"):
    _variant(engine, variant)
    n = off.shape[0] - 1
    leaf_ids = [i for i in range(n) if off[i] == off[i + 1]]
    node_row = np.full(n, -1, np.int32)
    for r, lid in enumerate(leaf_ids):
        if present[r]:
            node_row[lid] = r
    engine.tree_upload(off, idx, root)
    engine.leaves_upload(codes, node_row)
    engine.sites_upload(cons, forced)
    engine.run(panman_amd.MODE_FITCH)
    got = engine.mutations()
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, forced,
                                            algo=0, threads=8, with_root=True)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert (got == want).all()
    score, rootc = engine.site_results()
    assert (rootc == want_root).all()
    nonroot = want[want[:, 0] != root]
    assert (score == np.bincount(nonroot[:, 1], minlength=codes.shape[1])).all()
    return got


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("sites", [1, 31, 32, 33, 700, 2049])
def test_random_binary_vs_oracle(engine, oracle, sites, variant):
    rng = np.random.default_rng(sites)
    off, idx, root = panman_amd.random_join_tree(257, seed=sites)
    codes, present = _random_columns(rng, 257, sites)
    cons = rng.integers(0, 16, size=sites).astype(np.uint8)
    _compare(engine, oracle, off, idx, root, codes, present, cons, None, variant)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("seed", range(4))
def test_all_present_random_codes_vs_oracle(engine, oracle, seed, variant):
    """Every leaf present (the subtree form's condition) with unrelated random codes, so
    cherries and three- / four-leaf subtrees disagree everywhere; binary, unary and
    polytomy trees; forced root on odd seeds."""
    rng = np.random.default_rng(900 + seed)
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
@pytest.mark.parametrize("seed", range(6))
def test_random_polytomy_vs_oracle(engine, oracle, seed, variant):
    rng = np.random.default_rng(100 + seed)
    off, idx, root = random_tree(300, rng, max_children=[6, 3, 4, 26, 2, 12][seed], unary=[0.1, 0.3, 0, 0.1, 0.5, 0][seed])
    sites = 333
    codes, present = _random_columns(rng, 300, sites, absent_frac=0.2)
    cons = rng.choice(np.array([0, 1, 2, 4, 8], np.uint8), size=sites)
    forced = rng.integers(0, 16, size=sites).astype(np.uint8) if seed % 2 else None
    _compare(engine, oracle, off, idx, root, codes, present, cons, forced, variant)


def test_all_absent_subtree_and_tiny_tree(engine, oracle):
    # ((a,b),c): a,b absent -> node_2 has state 0 and stays unresolved (src/fitchSankoff.cpp:101-103)
    off = np.array([0, 2, 4, 4, 4, 4], np.int32)
    idx = np.array([1, 4, 2, 3], np.int32)
    codes = np.array([[1, 2, 0, 8]], np.uint8)
    present = np.array([False, False, True])
    cons = np.array([1, 1, 1, 1], np.uint8)
    _compare(engine, oracle, off, idx, 0, np.vstack([codes, codes, codes]), present, cons, None)


@pytest.mark.parametrize("variant", VARIANTS)
def test_synthetic_columns_sample_vs_oracle(engine, oracle, variant):
    """Tree-evolved columns from the on-device generator (bench workload, reduced size)."""
    leaves, sites = 20000, 4096
    off, idx, root = panman_amd.random_join_tree(leaves, seed=1)
    _variant(engine, variant)
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, sites, seed=2)
    engine.run(panman_amd.MODE_FITCH)
    got = engine.mutations()
    score, rootc = engine.site_results()
    assert (score == np.bincount(got[got[:, 0] != root][:, 1], minlength=sites)).all()
    sample = slice(1000, 1096)
    codes = engine.leaf_codes(sample.start, sample.stop - sample.start, leaves)
    cons = engine.consensus(sample.start, sample.stop - sample.start)
    node_row = np.full(2 * leaves - 1, -1, np.int32)
    node_row[:leaves] = np.arange(leaves)
    _, want = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, None, algo=0,
                                 threads=8)
    want[:, 1] += sample.start
    sel = got[(got[:, 1] >= sample.start) & (got[:, 1] < sample.stop)]
    assert sel.shape == want.shape and (sel == want).all()
    assert got.shape[0] > 0


def _random_msa(rng, leaves, sites, with_ref):
    off, idx, root = random_tree(leaves, rng, max_children=3, unary=0.0)
    names = names_for(off)
    nwk = to_newick(off, idx, root, names)
    root_seq = rng.choice(list("ACGT"), size=sites)
    rows = {}
    for i in range(len(names)):
        if off[i] == off[i + 1]:
            s = root_seq.copy()
            flip = rng.random(sites) < 0.3
            s[flip] = rng.choice(list("ACGTNRY-"), size=flip.sum())
            rows[names[i]] = "".join(s)
    # drop one leaf from the alignment; add a row that is not in the tree
    drop = sorted(rows)[1]
    del rows[drop]
    rows["zz_outgroup"] = "".join(rng.choice(list("ACGT-"), size=sites))
    if with_ref:
        rows["ref"] = "".join(rng.choice(list("ACGT"), size=sites))
    text = "".join(f">{k} desc\n{v[:sites // 2]}\n{v[sites // 2:]}\n" for k, v in rows.items())
    return nwk, text


@pytest.mark.parametrize("with_ref", [False, True])
def test_msa_driver_m1_vs_oracle(oracle, with_ref):
    rng = np.random.default_rng(7 + with_ref)
    nwk, msa = _random_msa(rng, 60, 150, with_ref)
    ref = "ref" if with_ref else ""
    want = oracle.msa_build(nwk, msa, ref, mode=0)
    got = panman_amd.msa_build(nwk, msa, ref, panman_amd.MODE_FITCH)
    assert not want.startswith("#error"), want
    assert got == want


@pytest.mark.parametrize("variant", VARIANTS)
def test_sars_like_tree_vs_oracle(engine, oracle, variant):
    """SURVEY.md §8d family T2 (deep ladder + polytomies up to 64) with tree-evolved columns."""
    leaves, sites = 6000, 2500
    off, idx, root = panman_amd.sars_like_tree(leaves, seed=5)
    n = off.shape[0] - 1
    _variant(engine, variant)
    engine.tree_upload(off, idx, root)
    engine.synth_columns(0, sites, seed=2)
    engine.run(panman_amd.MODE_FITCH)
    got = engine.mutations()
    score, rootc = engine.site_results()
    sample = slice(700, 956)
    codes = engine.leaf_codes(sample.start, sample.stop - sample.start, leaves)
    cons = engine.consensus(sample.start, sample.stop - sample.start)
    node_row = np.full(n, -1, np.int32)
    node_row[:leaves] = np.arange(leaves)
    _, want, want_root = oracle.csr_columns(off, idx, root, names_for(off), codes, node_row, cons, None,
                                            algo=0, threads=8, with_root=True)
    want[:, 1] += sample.start
    sel = got[(got[:, 1] >= sample.start) & (got[:, 1] < sample.stop)]
    assert sel.shape == want.shape and (sel == want).all()
    assert (rootc[sample] == want_root).all()
    assert (score == np.bincount(got[got[:, 0] != root][:, 1], minlength=sites)).all()
