"""Parity at the benchmark's full sizes (BASELINE.json C2: 4k leaves x 15k sites; north_star
N*: 1M leaves x 30k sites, random-join tree T1; C3: 100k leaves x 30k sites, SARS-like tree T2; one rank's shard of C4,
8M leaves x 3 750 sites -- SURVEY.md §8d).

The oracle cannot walk every column of these in seconds, so each run is checked by
  * bit-exact oracle columns at the first word, across the first tile boundary
    (sites 2040-2055: words 63/64 = tiles 0/1) and at the ragged last word, for every
    node of the tree (src/fitchSankoff.cpp:30-171, :359-531 via oracle/pm_oracle.cpp);
  * size-independent properties over ALL columns: records sorted by (node, site) and unique,
    types/codes in range, and (Fitch) the per-site score equal to the number of non-root
    mutation records at that site (the parsimony score, src/fitchSankoff.cpp:131-171).
"""
import numpy as np
import pytest

import panman_amd
from _trees import names_for

pytestmark = pytest.mark.gpu

CONFIGS = {
    # C2 (RSV-like, BASELINE.json config 2): 4k leaves x 15k sites -- ragged last word
    # (15 000 = 468 x 32 + 24) and 8 tiles, the last one partial
    "c2": (panman_amd.random_join_tree, 4096, 15_000),
    "nstar": (panman_amd.random_join_tree, 1_000_000, 30_000),
    "c3": (panman_amd.sars_like_tree, 100_000, 30_000),
    # C4 (8M leaves x 30k sites over 8 GPUs): one rank's column shard of 3 750 sites, on the
    # random-join tree (T1) and on the SARS-like tree (T2: height 442, polytomies of 3-64), the
    # shape of the authors' 8 M SARS-CoV-2 run (scripts/experiments.sh:72, src/panman.cpp:1568-1613)
    "c4shard": (panman_amd.random_join_tree, 8_000_000, 3_750),
    "c4shard_t2": (panman_amd.sars_like_tree, 8_000_000, 3_750),
}
BIG = ("c4shard", "c4shard_t2")


def _samples(config, sites):
    """(first site, count) runs: first word, the tile 0/1 boundary, the ragged last word."""
    if config in BIG:   # 15-16M nodes: the faithful oracle walks ~1 column per thread-minute
        return [(0, 1), (2047, 2), (sites - 1, 1)]
    return [(0, 8), (2044, 8), (sites - 8, 8)]


@pytest.fixture(scope="module")
def trees():
    return {}


@pytest.mark.timeout(900)   # the 8M-leaf oracle columns: ~2-3 min on 16 host threads
@pytest.mark.parametrize("config,mode", [(c, m) for c in CONFIGS for m in ("fitch", "sankoff")
                                         if c != "c4shard" or m == "fitch"])
def test_full_size_run(oracle, trees, config, mode):
    make, leaves, sites = CONFIGS[config]
    if config not in trees:
        off, idx, root = make(leaves, seed=1)
        trees[config] = (off, idx, root, names_for(off))
    _check_run(oracle, trees[config], leaves, sites, mode, _samples(config, sites),
               threads=16 if config in BIG else 8)


@pytest.mark.parametrize("tree", ["random-join", "sars-like"])
@pytest.mark.parametrize("nt", [0, 1])
@pytest.mark.parametrize("mode", ["fitch", "sankoff"])
def test_forced_load_policy_vs_oracle(oracle, trees, tree, nt, mode):
    """Both builds of the passes (ordinary set-record loads: pm_fitch.hip / pm_sankoff.hip; the
    non-temporal copies pm_fitch_nt.hip / pm_sankoff_nt.hip, PM_NT_LOADS) forced on a tree whose
    widest level holds >= 64k (node, tile) waves (200k leaves x 4096 sites = 2 tiles), each checked
    against the ORACLE (not against the other build) at 40 sampled columns over every node."""
    key = f"nt200k_{tree}"
    make = panman_amd.random_join_tree if tree == "random-join" else panman_amd.sars_like_tree
    if key not in trees:
        off, idx, root = make(200_000, seed=3)
        trees[key] = (off, idx, root, names_for(off))
    sites = 4096
    runs = [(0, 8), (1000, 8), (2044, 8), (3000, 8), (sites - 8, 8)]
    _check_run(oracle, trees[key], 200_000, sites, mode, runs, threads=8, nt=nt)


def _check_run(oracle, tree, leaves, sites, mode, runs, threads, nt=None):
    off, idx, root, names = tree
    n = off.shape[0] - 1
    e = panman_amd.Engine(0)
    try:
        e.tree_upload(off, idx, root)
        e.synth_columns(0, sites, seed=2)
        if nt is not None:
            e.set_nt_loads(nt)
        panman_amd.phase_reset()
        e.run(panman_amd.MODE_FITCH if mode == "fitch" else panman_amd.MODE_SANKOFF)
        phases = dict(panman_amd.phase_report())
        got = e.mutations()
        score, rootc = e.site_results()
        codes = np.hstack([e.leaf_codes(s0, ns, leaves) for s0, ns in runs])
        cons = np.concatenate([e.consensus(s0, ns) for s0, ns in runs])
    finally:
        e.close()
    if nt is not None:   # the run took the forced build (phase log of launch_all)
        assert phases.get("run.nt_loads") == nt, phases

    # all columns: order, uniqueness, ranges
    assert got.shape[0] > n // 10
    key = got[:, 0].astype(np.int64) * sites + got[:, 1]
    assert (np.diff(key) > 0).all()
    assert (got[:, 0] < n).all() and (got[:, 1] < sites).all()
    assert (got[:, 2] <= 2).all() and (got[:, 3] < 16).all()
    if mode == "fitch":
        assert (score == np.bincount(got[got[:, 0] != root][:, 1], minlength=sites)).all()

    # sampled columns (one oracle call over all of them): every node, bit-exact
    cols = np.concatenate([np.arange(s0, s0 + ns) for s0, ns in runs]).astype(np.uint32)
    node_row = np.full(n, -1, np.int32)
    node_row[:leaves] = np.arange(leaves)
    _, want, want_root = oracle.csr_columns(off, idx, root, names, codes, node_row, cons, None,
                                            algo=0 if mode == "fitch" else 1, threads=threads,
                                            with_root=True)
    want[:, 1] = cols[want[:, 1]]
    sel = got[np.isin(got[:, 1], cols)]
    assert sel.shape == want.shape and (sel == want).all(), (sel.shape, want.shape)
    assert (rootc[cols] == want_root).all()


def test_c5_full_fasta(oracle):
    """C5 (BASELINE.json config 5): the aligned FASTA of all 1000 leaves x 5.03 M columns of
    the synthetic C5 PanMAT (5.1 GB of text: offsets past 4 GiB) -- every record present and
    of the aligned length, the first 32 leaves by name bit-exact against the oracle's
    printFASTAUltraFast restatement (src/fasta.cpp:1981-2099)."""
    from panman_amd.synth import c5_panmat
    pm = c5_panmat(leaves=1000)
    e = panman_amd.Engine(0)
    try:
        got = e.fasta(pm, True)
    finally:
        e.close()
    recs = {}
    for rec in got.split(">")[1:]:
        name, _, body = rec.partition("\n")
        recs[name] = body
    del got
    assert len(recs) == 1000
    assert len({len(b) for b in recs.values()}) == 1   # aligned: one length for every leaf
    want = oracle.fasta(pm, True, leaf_limit=32)
    n = 0
    for rec in want.split(">")[1:]:
        name, _, body = rec.partition("\n")
        assert recs[name] == body, name
        n += 1
    assert n == 32
