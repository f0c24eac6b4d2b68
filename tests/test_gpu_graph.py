"""PM_OPT_GRAPH: pm_run replayed from a captured hipGraph gives the same mutations, scores
and root codes as the eager launch sequence, in every mode, and re-captures when the
columns or the tree change."""
import numpy as np
import pytest

import panman_amd
from _trees import random_tree

pytestmark = pytest.mark.gpu

MODES = [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF, panman_amd.MODE_BLOCK_FITCH,
         panman_amd.MODE_BLOCK_SANKOFF]


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _columns(rng, leaves, sites, block):
    if block:
        codes = rng.integers(0, 2, size=(leaves, sites)).astype(np.uint8)
    else:
        alphabet = np.array([1, 2, 4, 8, 1, 2, 4, 8, 0, 15, 5, 10], np.uint8)
        codes = alphabet[rng.integers(0, alphabet.size, size=(leaves, sites))]
    present = rng.random(leaves) >= 0.1
    return codes, present


def _load(engine, off, idx, root, codes, present, block, rng):
    n = off.shape[0] - 1
    node_row = np.full(n, -1, np.int32)
    for r, lid in enumerate(i for i in range(n) if off[i] == off[i + 1]):
        if present[r]:
            node_row[lid] = r
    engine.leaves_upload(codes, node_row)
    sites = codes.shape[1]
    cons = (np.zeros(sites, np.uint8) if block else np.array([1, 2, 4, 8], np.uint8)[rng.integers(0, 4, sites)])
    engine.sites_upload(cons.astype(np.uint8), None)


def _results(engine, mode):
    engine.run(mode)
    score, rootc = engine.site_results()
    return engine.mutations(), score, rootc


@pytest.mark.parametrize("mode", MODES)
def test_graph_matches_eager(engine, mode):
    block = mode in (panman_amd.MODE_BLOCK_FITCH, panman_amd.MODE_BLOCK_SANKOFF)
    rng = np.random.default_rng(100 + mode)
    off, idx, root = random_tree(300, rng, max_children=5)
    leaves = int((off[1:] == off[:-1]).sum())
    engine.tree_upload(off, idx, root)
    for step in range(3):   # new column data each step: the graph must see it
        codes, present = _columns(rng, leaves, 2500 + 700 * step, block)
        _load(engine, off, idx, root, codes, present, block, rng)
        engine.set_graph(False)
        want = _results(engine, mode)
        engine.set_graph(True)
        engine.set_profiling(True)
        for _ in range(2):   # capture, then replay
            got = _results(engine, mode)
            for g, w in zip(got, want):
                assert g.shape == w.shape and (g == w).all()
        ms, launches = engine.kernel_times()
        engine.set_profiling(False)
        assert launches[4] >= 1 and launches[0] == 0
    engine.set_graph(False)


def test_graph_follows_tree_change(engine):
    rng = np.random.default_rng(7)
    engine.set_graph(True)
    try:
        for leaves in (50, 400, 50):
            off, idx, root = random_tree(leaves, rng, max_children=3)
            engine.tree_upload(off, idx, root)
            codes, present = _columns(rng, leaves, 1000, False)
            _load(engine, off, idx, root, codes, present, False, rng)
            got = _results(engine, panman_amd.MODE_FITCH)
            engine.set_graph(False)
            want = _results(engine, panman_amd.MODE_FITCH)
            engine.set_graph(True)
            for g, w in zip(got, want):
                assert g.shape == w.shape and (g == w).all()
    finally:
        engine.set_graph(False)


def test_warmup_then_run_and_write_probe(engine):
    """pm_warmup (HIP initialisation + code objects, callable from any thread: the CLI's -I
    overlap) leaves the context working, and the write-only roof probe measures something
    plausible on the device."""
    import threading
    from panman_amd._lib import load
    rc = []
    t = threading.Thread(target=lambda: rc.append(load().pm_warmup(0)))
    t.start()
    t.join()
    assert rc == [0]
    assert load().pm_warmup(1 << 20) != 0   # no such device: an error, not a crash
    rng = np.random.default_rng(3)
    off, idx, root = random_tree(200, rng, max_children=4)
    leaves = int((off[1:] == off[:-1]).sum())
    engine.tree_upload(off, idx, root)
    codes, present = _columns(rng, leaves, 1500, False)
    _load(engine, off, idx, root, codes, present, False, rng)
    engine.set_graph(False)
    recs, score, rootc = _results(engine, panman_amd.MODE_FITCH)
    assert recs.shape[0] > 0 and score.shape[0] == 1500
    gbs = panman_amd.stream_write_rate(0, gib=1, reps=2)
    assert 100.0 < gbs < 20000.0


@pytest.mark.parametrize("mode", MODES)
def test_nt_load_builds_match(engine, mode):
    """The two builds of the passes (ordinary / non-temporal set-record loads, PM_OPT_NT_LOADS)
    give the same mutations, scores and root codes, with and without graph replay; small trees
    take the ordinary build by default, so the non-temporal one is forced here."""
    block = mode in (panman_amd.MODE_BLOCK_FITCH, panman_amd.MODE_BLOCK_SANKOFF)
    rng = np.random.default_rng(300 + mode)
    off, idx, root = random_tree(400, rng, max_children=6)
    leaves = int((off[1:] == off[:-1]).sum())
    engine.tree_upload(off, idx, root)
    codes, present = _columns(rng, leaves, 3000, block)
    _load(engine, off, idx, root, codes, present, block, rng)
    engine.set_graph(False)
    engine.set_nt_loads(0)
    want = _results(engine, mode)
    try:
        for graph in (False, True):
            engine.set_graph(graph)
            engine.set_nt_loads(1)
            got = _results(engine, mode)
            for g, w in zip(got, want):
                assert g.shape == w.shape and (g == w).all()
    finally:
        engine.set_nt_loads(-1)
        engine.set_graph(False)
