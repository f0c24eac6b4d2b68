"""GPU PanGraph driver (M3): pm_pangraph_build vs the oracle restatement record for record on
test/sars_20 (TBB-order contract), plus the end-to-end property that the built PanMAN
replays every input genome (test/sars_20.fa) exactly."""
import json
import os

import pytest

import panman_amd
from _pangraph import flatten, m3_dump
from _panmat import parse_records

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def sars20():
    text = open(os.path.join(GOLD, "sars_20.json")).read()
    return text, json.loads(text), open(os.path.join(GOLD, "sars_20.nwk")).read()


def test_sars20_matches_oracle(engine, oracle, sars20):
    text, d, nwk = sars20
    f = engine.pangraph_build(text, nwk)
    try:
        assert m3_dump(f) == oracle.pangraph(flatten(d), nwk)
    finally:
        f.close()


def test_sars20_with_reference_matches_oracle(engine, oracle, sars20):
    text, d, nwk = sars20
    ref = d["paths"][3]["name"][:12]
    f = engine.pangraph_build(text, nwk, ref)
    try:
        assert m3_dump(f) == oracle.pangraph(flatten(d), nwk, ref)
    finally:
        f.close()


def test_sars20_replays_input_genomes(engine, sars20, tmp_path):
    text, d, nwk = sars20
    f = engine.pangraph_build(text, nwk)
    path = str(tmp_path / "s.panman")
    f.write(path)
    f.close()
    g = panman_amd.PanmanFile(path)
    try:
        got = parse_records(engine.fasta(g.view(0), False))
    finally:
        g.close()
    want = {}
    name = None
    for line in open(os.path.join(GOLD, "sars_20.fa")):
        line = line.strip()
        if line.startswith(">"):
            name = line[1:]
            want[name] = ""
        elif line:
            want[name] += line.upper()
    assert set(got) == set(want)
    assert got == want


@pytest.mark.parametrize("seed", range(16))
def test_random_pangraph_matches_oracle(engine, oracle, seed):
    """Binary trees (Fitch) and polytomies (Sankoff), linear and circular paths, duplicated
    and reversed blocks, with and without a reference name."""
    import numpy as np
    from _pangraph import random_pangraph
    from _trees import random_tree, to_newick
    rng = np.random.default_rng(100 + seed)
    text, names = random_pangraph(rng, seqs=10 + seed, circular=seed % 4 >= 2)
    off, idx, root = random_tree(len(names), rng, max_children=2 if seed % 2 == 0 else 4, unary=0.0)
    nm = [names[i] if off[i] == off[i + 1] else "" for i in range(len(off) - 1)]
    nwk = to_newick(off, idx, root, nm)
    ref = names[seed % len(names)][:5] if seed % 3 == 0 else ""
    f = engine.pangraph_build(text, nwk, ref)
    try:
        assert m3_dump(f) == oracle.pangraph(flatten(json.loads(text)), nwk, ref)
    finally:
        f.close()
