"""Oracle restatement of the PanGraph driver (M3, src/panman.cpp:820-1273) pinned by the
survey's runs of the compiled reference on test/sars_20: 39 nodes,
10 blocks, 12 block mutations, and 1343 NucMut records with oneTBB's iteration order of
individualSequences (1301 with a std::unordered_map in its place)."""
import json
import os

import pytest

from _pangraph import flatten

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def sars20():
    d = json.load(open(os.path.join(GOLD, "sars_20.json")))
    return flatten(d), open(os.path.join(GOLD, "sars_20.nwk")).read()


def _counts(dump):
    lines = dump.splitlines()
    return (sum(line.startswith("block\t") for line in lines), sum("\tB\t" in line for line in lines),
            sum("\tN\t" in line for line in lines))


def test_sars20_counts_tbb_order(oracle, sars20):
    assert _counts(oracle.pangraph(*sars20)) == (10, 12, 1343)


def test_sars20_counts_std_order(oracle, sars20):
    assert _counts(oracle.pangraph(*sars20, tbb_order=False)) == (10, 12, 1301)


def test_sars20_node_count(oracle, sars20):
    nwk = sars20[1]
    assert nwk.count("(") == 19 and nwk.count(",") == 19   # 20 leaves + 19 internal = 39 nodes


def test_random_pangraphs_run_on_oracle(oracle):
    """The synthetic generator produces inputs the restatement accepts (GPU parity uses them)."""
    import numpy as np
    from _pangraph import random_pangraph
    from _trees import random_tree, to_newick
    for seed in range(4):
        rng = np.random.default_rng(seed)
        text, names = random_pangraph(rng, circular=seed % 2 == 1)
        off, idx, root = random_tree(len(names), rng, max_children=2 + seed % 2, unary=0.0)
        nm = [names[i] if off[i] == off[i + 1] else "" for i in range(len(off) - 1)]
        dump = oracle.pangraph(flatten(json.loads(text)), to_newick(off, idx, root, nm) + ";")
        assert not dump.startswith("#error") and dump.count("block\t") >= 1


def _genomes():
    want, name = {}, None
    for line in open(os.path.join(GOLD, "sars_20.fa")):
        line = line.strip()
        if line.startswith(">"):
            name = line[1:]
            want[name] = ""
        elif line:
            want[name] += line.upper()
    return want


@pytest.mark.parametrize("tbb_order", [True, False])
def test_sars20_built_tree_replays_input_genomes(oracle, sars20, tbb_order):
    """Pins the oracle to the reference's own genomes: the oracle's PanGraph driver (M3,
    src/panman.cpp:820-1273) on test/sars_20.{json,nwk}, then the oracle's unaligned
    printFASTAUltraFast (R1-R3, src/fasta.cpp:1981-2099, :155-254) on the Tree it built,
    gives back test/sars_20.fa record for record (sequences uppercased, as the driver
    uppercases its input, src/panman.cpp:6221-6247) -- under either iteration order."""
    from _panmat import parse_records
    got = parse_records(oracle.pangraph_fasta(*sars20, tbb_order=tbb_order, aligned=False))
    want = _genomes()
    assert set(got) == set(want)
    for name in want:
        assert got[name] == want[name], name


def test_sars20_aligned_rows_share_one_width(oracle, sars20):
    """The aligned records of the same build are one MSA: equal widths, and with the gap
    characters removed each row is its input genome."""
    from _panmat import parse_records
    got = parse_records(oracle.pangraph_fasta(*sars20, aligned=True))
    want = _genomes()
    assert len({len(v) for v in got.values()}) == 1
    for name, row in got.items():
        assert row.replace("-", "") == want[name]
