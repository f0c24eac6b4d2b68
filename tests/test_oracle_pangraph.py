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
