"""Pin the CPU oracle against the reference's known answers (SURVEY.md §8a')."""
import json
import os

import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kats.json")
KATS = json.load(open(GOLDEN))["column"]


@pytest.mark.parametrize("kat", KATS, ids=[k["id"] for k in KATS])
def test_column_kat(oracle, kat):
    got = oracle.column(kat["newick"], kat["leaves"], kat["algo"], kat["forced"], kat["parent"])
    exp = kat["expect"]
    for name, v in exp.get("fwd", {}).items():
        assert got["fwd"][name] == v, (name, got["fwd"])
    for name, v in exp.get("final", {}).items():
        assert got["final"][name] == v, (name, got["final"])
    assert got["muts"] == {k: list(v) for k, v in exp["muts"].items()}
