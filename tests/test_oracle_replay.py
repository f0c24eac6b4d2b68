"""Pin the replay oracle (printFASTAUltraFast restatement) against the survey's replay KATs
and the MSA -> PanMAT -> FASTA round trip."""
import json
import os

import numpy as np
import pytest

from _panmat import from_fixture, parse_records
from _trees import names_for, random_tree, to_newick, parse_newick
from panman_amd.panmat import from_msa_dump

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kats.json")
REPLAY = json.load(open(GOLDEN))["replay"]


@pytest.mark.parametrize("kat", REPLAY, ids=[k["id"] for k in REPLAY])
def test_replay_kats(oracle, kat):
    pm = from_fixture(kat)
    for aligned in (True, False):
        got = parse_records(oracle.fasta(pm, aligned))
        for name, exp in kat["expect"].items():
            key = "aligned" if aligned else "unaligned"
            if key in exp:
                assert got[name] == exp[key], (name, key, got[name])


def test_wrap_exact_multiple_of_70_gives_empty_line(oracle):
    from panman_amd.panmat import PanMAT
    names, off, idx, root = parse_newick("(a,b);")
    pm = PanMAT(names, off, idx, root)
    pm.add_block(0, "ACGT" * 35)   # 140 = 2 x 70
    pm.add_block_mut(root, 0, True, False)
    text = oracle.fasta(pm, True)
    assert text.startswith(">a\n" + "ACGT" * 17 + "AC\n" + "GT" + "ACGT" * 17 + "\n\n")


@pytest.mark.parametrize("seed", range(3))
def test_msa_round_trip_through_replay(oracle, seed):
    """MSA -> M1 (oracle) -> PanMAT -> aligned FASTA reproduces every input row."""
    rng = np.random.default_rng(seed)
    off, idx, root = random_tree(25, rng, max_children=3)
    names = names_for(off)
    nwk = to_newick(off, idx, root, names)
    sites = 180
    base = rng.choice(list("ACGT"), size=sites)
    rows = {}
    for i in range(len(names)):
        if off[i] == off[i + 1]:
            s = base.copy()
            f = rng.random(sites) < 0.2
            s[f] = rng.choice(list("ACGTN-RY"), size=f.sum())
            rows[names[i]] = "".join(s)
    msa = "".join(f">{k}\n{v}\n" for k, v in rows.items())
    dump = oracle.msa_build(nwk, msa, "", mode=seed % 2)
    pnames, poff, pidx, proot = parse_newick(nwk)
    pm = from_msa_dump(dump, pnames, poff, pidx, proot)
    got = parse_records(oracle.fasta(pm, True))
    assert got == rows
