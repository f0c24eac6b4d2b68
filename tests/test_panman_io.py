"""PanMAN file IO (next row SURVEY.md §8f-1): writer/reader round trip, layout checked by an
independent decoder, corrupt input rejected.  Host-only (no GPU).  Parity with the
reference's capnp library is unpinned: no .panman fixture exists offline."""
import os

import numpy as np
import pytest

from _capnp import LAYOUT, root
from _panmat import parse_records, random_panmat
from _trees import names_for, random_tree
from panman_amd.panmat import PanmanFile, write_panman


def test_layout_matches_survey_derivation():
    nuc, dw, pc = LAYOUT["NucMut"]
    assert (nuc["nucPosition"], nuc["nucGapPosition"], nuc["nucGapExist"], nuc["mutInfo"], dw, pc) == \
        (0, 32, 64, 96, 2, 0)
    mu, dw, pc = LAYOUT["Mutation"]
    assert (mu["blockId"], mu["blockGapExist"], mu["blockMutExist"], mu["blockMutInfo"], mu["blockInversion"],
            dw, pc) == (0, 64, 65, 66, 67, 2, 1)
    assert LAYOUT["GapList"][1:] == (2, 2) and LAYOUT["CircularOffset"][1:] == (1, 1)
    assert LAYOUT["Tree"][1:] == (0, 8)


@pytest.mark.parametrize("seed", range(4))
def test_round_trip_replays_identically(tmp_path, oracle, seed):
    rng = np.random.default_rng(40 + seed)
    off, idx, root_ = random_tree(30, rng, max_children=3, unary=0.1)
    pm = random_panmat(rng, off, idx, root_, names_for(off), blocks=int(rng.integers(1, 6)))
    path = str(tmp_path / "t.panman")
    write_panman(path, [pm], compress=bool(seed % 2 == 0))
    f = PanmanFile(path)
    assert len(f) == 1
    back = f.to_panmat(0)
    for aligned in (True, False):
        assert parse_records(oracle.fasta(back, aligned)) == parse_records(oracle.fasta(pm, aligned))


def test_independent_decoder_reads_fields(tmp_path):
    rng = np.random.default_rng(3)
    off, idx, root_ = random_tree(12, rng, max_children=2)
    pm = random_panmat(rng, off, idx, root_, names_for(off), blocks=3)
    path = str(tmp_path / "t.panman")
    write_panman(path, [pm])
    tg = root(open(path, "rb").read())
    trees = tg.items("trees", "Tree")
    assert len(trees) == 1 and tg.items("complexMutations", "ComplexMutation") == []
    t = trees[0]
    assert t.text("newick").endswith(";")
    nodes = t.items("nodes", "Node")
    assert len(nodes) == pm.num_nodes + 1          # trailing empty node, as the reference writes
    # every nucleotide mutation of the file decodes to one of the PanMAT's records
    want = set()
    for lst in pm.nuc_muts:
        for prim, sec, pos, gap, info, nucs in lst:
            ln = info >> 4
            want.add((prim, pos, gap, ((nucs >> (24 - 4 * ln)) << 8) + info))
    got = set()
    for node in nodes:
        for m in node.items("mutations", "Mutation"):
            prim = m.bits("blockId", 64) >> 32
            for nm in m.items("nucMutation", "NucMut"):
                gap = nm.bits("nucGapPosition", 32, True) if nm.bits("nucGapExist", 1) else -1
                got.add((prim, nm.bits("nucPosition", 32, True), gap, nm.bits("mutInfo", 32)))
    assert got == want
    blocks = t.items("consensusSeqMap", "ConsensusSeqToBlockIds")
    ids = sorted(i >> 32 for c in blocks for i in c.items("blockId"))
    assert ids == sorted(p for p, _ in pm.blocks)


def test_corrupt_files_are_errors(tmp_path):
    import panman_amd
    bad = tmp_path / "bad.panman"
    bad.write_bytes(b"\xfd7zXZ\x00garbage")
    with pytest.raises(panman_amd.PanmanError):
        PanmanFile(str(bad))
    trunc = tmp_path / "trunc.panman"
    trunc.write_bytes(b"\x00\x00\x00\x00\xff\x00\x00\x00" + b"\x00" * 16)
    with pytest.raises(panman_amd.PanmanError):
        PanmanFile(str(trunc))
