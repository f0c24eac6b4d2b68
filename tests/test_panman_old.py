"""Older Protobuf PanMAN (panmanOld.treeGroup, /root/reference/panman.proto) reader
(pm_panman_load_old, SURVEY.md §8f-1 / the reference's --protobuf2capnp): a file encoded by
an independent encoder (tests/_protobuf.py) from a loaded .panman must load to the same
PanMAT as the .panman itself -- every array, and the same FASTA on the oracle.  Host only.
Parity with the protobuf library is unpinned (no library or fixture offline)."""
import random

import numpy as np
import pytest

from _panmat import parse_records, random_panmat
from _protobuf import encode_tree, encode_tree_group
from _trees import names_for, random_tree
from panman_amd import PanmanError
from panman_amd.panmat import PanmanFile, write_panman

ARRAYS = ["block_primary", "block_seq_offsets", "block_seq", "gap_primary", "gap_offsets", "gap_position",
          "gap_length", "block_mut_offsets", "block_mut_primary", "block_mut_info", "block_mut_inversion",
          "nuc_mut_offsets", "nuc_mut_primary", "nuc_mut_secondary", "nuc_mut_position",
          "nuc_mut_gap_position", "nuc_mut_info", "nuc_mut_nucs"]


def _same(p, q):
    assert p.names == q.names and p.root == q.root
    assert (p.child_offsets == q.child_offsets).all() and (p.child_index == q.child_index).all()
    for k in ARRAYS:
        assert np.array_equal(p._arrays[k], q._arrays[k]), k
    assert (p.circular == q.circular).all() and (p.rotation == q.rotation).all() and (p.inverted == q.inverted).all()


def _canonical(tmp_path, rng, n=30, trees=1):
    pms = []
    for _ in range(trees):
        off, idx, root_ = random_tree(n, rng, max_children=3, unary=0.1)
        pms.append(random_panmat(rng, off, idx, root_, names_for(off), blocks=int(rng.integers(1, 6))))
    path = str(tmp_path / "c.panman")
    write_panman(path, pms)
    return PanmanFile(path)


@pytest.mark.parametrize("seed", range(6))
def test_old_format_loads_like_capnp(tmp_path, oracle, seed):
    rng = np.random.default_rng(700 + seed)
    f = _canonical(tmp_path, rng, trees=1 + seed % 2)
    msgs = [encode_tree(f.to_panmat(i), f.newick(i), packed=seed % 3 != 0,
                        shuffle=random.Random(seed) if seed % 2 else None, extra_unknown=seed >= 3)
            for i in range(len(f))]
    old = str(tmp_path / "o.pb.xz")
    open(old, "wb").write(encode_tree_group(msgs, compress=seed != 4))
    g = PanmanFile(old, old=True)
    assert len(g) == len(f)
    for i in range(len(f)):
        want, got = f.to_panmat(i), g.to_panmat(i)
        _same(want, got)
        for aligned in (True, False):
            assert parse_records(oracle.fasta(got, aligned)) == parse_records(oracle.fasta(want, aligned))


def test_old_format_converts_to_capnp(tmp_path):
    """--protobuf2capnp: the old file written back as .panman equals the original tree."""
    rng = np.random.default_rng(5)
    f = _canonical(tmp_path, rng)
    old = str(tmp_path / "o.pb.xz")
    open(old, "wb").write(encode_tree_group([encode_tree(f.to_panmat(0), f.newick(0))]))
    g = PanmanFile(old, old=True)
    out = str(tmp_path / "back.panman")
    g.write(out)
    _same(f.to_panmat(0), PanmanFile(out).to_panmat(0))


@pytest.mark.parametrize("bad", [b"\x0a\x05abc", b"\x0a", b"\x0b\x00", b"\x00\x01", b""])
def test_old_format_rejects_corrupt(tmp_path, bad):
    p = str(tmp_path / "bad.pb")
    open(p, "wb").write(bad)
    with pytest.raises(PanmanError):
        PanmanFile(p, old=True)
