"""Oracle restatement of Tree::reroot (src/reroot.cpp:4-262), pinned by properties: no
reference fixture exists for reroot, so the restatement is checked by (i) every leaf's
FASTA record (aligned and unaligned) being unchanged by rerooting, (ii) the new root
being adjacent to the chosen leaf with that leaf carrying no mutations, and (iii) the
root's old-child rule (parent already root: topology unchanged)."""
import numpy as np
import pytest

from _panmat import _parse_labelled, panmat_from_dump, random_panmat
from _trees import names_for, parse_newick, random_tree, to_newick


def _case(seed, leaves=24, blocks=4):
    rng = np.random.default_rng(seed)
    off, idx, root = random_tree(leaves, rng, max_children=3, unary=0.0)
    # reference naming (node_1.. in pre-order), as a loaded PanMAN has
    names, off, idx, root = parse_newick(to_newick(off, idx, root, names_for(off)))
    pm = random_panmat(rng, off, idx, root, names, blocks=blocks)
    leaf_names = [names[v] for v in pm.leaves()]
    return rng, pm, leaf_names


@pytest.mark.parametrize("seed", range(6))
def test_reroot_preserves_every_leaf_sequence(oracle, seed):
    rng, pm, leaf_names = _case(500 + seed)
    leaf = leaf_names[int(rng.integers(len(leaf_names)))]
    dump = oracle.reroot(pm, leaf)
    assert not dump.startswith("#error"), dump
    back = panmat_from_dump(dump, pm)
    for aligned in (True, False):
        assert oracle.fasta(back, aligned) == oracle.fasta(pm, aligned)
    names, kids, root = _parse_labelled(dump.splitlines()[0][7:])
    child_names = [names[c] for c in kids[root]]
    assert leaf in child_names
    assert not any(line.startswith(leaf + "\t") for line in dump.splitlines()[1:])


def _leaf_under_root(seed0):
    for seed in range(seed0, seed0 + 50):
        rng, pm, leaf_names = _case(seed, leaves=6)
        kids_of_root = pm.child_index[pm.child_offsets[pm.root]:pm.child_offsets[pm.root + 1]]
        for c in kids_of_root:
            if pm.child_offsets[c] == pm.child_offsets[c + 1]:
                return pm, pm.names[c]
    raise AssertionError("no tree with a leaf under the root")


def test_reroot_at_child_of_root_keeps_topology(oracle):
    pm, leaf = _leaf_under_root(77)
    dump = oracle.reroot(pm, leaf)
    names, kids, root = _parse_labelled(dump.splitlines()[0][7:])
    assert names[root] == pm.names[pm.root] and len(names) == pm.num_nodes
    back = panmat_from_dump(dump, pm)
    assert oracle.fasta(back, True) == oracle.fasta(pm, True)


def test_reroot_errors(oracle):
    _, pm, _ = _case(3)
    assert oracle.reroot(pm, "nope").startswith("#error\tSequence with name nope not found!")
    assert oracle.reroot(pm, pm.names[pm.root]).startswith("#error\tNode with id")
