"""Build PanMATs for replay tests: from the KAT fixtures, and random block PanMATs."""
from __future__ import annotations

import numpy as np

from _trees import parse_newick
from panman_amd.panmat import PanMAT


def from_fixture(k) -> PanMAT:
    names, off, idx, root = parse_newick(k["newick"])
    pm = PanMAT(names, off, idx, root)
    for b, seq in k["blocks"]:
        pm.add_block(b, seq)
    for b, slots in k["gaps"]:
        pm.add_gaps(b, [tuple(s) for s in slots])
    for node, lst in k["block_muts"].items():
        for b, ins, inv in lst:
            pm.add_block_mut(pm.index(node), b, bool(ins), bool(inv))
    for node, lst in k["nuc_muts"].items():
        for b, pos, gap, typ, codes in lst:
            pm.add_nuc_mut(pm.index(node), b, pos, gap, typ, codes)
    for node, v in k["rotation"].items():
        pm.rotation[pm.index(node)] = v
    for node, v in k["inverted"].items():
        pm.inverted[pm.index(node)] = v
    for node, v in k["circular"].items():
        pm.circular[pm.index(node)] = v
    return pm


def parse_records(text: str) -> dict[str, str]:
    """FASTA records -> {name: sequence with newlines removed}; checks the 70-column wrap."""
    out = {}
    for rec in text.split(">")[1:]:
        head, _, body = rec.partition("\n")
        lines = body.split("\n")
        assert lines[-1] == "" and lines[-2] == "" or body.endswith("\n"), rec
        out[head] = body.replace("\n", "")
    return out


BASES = "ACGT"


def random_panmat(rng, off, idx, root, names, blocks=6, block_len=(5, 40), gap_rate=0.2, mut_rate=0.05,
                  block_rate=0.1, options=True) -> PanMAT:
    """Random PanMAT exercising blocks, gap slots, MNPs of every type, block insertions,
    deletions and inversions, rotation / inversion / circular offsets at leaves."""
    pm = PanMAT(names, off, idx, root)
    n = len(names)
    lens = []
    for b in range(blocks):
        L = int(rng.integers(*block_len))
        lens.append(L)
        pm.add_block(b, "".join(rng.choice(list(BASES), size=L)))
        if rng.random() < 0.7:
            pos = sorted(set(rng.integers(0, L + 1, size=int(rng.integers(1, 4))).tolist()))
            pm.add_gaps(b, [(p, int(rng.integers(1, 5))) for p in pos])
    gaplen = {}
    for b, slots in pm.gaps:
        for p, l in slots:
            gaplen[(b, p)] = l
    # root inserts most blocks
    for b in range(blocks):
        if rng.random() < 0.85:
            pm.add_block_mut(root, b, True, bool(rng.random() < 0.2))
    for v in range(n):
        if v != root and rng.random() < block_rate:
            b = int(rng.integers(0, blocks))
            kind = rng.integers(0, 3)
            pm.add_block_mut(v, b, kind == 0, kind != 1)
        k = rng.poisson(mut_rate * sum(lens))
        for _ in range(k):
            b = int(rng.integers(0, blocks))
            typ = int(rng.choice([0, 1, 2, 3, 4, 5]))
            if rng.random() < 0.3:
                gp = [p for (bb, p) in gaplen if bb == b]
                if not gp:
                    continue
                p = int(rng.choice(gp))
                g = int(rng.integers(0, gaplen[(b, p)]))
                ln = 1 if typ >= 3 else int(rng.integers(1, gaplen[(b, p)] - g + 1))
                pos, gap = p, g
            else:
                ln = 1 if typ >= 3 else int(rng.integers(1, 7))
                pos = int(rng.integers(0, max(1, lens[b] - ln + 1)))
                ln = min(ln, lens[b] - pos)
                if ln <= 0:
                    continue
                gap = -1
            codes = [0 if typ in (1, 5) else int(rng.choice([1, 2, 4, 8, 15, 5])) for _ in range(ln)]
            pm.add_nuc_mut(v, b, pos, gap, typ, codes)
    if options:
        for v in pm.leaves():
            r = rng.random()
            if r < 0.15:
                pm.rotation[v] = int(rng.integers(1, 4))
            elif r < 0.3:
                pm.inverted[v] = 1
            elif r < 0.45:
                pm.circular[v] = int(rng.integers(0, 30))
    return pm
