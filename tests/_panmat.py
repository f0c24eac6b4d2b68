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


def tree_dump(f, i: int = 0) -> str:
    """The oracle's reroot dump format for tree i of a PanmanFile: Newick, then per node in
    name order its block mutations (stored order) and NucMut records (list order)."""
    pm = f.to_panmat(i)
    a = pm._arrays
    out = ["newick\t" + f.newick(i)]
    for name in sorted(pm.names):
        v = pm.index(name)
        for k in range(a["block_mut_offsets"][v], a["block_mut_offsets"][v + 1]):
            out.append(f"{name}\tB\t{a['block_mut_primary'][k]}\t{a['block_mut_info'][k]}\t{a['block_mut_inversion'][k]}")
        for k in range(a["nuc_mut_offsets"][v], a["nuc_mut_offsets"][v + 1]):
            out.append(f"{name}\tN\t{a['nuc_mut_primary'][k]}\t{a['nuc_mut_position'][k]}\t"
                       f"{a['nuc_mut_gap_position'][k]}\t{a['nuc_mut_info'][k]}\t{int(a['nuc_mut_nucs'][k]):06x}")
    return "\n".join(out) + "\n"


def _parse_labelled(newick: str):
    """'(a:1,b:1)x:0;' with every node labelled -> (names, child lists, root) in pre-order."""
    s = newick.strip().rstrip(";")
    names, kids = [], []
    pos = 0

    def node():
        nonlocal pos
        me = len(names)
        names.append(None)
        kids.append([])
        if s[pos] == "(":
            pos += 1
            while True:
                kids[me].append(node())
                if s[pos] == ",":
                    pos += 1
                    continue
                assert s[pos] == ")"
                pos += 1
                break
        start = pos
        while pos < len(s) and s[pos] not in ",():":
            pos += 1
        names[me] = s[start:pos]
        if pos < len(s) and s[pos] == ":":
            pos += 1
            while pos < len(s) and s[pos] not in ",()":
                pos += 1
        return me

    root = node()
    return names, kids, root


def panmat_from_dump(dump: str, original: PanMAT) -> PanMAT:
    """Rebuild a PanMAT from a reroot dump plus the original's blocks, gaps and per-name
    rotation / inversion / circular offsets."""
    lines = dump.splitlines()
    assert lines[0].startswith("newick\t"), lines[0]
    names, kids, root = _parse_labelled(lines[0][7:])
    off = np.zeros(len(names) + 1, np.int32)
    idx = []
    for v in range(len(names)):
        idx += kids[v]
        off[v + 1] = len(idx)
    pm = PanMAT(names, off, np.array(idx, np.int32), root)
    a = getattr(original, "_arrays", None)
    assert a is None, "use a list-built PanMAT"
    pm.blocks = list(original.blocks)
    pm.gaps = list(original.gaps)
    by_name = {n: i for i, n in enumerate(original.names)}
    for v, n in enumerate(names):
        o = by_name.get(n)
        if o is not None and off[v] == off[v + 1]:
            pm.rotation[v] = original.rotation[o]
            pm.inverted[v] = original.inverted[o]
            pm.circular[v] = original.circular[o]
    for line in lines[1:]:
        f = line.split("\t")
        v = pm.index(f[0])
        if f[1] == "B":
            pm.add_block_mut(v, int(f[2]), f[3] == "1", f[4] == "1")
        else:
            pm.add_nuc_mut_raw(v, int(f[2]), int(f[3]), int(f[4]), int(f[5]), int(f[6], 16))
    return pm
