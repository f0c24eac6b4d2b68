"""Test helpers: Newick -> CSR with the reference's node naming, random trees and MSAs."""
from __future__ import annotations

import numpy as np

CODE = {c: i for i, c in enumerate("-ACMGRSVTWYHKDBN")}
CHAR = "-ACMGRSVTWYHKDBN"


def parse_newick(text: str):
    """Minimal Newick parser (no quotes) naming internal nodes node_<k> in order of '('
    like src/panman.cpp:310-450.  Returns names, child_offsets, child_index, root."""
    names, kids, stack = [], [], []
    tok = ""
    k = 0

    def add(name):
        names.append(name)
        kids.append([])
        nid = len(names) - 1
        if stack:
            kids[stack[-1]].append(nid)
        return nid

    i = 0
    text = text.strip().rstrip(";")
    after_close = False
    while i < len(text):
        c = text[i]
        if c == "(":
            k += 1
            stack.append(add(f"node_{k}"))
            after_close = False
        elif c in ",)":
            if tok and not after_close:
                add(tok)
            tok = ""
            if c == ")":
                stack.pop()
                after_close = True
            else:
                after_close = False
        elif c == ":":
            while i + 1 < len(text) and text[i + 1] not in ",)":
                i += 1
        else:
            if not after_close:
                tok += c
        i += 1
    off = np.zeros(len(names) + 1, np.int32)
    idx = []
    for n, ch in enumerate(kids):
        idx += ch
        off[n + 1] = len(idx)
    return names, off, np.array(idx, np.int32), 0


def random_tree(leaves: int, rng, max_children: int = 4, unary: float = 0.05):
    """Random rooted tree with polytomies and unary nodes; leaves are ids [0, leaves)."""
    pool = list(range(leaves))
    kids = {}
    nxt = leaves
    while len(pool) > 1:
        k = int(rng.integers(2, max_children + 1))
        k = min(k, len(pool))
        pick = rng.choice(len(pool), size=k, replace=False)
        chosen = [pool[p] for p in pick]
        for p in sorted(pick, reverse=True):
            pool.pop(p)
        kids[nxt] = chosen
        node = nxt
        nxt += 1
        if rng.random() < unary:
            kids[nxt] = [node]
            node = nxt
            nxt += 1
        pool.append(node)
    n = nxt
    off = np.zeros(n + 1, np.int32)
    idx = []
    for v in range(n):
        idx += kids.get(v, [])
        off[v + 1] = len(idx)
    return off, np.array(idx, np.int32), pool[0]


def names_for(off) -> list[str]:
    n = off.shape[0] - 1
    return [f"s{i}" if off[i] == off[i + 1] else f"node_{i}" for i in range(n)]


def to_newick(off, idx, root, names) -> str:
    def rec(v):
        ch = idx[off[v]:off[v + 1]]
        if len(ch) == 0:
            return names[v]
        return "(" + ",".join(rec(c) for c in ch) + ")"
    import sys
    sys.setrecursionlimit(100000)
    return rec(root) + ";"
