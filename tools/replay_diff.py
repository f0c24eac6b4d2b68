"""Diagnostic: C5-like PanMAT (the replay bench workload), GPU FASTA records of the first
K leaves by name vs the oracle restatement; prints the leaves that differ and the first
differing position.  Usage: PYTHONPATH=.:oracle python tools/replay_diff.py [K] [leaves]"""
import sys

import torch  # noqa: F401

import oracle as orc
import panman_amd
from panman_amd.synth import c5_panmat

K = int(sys.argv[1]) if len(sys.argv) > 1 else 128
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
pm = c5_panmat(leaves=L)
e = panman_amd.Engine(0)
got = e.fasta(pm, True)
want = orc.load().fasta(pm, True, leaf_limit=K)


def records(text):
    out = {}
    for rec in text.split(">")[1:]:
        name, _, body = rec.partition("\n")
        out[name] = body
    return out


g, w = records(got), records(want)
bad = [n for n in w if g.get(n) != w[n]]
print(f"{len(w)} oracle records, {len(bad)} differ")
for n in bad[:5]:
    a, b = g.get(n, ""), w[n]
    i = next((k for k in range(min(len(a), len(b))) if a[k] != b[k]), min(len(a), len(b)))
    print(n, "len", len(a), len(b), "first diff at", i, "gpu", repr(a[max(0, i - 20):i + 20]), "oracle", repr(b[max(0, i - 20):i + 20]))
