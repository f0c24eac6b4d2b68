"""`--summary` (Tree::printSummary, src/summary.cpp:257-273): the oracle restatement is
cross-checked here against an independent straight-line count on random PanMATs (CPU);
the GPU reduction (pm_summary_compute) and the CLI text must equal the oracle's.  No
reference fixture exists for this command (parity anchored on the restatement)."""
import os
import subprocess

import numpy as np
import pytest

from _panmat import random_panmat
from _trees import names_for, random_tree
from panman_amd.panmat import write_panman

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "panmanUtils")


def _with_duplicates(rng, pm, blocks):
    """Add copies of existing blocks (identical consensusSeq) and insert / delete them
    along the tree, so duplications and translocations occur."""
    seqs = {b: s for b, s in pm.blocks}
    nb = blocks
    for src in range(min(3, blocks)):
        for _ in range(2):
            pm.blocks.append((nb, list(seqs[src])))
            nb += 1
    n = len(pm.names)
    for v in range(n):
        if rng.random() < 0.3:
            b = int(rng.integers(0, nb))
            pm.add_block_mut(v, b, bool(rng.random() < 0.6), bool(rng.random() < 0.3))
        if v != pm.root and rng.random() < 0.15:   # a block moved to its copy: translocation
            src = int(rng.integers(0, min(3, blocks)))
            pm.add_block_mut(v, src, False, False)
            pm.add_block_mut(v, blocks + 2 * src + int(rng.integers(0, 2)), True, False)
    return pm


def _cases(k=6):
    out = []
    for seed in range(k):
        rng = np.random.default_rng(100 + seed)
        off, idx, root = random_tree(int(rng.integers(5, 60)), rng, max_children=4)
        pm = random_panmat(rng, off, idx, root, names_for(off), blocks=5)
        out.append(_with_duplicates(rng, pm, 5))
    return out


def _straight_count(pm):
    """printSummary's counts written out plainly from the PanMAT lists (independent of the
    oracle's code): NucMut (primary, secondary, pos, gap, info, nucs), BlockMut (primary,
    insertion, inversion)."""
    n = len(pm.names)
    nm = [m for lst in pm.nuc_muts for m in lst]
    bm = [m for lst in pm.block_muts for m in lst]
    ns = sum(m[4] >> 4 for m in nm if m[4] & 7 == 0)
    ni = sum(1 for m in nm if m[4] & 7 == 2)
    nd = sum(1 for m in nm if m[4] & 7 == 1)
    bi = sum(1 for m in bm if m[1])
    bd = sum(1 for m in bm if not m[1] and not m[2])
    inv = sum(1 for m in bm if m[2])
    bdi = sum(1 for m in bm if not m[1] and m[2])
    off = pm.child_offsets
    depth = np.zeros(n, np.int64)
    order = [pm.root]
    for v in order:
        for c in pm.child_index[off[v]:off[v + 1]]:
            depth[c] = depth[v] + 1
            order.append(int(c))
    leaves = [v for v in range(n) if off[v] == off[v + 1]]
    return {"nodes": n, "samples": len(leaves), "substitutions": ns, "insertions": ni + bi, "deletions": nd + bd,
            "inversions": inv, "max_depth": int(depth[leaves].max()), "block_insertions": bi,
            "block_deletions": bd, "block_inversions": bdi}


def _parse(out_text, cout_text):
    d = {}
    for line in (out_text + cout_text).splitlines():
        k, _, v = line.partition(": ")
        d[k] = v
    return d


KEYS = {"nodes": "Total Nodes in Tree", "samples": "Total Samples in Tree", "substitutions": "Total Substitutions",
        "insertions": "Total Insertions", "deletions": "Total Deletions", "inversions": "Total Inversions",
        "max_depth": "Max Tree Depth", "block_insertions": "Total Block Insertions",
        "block_deletions": "Total Block Deletions", "block_inversions": "Total Block Inversion"}


def test_oracle_summary_matches_straight_count(oracle):
    for pm in _cases():
        out, rest = oracle.summary(pm)
        got = _parse(out, rest)
        want = _straight_count(pm)
        for k, label in KEYS.items():
            assert int(got[label]) == want[k], (k, got[label], want[k])
        assert "Mean Tree Depth" in got and "Total Block Duplications" in got and "Total Block Translocation" in got


@pytest.mark.gpu
def test_gpu_summary_equals_oracle(oracle):
    import panman_amd
    eng = panman_amd.Engine(0)
    for pm in _cases():
        out, rest = oracle.summary(pm)
        want = _parse(out, rest)
        s = eng.summary(pm)
        assert str(s["nodes"]) == want["Total Nodes in Tree"]
        assert str(s["block_duplications"]) == want["Total Block Duplications"]
        assert str(s["block_translocations"]) == want["Total Block Translocation"]
        for k, label in KEYS.items():
            assert str(s[k]) == want[label], k
    eng.close()


@pytest.mark.gpu
def test_cli_summary_text_equals_oracle(oracle, tmp_path):
    pms = _cases(3)
    path = str(tmp_path / "in.panman")
    write_panman(path, pms)
    r = subprocess.run([CLI, "-I", path, "--summary", "-o", "s"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    from panman_amd.panmat import PanmanFile
    f = PanmanFile(path)
    cout = ""
    for i in range(3):
        out, rest = oracle.summary(f.to_panmat(i))
        assert open(tmp_path / "info" / f"s_{i}.summary").read() == out
        cout += rest
    f.close()
    assert cout in r.stdout and "Summary creation time:" in r.stdout
    # without -o the summary goes to stdout (src/panmanUtils.cpp:367-373)
    r = subprocess.run([CLI, path, "-s"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "Total Nodes in Tree:" in r.stdout
