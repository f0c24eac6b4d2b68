"""The C++ facade include/panman_tree.hpp (panmanUtils::Tree / TreeGroup shape,
src/panman.hpp:819-1271), driven by bin/facade_demo the way a reference caller would:
every output must equal what the CLI (and therefore the C-ABI) produces."""
import os
import subprocess

import numpy as np
import pytest

from _panmat import parse_records, random_panmat
from _trees import names_for, parse_newick, random_tree, to_newick
from panman_amd.panmat import PanmanFile, write_panman
from test_cli import _msa_case, _run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "bin", "facade_demo")

pytestmark = pytest.mark.gpu


def _demo(args, cwd):
    if not os.path.exists(DEMO):
        pytest.fail(f"{DEMO} missing: run `make`")
    return subprocess.run([DEMO] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_facade_msa_build_equals_cli(tmp_path):
    rng = np.random.default_rng(31)
    nwk, rows = _msa_case(rng, 40, 333)
    (tmp_path / "t.nwk").write_text(nwk + "\n")
    (tmp_path / "a.fa").write_text("".join(f">{k}\n{v}\n" for k, v in rows.items()))
    r = _demo(["msa", "a.fa", "t.nwk", "f.panman"], tmp_path)
    assert r.returncode == 0, r.stderr
    c = _run(["-M", "a.fa", "-N", "t.nwk", "-o", "c"], tmp_path)
    assert c.returncode == 0, c.stderr
    a, b = PanmanFile(str(tmp_path / "f.panman")), PanmanFile(str(tmp_path / "panman" / "c.panman"))
    assert a.newick(0) == b.newick(0) == r.stdout.strip()
    a.close()
    b.close()
    fa = _demo(["fasta", "f.panman", "1"], tmp_path)
    assert fa.returncode == 0, fa.stderr
    assert parse_records(fa.stdout) == rows


def test_facade_fasta_summary_reroot(tmp_path, oracle):
    rng = np.random.default_rng(32)
    off, idx, root = random_tree(30, rng, max_children=3, unary=0.0)
    names, off, idx, root = parse_newick(to_newick(off, idx, root, names_for(off)))
    pm = random_panmat(rng, off, idx, root, names, blocks=4)
    write_panman(str(tmp_path / "in.panman"), [pm])
    for aligned in (0, 1):
        d = _demo(["fasta", "in.panman", str(aligned)], tmp_path)
        c = _run(["-I", "in.panman", "-m" if aligned else "-f"], tmp_path)
        assert d.returncode == 0 and c.returncode == 0
        text = c.stdout[c.stdout.index(">"):c.stdout.index("\nFASTA execution time")]
        assert d.stdout == text
    s = _demo(["summary", "in.panman"], tmp_path)
    assert s.returncode == 0, s.stderr
    out, rest = oracle.summary(pm)
    assert s.stdout == out + rest
    leaf = names[pm.leaves()[3]]
    r = _demo(["reroot", "in.panman", leaf, "rr.panman"], tmp_path)
    assert r.returncode == 0, r.stderr
    c = _run(["-I", "in.panman", "--reroot", "-n", leaf, "-d", "0", "-o", "rr"], tmp_path)
    assert c.returncode == 0, c.stderr
    a, b = PanmanFile(str(tmp_path / "rr.panman")), PanmanFile(str(tmp_path / "panman" / "rr.panman"))
    assert a.newick(0) == b.newick(0)
    a.close()
    b.close()
    d1 = _demo(["fasta", "rr.panman", "1"], tmp_path)
    d0 = _demo(["fasta", "in.panman", "1"], tmp_path)
    assert parse_records(d1.stdout) == parse_records(d0.stdout)


def test_facade_errors_are_exceptions(tmp_path):
    (tmp_path / "bad.panman").write_bytes(b"\xfd7zXZ\x00garbage")
    r = _demo(["fasta", "bad.panman", "0"], tmp_path)
    assert r.returncode == 1 and "Error" in r.stderr
