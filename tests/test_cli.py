"""panmanUtils-compatible CLI (bin/panmanUtils, src/panmanUtils.cpp:128-182, :271-299,
:385-490, :766-786).  Host commands run here; -M builds and -f/-m replays need the GPU."""
import os
import subprocess

import numpy as np
import pytest

from _panmat import parse_records, random_panmat
from _trees import names_for, random_tree, to_newick
from panman_amd.panmat import PanmanFile, write_panman

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "panmanUtils")


def _run(args, cwd):
    if not os.path.exists(CLI):
        pytest.fail(f"{CLI} missing: run `make`")
    return subprocess.run([CLI] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_help_and_unknown_commands(tmp_path):
    r = _run(["-h"], tmp_path)
    assert r.returncode == 0 and "--input-panman" in r.stdout and "--fasta-aligned" in r.stdout
    r = _run(["x.panman", "--vcf"], tmp_path)
    assert r.returncode != 0 and "not part of the GPU path" in r.stderr
    r = _run(["--bogus"], tmp_path)
    assert r.returncode != 0 and "unrecognised option" in r.stderr
    r = _run(["-M", "a.fa", "-o", "x"], tmp_path)
    assert r.returncode != 0 and "newick string not provided" in r.stderr


def test_backend_and_gpus_arguments(tmp_path):
    r = _run(["--backend", "cpu", "-I", "x.panman"], tmp_path)
    assert r.returncode == 1 and "GPU only" in r.stderr
    r = _run(["--gpus", "0", "-I", "x.panman"], tmp_path)
    assert r.returncode == 1 and "--gpus" in r.stderr


def test_newick_to_info_file_and_stdout(tmp_path):
    rng = np.random.default_rng(3)
    off, idx, root = random_tree(25, rng, max_children=3)
    pm = random_panmat(rng, off, idx, root, names_for(off), blocks=2)
    path = str(tmp_path / "in.panman")
    write_panman(path, [pm, pm])
    f = PanmanFile(path)
    want = [f.newick(0), f.newick(1)]
    f.close()
    r = _run(["-I", path, "-t", "-o", "out"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Data load time:" in r.stdout
    for i in range(2):
        assert open(tmp_path / "info" / f"out_{i}.newick").read() == want[i] + "\n"
    r = _run([path, "--newick"], tmp_path)   # positional input file, output to stdout
    assert r.returncode == 0 and r.stdout.count(want[0] + "\n") == 2


def test_corrupt_input_is_an_error(tmp_path):
    p = tmp_path / "bad.panman"
    p.write_bytes(b"\xfd7zXZ\x00garbage")
    r = _run(["-I", str(p), "-t"], tmp_path)
    assert r.returncode != 0 and "Error" in r.stderr


def _msa_case(rng, n, width):
    off, idx, root = random_tree(n, rng, max_children=3)
    names = names_for(off)
    base = rng.choice(list("ACGT"), size=width)
    rows = {}
    for i in range(len(names)):
        if off[i] == off[i + 1]:
            s = base.copy()
            f = rng.random(width) < 0.12
            s[f] = rng.choice(list("ACGTN-"), size=f.sum())
            rows[names[i]] = "".join(s)
    return to_newick(off, idx, root, names), rows


@pytest.mark.gpu
@pytest.mark.parametrize("low_mem", [False, True])
def test_msa_build_then_fasta(tmp_path, low_mem):
    rng = np.random.default_rng(12 + low_mem)
    nwk, rows = _msa_case(rng, 45, 401)
    (tmp_path / "t.nwk").write_text(nwk + "\n")
    (tmp_path / "a.fa").write_text("".join(f">{k}\n{v}\n" for k, v in rows.items()))
    args = ["-M", "a.fa", "-N", "t.nwk", "-o", "demo"]
    if low_mem:
        args += ["--low-mem-mode", "-n", next(iter(rows))]
    r = _run(args, tmp_path)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(tmp_path / "panman" / "demo.panman")
    r = _run(["-I", "panman/demo.panman", "-m", "-o", "demo"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert parse_records(open(tmp_path / "info" / "demo_0.msa").read()) == rows
    r = _run(["-I", "panman/demo.panman", "-f"], tmp_path)
    assert r.returncode == 0, r.stderr
    text = r.stdout[r.stdout.index(">"):r.stdout.index("\nFASTA execution time")]
    assert parse_records(text) == {k: v.replace("-", "") for k, v in rows.items()}


@pytest.mark.gpu
def test_reroot_command(tmp_path):
    """--reroot -n <leaf> -d 0 -o out writes ./panman/out.panman whose FASTA equals the
    input's (rerooting re-derives mutations, sequences are unchanged)."""
    from _panmat import random_panmat
    from _trees import parse_newick
    rng = np.random.default_rng(21)
    off, idx, root = random_tree(30, rng, max_children=3, unary=0.0)
    names, off, idx, root = parse_newick(to_newick(off, idx, root, names_for(off)))
    pm = random_panmat(rng, off, idx, root, names, blocks=4)
    write_panman(str(tmp_path / "in.panman"), [pm, pm])
    leaf = names[pm.leaves()[5]]
    r = _run(["-I", "in.panman", "--reroot", "-n", leaf, "-d", "1", "-o", "rr"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Reroot execution time" in r.stdout
    f = PanmanFile(str(tmp_path / "panman" / "rr.panman"))
    assert len(f) == 2
    nw0, nw1 = f.newick(0), f.newick(1)
    f.close()
    assert f"{leaf}:0.000000" in nw1 and f"{leaf}:0.000000" not in nw0
    a = _run(["-I", "in.panman", "-m", "-o", "a"], tmp_path)
    b = _run(["-I", "panman/rr.panman", "-m", "-o", "b"], tmp_path)
    assert a.returncode == 0 and b.returncode == 0
    for i in range(2):
        ra = parse_records(open(tmp_path / "info" / f"a_{i}.msa").read())
        rb = parse_records(open(tmp_path / "info" / f"b_{i}.msa").read())
        assert ra == rb


def test_reroot_command_arguments(tmp_path):
    rng = np.random.default_rng(2)
    off, idx, root = random_tree(8, rng, max_children=3)
    pm = random_panmat(rng, off, idx, root, names_for(off), blocks=2)
    write_panman(str(tmp_path / "in.panman"), [pm])
    r = _run(["-I", "in.panman", "--reroot", "-n", "s1", "-o", "x"], tmp_path)
    assert r.returncode != 0 and "TreeID not provided" in r.stderr
    r = _run(["-I", "in.panman", "--reroot", "-d", "0", "-o", "x"], tmp_path)
    assert r.returncode != 0 and "Refence ID not provided" in r.stderr


@pytest.mark.gpu
def test_pangraph_build_then_fasta(tmp_path):
    """-P sars_20.json -N sars_20.nwk -o s, then -I ./panman/s.panman --fasta -o s replays
    the input genomes."""
    gold = os.path.join(ROOT, "tests", "golden")
    r = _run(["-P", os.path.join(gold, "sars_20.json"), "-N", os.path.join(gold, "sars_20.nwk"), "-o", "s"], tmp_path)
    assert r.returncode == 0, r.stderr
    r = _run(["-I", "panman/s.panman", "-f", "-o", "s"], tmp_path)
    assert r.returncode == 0, r.stderr
    got = parse_records(open(tmp_path / "info" / "s_0.fasta").read())
    want, name = {}, None
    for line in open(os.path.join(gold, "sars_20.fa")):
        line = line.strip()
        if line.startswith(">"):
            name = line[1:]
            want[name] = ""
        elif line:
            want[name] += line.upper()
    assert got == want


def test_protobuf2capnp_converts_old_panman(tmp_path):
    """--protobuf2capnp -I old -o out (src/panmanUtils.cpp:939-952): ./panman/out.panman holds
    the same trees as the Cap'n Proto file the old one was encoded from (tests/_protobuf.py)."""
    from _protobuf import encode_tree, encode_tree_group
    rng = np.random.default_rng(12)
    pms = []
    for _ in range(2):
        off, idx, root = random_tree(20, rng, max_children=3)
        pms.append(random_panmat(rng, off, idx, root, names_for(off), blocks=3))
    ref = str(tmp_path / "ref.panman")
    write_panman(ref, pms)
    f = PanmanFile(ref)
    old = tmp_path / "old.pb.xz"
    old.write_bytes(encode_tree_group([encode_tree(f.to_panmat(i), f.newick(i)) for i in range(len(f))]))
    r = _run(["-I", str(old), "--protobuf2capnp", "-o", "conv"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Writing PanMAN" in r.stdout and "Network Write execution time" in r.stdout
    g = PanmanFile(str(tmp_path / "panman" / "conv.panman"))
    assert len(g) == len(f)
    for i in range(len(f)):
        a, b = f.to_panmat(i), g.to_panmat(i)
        assert a.names == b.names and (a.child_offsets == b.child_offsets).all()
        assert (a.child_index == b.child_index).all()
        for k in a._arrays:
            assert np.array_equal(a._arrays[k], b._arrays[k]), k
    r = _run(["-I", str(old), "--protobuf2capnp"], tmp_path)
    assert r.returncode == 1 and "Output file not provided" in r.stderr


@pytest.mark.gpu
def test_protobuf2capnp_then_fasta_on_gpu(tmp_path, oracle):
    """An old Protobuf PanMAN converted by --protobuf2capnp replays on the GPU to the same
    aligned FASTA the oracle gives for the tree it was encoded from."""
    from _protobuf import encode_tree, encode_tree_group
    rng = np.random.default_rng(21)
    off, idx, root = random_tree(30, rng, max_children=3, unary=0.1)
    ref = str(tmp_path / "ref.panman")
    write_panman(ref, [random_panmat(rng, off, idx, root, names_for(off), blocks=4)])
    f = PanmanFile(ref)
    (tmp_path / "old.pb.xz").write_bytes(encode_tree_group([encode_tree(f.to_panmat(0), f.newick(0))]))
    r = _run(["-I", "old.pb.xz", "--protobuf2capnp", "-o", "conv"], tmp_path)
    assert r.returncode == 0, r.stderr
    r = _run(["-I", "panman/conv.panman", "-m", "-o", "conv"], tmp_path)
    assert r.returncode == 0, r.stderr
    got = parse_records(open(tmp_path / "info" / "conv_0.msa").read())
    assert got == parse_records(oracle.fasta(f.to_panmat(0), True))
