"""GPU parity for FASTA replay (R1-R3): pm_fasta vs the oracle's printFASTAUltraFast
restatement, record for record."""
import json
import os

import numpy as np
import pytest

import panman_amd
from _panmat import from_fixture, parse_records, random_panmat
from _trees import names_for, parse_newick, random_tree, to_newick
from panman_amd.panmat import from_msa_dump

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kats.json")
REPLAY = json.load(open(GOLDEN))["replay"]


@pytest.fixture(scope="module")
def engine():
    e = panman_amd.Engine(0)
    yield e
    e.close()


def _records(text):
    recs = [">" + r for r in text.split(">")[1:]]
    return sorted(recs)


@pytest.mark.parametrize("kat", REPLAY, ids=[k["id"] for k in REPLAY])
def test_replay_kats_on_gpu(engine, kat):
    pm = from_fixture(kat)
    for aligned in (True, False):
        got = parse_records(engine.fasta(pm, aligned))
        for name, exp in kat["expect"].items():
            key = "aligned" if aligned else "unaligned"
            if key in exp:
                assert got[name] == exp[key], (name, key, got[name])


@pytest.mark.parametrize("seed", range(8))
def test_random_panmat_vs_oracle(engine, oracle, seed):
    rng = np.random.default_rng(900 + seed)
    off, idx, root = random_tree(40, rng, max_children=4, unary=0.1)
    pm = random_panmat(rng, off, idx, root, names_for(off), blocks=int(rng.integers(1, 9)))
    for aligned in (True, False):
        want = _records(oracle.fasta(pm, aligned))
        got = _records(engine.fasta(pm, aligned))
        assert got == want


@pytest.mark.parametrize("seed", range(3))
def test_secondary_block_mutation_lands_on_primary(engine, oracle, seed):
    """printFASTAUltraFastHelper reads a NucMut's secondaryBlockId and never uses it
    (src/fasta.cpp:1838-1842): the mutation is applied to the primary block.  Same here, vs
    the oracle's restatement of that loop."""
    rng = np.random.default_rng(11 + seed)
    off, idx, root = random_tree(12, rng, max_children=3)
    pm = random_panmat(rng, off, idx, root, names_for(off), blocks=2, options=False)
    for leaf in pm.leaves()[:4]:
        pm.add_nuc_mut(leaf, 0, 1, -1, 0, [2], secondary=int(rng.integers(0, 3)))
        pm.add_nuc_mut(leaf, 1, 0, -1, 3, [8], secondary=0)
    for aligned in (True, False):
        assert _records(engine.fasta(pm, aligned)) == _records(oracle.fasta(pm, aligned))


def test_reroot_refuses_secondary_blocks(engine):
    """The same PanMAT replays (above) but reroot refuses it with PM_ERR_UNSUPPORTED and says
    why: the reference rebuilds secondary blocks' sequences and states (src/reroot.cpp:55-89),
    which this layout does not hold (include/panman_gpu.h, pm_reroot)."""
    rng = np.random.default_rng(11)
    off, idx, root = random_tree(12, rng, max_children=3)
    pm = random_panmat(rng, off, idx, root, names_for(off), blocks=2, options=False)
    leaves = pm.leaves()
    pm.add_nuc_mut(leaves[0], 0, 1, -1, 0, [2], secondary=1)
    with pytest.raises(panman_amd.PanmanError, match="secondary blocks"):
        engine.reroot(pm, pm.names[leaves[1]])


def test_long_blocks_wrap_vs_oracle(engine, oracle):
    rng = np.random.default_rng(5)
    off, idx, root = random_tree(30, rng, max_children=3)
    pm = random_panmat(rng, off, idx, root, names_for(off), blocks=5, block_len=(100, 400), mut_rate=0.02)
    for aligned in (True, False):
        assert _records(engine.fasta(pm, aligned)) == _records(oracle.fasta(pm, aligned))


def test_msa_to_fasta_round_trip_on_gpu(engine, oracle):
    """MSA -> pm_msa_build (GPU) -> PanMAT -> pm_fasta (GPU) reproduces the alignment."""
    rng = np.random.default_rng(77)
    off, idx, root = random_tree(50, rng, max_children=3)
    names = names_for(off)
    nwk = to_newick(off, idx, root, names)
    base = rng.choice(list("ACGT"), size=333)
    rows = {}
    for i in range(len(names)):
        if off[i] == off[i + 1]:
            s = base.copy()
            f = rng.random(333) < 0.15
            s[f] = rng.choice(list("ACGTN-"), size=f.sum())
            rows[names[i]] = "".join(s)
    msa = "".join(f">{k}\n{v}\n" for k, v in rows.items())
    dump = panman_amd.msa_build(nwk, msa, "", panman_amd.MODE_FITCH)
    pnames, poff, pidx, proot = parse_newick(nwk)
    pm = from_msa_dump(dump, pnames, poff, pidx, proot)
    assert parse_records(engine.fasta(pm, True)) == rows


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_msa_to_panman_file_round_trip(engine, oracle, tmp_path, mode):
    """MSA -> pm_msa_to_panman (GPU build + writer) -> .panman -> loader -> pm_fasta
    reproduces the alignment rows; the file's tree equals the in-memory dump's."""
    rng = np.random.default_rng(78 + mode)
    off, idx, root = random_tree(60, rng, max_children=4)
    names = names_for(off)
    nwk = to_newick(off, idx, root, names)
    base = rng.choice(list("ACGT"), size=517)
    rows = {}
    for i in range(len(names)):
        if off[i] == off[i + 1]:
            s = base.copy()
            f = rng.random(517) < 0.1
            s[f] = rng.choice(list("ACGTRN-"), size=f.sum())
            rows[names[i]] = "".join(s)
    msa = "".join(f">{k}\n{v}\n" for k, v in rows.items())
    ref = next(iter(rows)) if mode == panman_amd.MODE_SANKOFF else ""
    path = str(tmp_path / "t.panman")
    panman_amd.msa_to_panman(nwk, msa, path, ref, mode)
    f = panman_amd.PanmanFile(path)
    try:
        assert len(f) == 1
        got = parse_records(engine.fasta(f.view(0), True))
        assert got == rows
        unal = parse_records(engine.fasta(f.view(0), False))
        assert unal == {k: v.replace("-", "") for k, v in rows.items()}
        pnames, poff, pidx, proot = parse_newick(nwk)
        pm = from_msa_dump(panman_amd.msa_build(nwk, msa, ref, mode), pnames, poff, pidx, proot)
        assert _records(engine.fasta(pm, True)) == _records(engine.fasta(f.view(0), True))
    finally:
        f.close()


@pytest.mark.parametrize("aligned", [True, False])
def test_c5_like_panmat_vs_oracle(engine, oracle, aligned):
    """Bulk generator (bench workload family C5) at reduced size, every leaf compared."""
    from panman_amd.synth import c5_panmat
    pm = c5_panmat(leaves=120, blocks=40, mean_len=1500, seed=11)
    assert _records(engine.fasta(pm, aligned)) == _records(oracle.fasta(pm, aligned))


@pytest.mark.parametrize("aligned", [True, False])
def test_fasta_multi_device_matches_single(engine, aligned):
    """Leaf-sharded FASTA: several contexts (here on one GPU) give the
    single-context text byte for byte, including more shards than leaves."""
    from panman_amd.synth import c5_panmat
    pm = c5_panmat(leaves=37, blocks=12, mean_len=900, seed=5)
    want = engine.fasta(pm, aligned)
    for devices in ([0, 0], [0, 0, 0], [0] * 50):
        assert panman_amd.fasta_multi(pm, aligned, devices) == want


@pytest.mark.parametrize("mode", [panman_amd.MODE_FITCH, panman_amd.MODE_SANKOFF])
def test_msa_build_multi_device_matches_single(tmp_path, mode):
    """Column-sharded MSA construction writes the same file as the one-context build."""
    rng = np.random.default_rng(300 + mode)
    off, idx, root = random_tree(80, rng, max_children=5)
    names = names_for(off)
    nwk = to_newick(off, idx, root, names)
    base = rng.choice(list("ACGT"), size=1999)
    rows = {}
    for i in range(len(names)):
        if off[i] == off[i + 1]:
            s = base.copy()
            f = rng.random(1999) < 0.08
            s[f] = rng.choice(list("ACGTRN-"), size=f.sum())
            rows[names[i]] = "".join(s)
    msa = "".join(f">{k}\n{v}\n" for k, v in rows.items())
    ref = next(iter(rows)) if mode == panman_amd.MODE_SANKOFF else ""
    one, many = str(tmp_path / "one.panman"), str(tmp_path / "many.panman")
    panman_amd.msa_to_panman(nwk, msa, one, ref, mode)
    panman_amd.msa_to_panman(nwk, msa, many, ref, mode, devices=[0, 0, 0])
    assert open(one, "rb").read() == open(many, "rb").read()


@pytest.mark.parametrize("aligned", [True, False])
def test_fasta_fd_streams_the_same_text(engine, tmp_path, aligned):
    """pm_fasta_fd / pm_fasta_multi_fd (the CLI's path: the device text streamed through the
    pinned slots to a descriptor) write pm_fasta's text byte for byte -- to a file, and through
    a pipe read concurrently (more than one 64 MiB slot: a multi-chunk stream) -- and fail on a
    descriptor that cannot be written."""
    import os
    import threading
    from panman_amd.synth import c5_panmat
    pm = c5_panmat(leaves=37, blocks=12, mean_len=900, seed=5)
    want = engine.fasta(pm, aligned).encode()
    path = tmp_path / "out.fa"
    with open(path, "wb") as f:
        n = engine.fasta_fd(pm, aligned, f.fileno())
    assert n == len(want) and path.read_bytes() == want
    for devices in ([0], [0, 0, 0], [0] * 50):
        with open(path, "wb") as f:
            assert panman_amd.engine.fasta_multi_fd(pm, aligned, devices, f.fileno()) == len(want)
        assert path.read_bytes() == want, devices
    big = c5_panmat(leaves=60, blocks=120, mean_len=12_000, seed=9)   # ~90 MB of aligned text
    want_big = engine.fasta(big, True).encode()
    assert len(want_big) > (64 << 20)
    r, w = os.pipe()
    got = []
    reader = threading.Thread(target=lambda: got.append(b"".join(iter(lambda: os.read(r, 1 << 20), b""))))
    reader.start()
    try:
        n = engine.fasta_fd(big, True, w)
    finally:
        os.close(w)
        reader.join()
        os.close(r)
    assert n == len(want_big) and got[0] == want_big
    rd, wr = os.pipe()
    os.close(rd)   # a pipe without a reader: EPIPE (SIGPIPE is ignored by Python)
    try:
        with pytest.raises(panman_amd.PanmanError):
            engine.fasta_fd(pm, aligned, wr)
    finally:
        os.close(wr)
