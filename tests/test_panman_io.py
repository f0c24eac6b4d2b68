"""PanMAN file IO (next row SURVEY.md §8f-1): writer/reader round trip, layout checked by an
independent decoder, corrupt input rejected.  Host-only (no GPU).  Parity with the
reference's capnp library is unpinned: no .panman fixture exists offline."""
import os

import numpy as np
import pytest

from _capnp import LAYOUT, root
from _panmat import parse_records, random_panmat
from _trees import names_for, random_tree
from panman_amd.panmat import PanmanFile, write_panman


def test_layout_matches_survey_derivation():
    nuc, dw, pc = LAYOUT["NucMut"]
    assert (nuc["nucPosition"], nuc["nucGapPosition"], nuc["nucGapExist"], nuc["mutInfo"], dw, pc) == \
        (0, 32, 64, 96, 2, 0)
    mu, dw, pc = LAYOUT["Mutation"]
    assert (mu["blockId"], mu["blockGapExist"], mu["blockMutExist"], mu["blockMutInfo"], mu["blockInversion"],
            dw, pc) == (0, 64, 65, 66, 67, 2, 1)
    assert LAYOUT["GapList"][1:] == (2, 2) and LAYOUT["CircularOffset"][1:] == (1, 1)
    assert LAYOUT["Tree"][1:] == (0, 8)


@pytest.mark.parametrize("seed", range(4))
def test_round_trip_replays_identically(tmp_path, oracle, seed):
    rng = np.random.default_rng(40 + seed)
    off, idx, root_ = random_tree(30, rng, max_children=3, unary=0.1)
    pm = random_panmat(rng, off, idx, root_, names_for(off), blocks=int(rng.integers(1, 6)))
    path = str(tmp_path / "t.panman")
    write_panman(path, [pm], compress=bool(seed % 2 == 0))
    f = PanmanFile(path)
    assert len(f) == 1
    back = f.to_panmat(0)
    for aligned in (True, False):
        assert parse_records(oracle.fasta(back, aligned)) == parse_records(oracle.fasta(pm, aligned))


def test_independent_decoder_reads_fields(tmp_path):
    rng = np.random.default_rng(3)
    off, idx, root_ = random_tree(12, rng, max_children=2)
    pm = random_panmat(rng, off, idx, root_, names_for(off), blocks=3)
    path = str(tmp_path / "t.panman")
    write_panman(path, [pm])
    tg = root(open(path, "rb").read())
    trees = tg.items("trees", "Tree")
    assert len(trees) == 1 and tg.items("complexMutations", "ComplexMutation") == []
    t = trees[0]
    assert t.text("newick").endswith(";")
    nodes = t.items("nodes", "Node")
    assert len(nodes) == pm.num_nodes + 1          # trailing empty node, as the reference writes
    # every nucleotide mutation of the file decodes to one of the PanMAT's records
    want = set()
    for lst in pm.nuc_muts:
        for prim, sec, pos, gap, info, nucs in lst:
            ln = info >> 4
            want.add((prim, pos, gap, ((nucs >> (24 - 4 * ln)) << 8) + info))
    got = set()
    for node in nodes:
        for m in node.items("mutations", "Mutation"):
            prim = m.bits("blockId", 64) >> 32
            for nm in m.items("nucMutation", "NucMut"):
                gap = nm.bits("nucGapPosition", 32, True) if nm.bits("nucGapExist", 1) else -1
                got.add((prim, nm.bits("nucPosition", 32, True), gap, nm.bits("mutInfo", 32)))
    assert got == want
    blocks = t.items("consensusSeqMap", "ConsensusSeqToBlockIds")
    ids = sorted(i >> 32 for c in blocks for i in c.items("blockId"))
    assert ids == sorted(p for p, _ in pm.blocks)


def test_corrupt_files_are_errors(tmp_path):
    import panman_amd
    bad = tmp_path / "bad.panman"
    bad.write_bytes(b"\xfd7zXZ\x00garbage")
    with pytest.raises(panman_amd.PanmanError):
        PanmanFile(str(bad))
    trunc = tmp_path / "trunc.panman"
    trunc.write_bytes(b"\x00\x00\x00\x00\xff\x00\x00\x00" + b"\x00" * 16)
    with pytest.raises(panman_amd.PanmanError):
        PanmanFile(str(trunc))


def _newick_only_message(newick: str) -> bytes:
    """Uncompressed capnp message: TreeGroup{trees=[Tree{newick}]} (other fields null)."""
    import struct
    text = newick.encode() + b"\0"
    tw = (len(text) + 7) // 8
    # words: 0 root ptr | 1-2 TreeGroup ptrs | 3 list tag | 4-11 Tree ptrs | 12.. text
    words = [0] * (12 + tw)

    def sptr(at, target, dw, pc):
        return ((target - at - 1) << 2) | (dw << 32) | (pc << 48)

    def lptr(at, target, size, n):
        return ((target - at - 1) << 2) | 1 | (size << 32) | (n << 35)

    words[0] = sptr(0, 1, 0, 2)
    words[1] = lptr(1, 3, 7, 8)                  # composite, 8 words of elements
    words[3] = (1 << 2) | (0 << 32) | (8 << 48)  # tag: 1 element, 0 data words, 8 ptrs
    words[4] = lptr(4, 12, 2, len(text))         # newick: List(UInt8) with NUL
    body = b"".join(struct.pack("<Q", w & (2**64 - 1)) for w in words[:12]) + text.ljust(tw * 8, b"\0")
    return struct.pack("<II", 0, len(body) // 8) + body


@pytest.mark.parametrize("newick,want", [
    # lengths kept, internal labels ignored and renamed, root printed with 0
    ("((a:1,b:2)X:0.5,c:3);", "((a:1.000000,b:2.000000)node_2:0.500000,c:3.000000)node_1:0.000000;"),
    # a clade without ':len' takes the last length of its piece; 0 and missing become 1
    ("(((a:0.5,b:0.7)),c:2);",
     "(((a:0.500000,b:0.700000)node_3:0.700000)node_2:0.700000,c:2.000000)node_1:0.000000;"),
    ("(a,b:0,(c:1e-05,d));", "(a:1.000000,b:1.000000,(c:105.000000,d:1.000000)node_2:1.000000)node_1:0.000000;"),
])
def test_newick_lengths_follow_reference_rules(tmp_path, newick, want):
    """createTreeFromNewickString length queues (src/panman.cpp:339-435) and
    getNewickString (:1921-2029), through load -> write -> load."""
    src = tmp_path / "n.capnp"
    src.write_bytes(_newick_only_message(newick))
    f = PanmanFile(str(src))
    assert f.newick(0) == newick
    pm = f.to_panmat(0)
    f.close()
    pm.add_block(0, "ACGT")
    out = str(tmp_path / "o.panman")
    write_panman(out, [pm])
    g = PanmanFile(out)
    assert g.newick(0) == want
    again = g.to_panmat(0)
    g.close()
    assert np.array_equal(again.branch_length, pm.branch_length)


def test_multi_block_xz_round_trip(tmp_path, monkeypatch, oracle):
    """A message above the xz block size is written as one .xz stream of independent blocks
    (decoded block-parallel by the reader) and as one block (PM_XZ_THREADS=1, what the
    reference writes, decoded serially): both decode with Python's lzma to the same bytes and
    load back to PanMATs that replay identically."""
    import lzma
    from panman_amd.synth import c5_panmat
    pm = c5_panmat(leaves=60, blocks=40, mean_len=4000, seed=5)
    paths = {}
    for threads, block in (("4", "65536"), ("1", None)):
        monkeypatch.setenv("PM_XZ_THREADS", threads)
        if block:
            monkeypatch.setenv("PM_XZ_BLOCK", block)
        else:
            monkeypatch.delenv("PM_XZ_BLOCK", raising=False)
        paths[threads] = str(tmp_path / f"x{threads}.panman")
        write_panman(paths[threads], [pm])
    multi, single = (open(paths[k], "rb").read() for k in ("4", "1"))
    assert multi != single                                   # several blocks vs one
    assert lzma.decompress(multi) == lzma.decompress(single)
    from panman_amd._lib import phase_report, phase_reset
    back = []
    for k in ("4", "1"):
        phase_reset()
        back.append(PanmanFile(paths[k]).to_panmat(0))
        blocks = [v for name, v in phase_report() if name == "panman.xz_parallel_blocks"]
        if k == "4":   # the re-wrapped one-block streams decoded on their own, none fell back
            assert blocks and blocks[0] == multi_blocks(multi)
        else:
            assert not blocks
    want = parse_records(oracle.fasta(pm, True))
    for b in back:
        assert parse_records(oracle.fasta(b, True)) == want


def _vli(b, i):
    v, k = 0, 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << (7 * k)
        k += 1
        if not x & 0x80:
            return v, i


def _vli_bytes(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _xz_index(data):
    """(index offset, [(unpadded, uncompressed)]) of a one-stream .xz file."""
    import struct
    backward = (struct.unpack("<I", data[-8:-4])[0] + 1) * 4
    at = len(data) - 12 - backward
    assert data[at] == 0
    n, i = _vli(data, at + 1)
    recs = []
    for _ in range(n):
        u, i = _vli(data, i)
        c, i = _vli(data, i)
        recs.append((u, c))
    return at, recs


def multi_blocks(data):
    return len(_xz_index(data)[1])


def _with_index(data, recs):
    """The stream with its index records replaced (index + footer CRCs recomputed)."""
    import struct
    import zlib
    at, _ = _xz_index(data)
    idx = bytearray(b"\x00") + _vli_bytes(len(recs))
    for u, c in recs:
        idx += _vli_bytes(u) + _vli_bytes(c)
    while len(idx) % 4:
        idx.append(0)
    idx += struct.pack("<I", zlib.crc32(idx))
    tail = struct.pack("<I", len(idx) // 4 - 1) + data[6:8]
    foot = struct.pack("<I", zlib.crc32(tail)) + tail + b"YZ"
    return data[:at] + bytes(idx) + foot


@pytest.mark.parametrize("attack", ["wrap", "huge", "overrun"])
def test_crafted_xz_index_is_rejected(tmp_path, monkeypatch, attack):
    """Index sizes are attacker-controlled (the CRC is computable): sizes whose sums wrap 2^64,
    a declared output far beyond the input, or a block running past the index must not reach
    the block-parallel decoder -- the load fails cleanly (PM_ERR_ARG) instead."""
    from panman_amd.synth import c5_panmat
    from panman_amd._lib import PanmanError
    monkeypatch.setenv("PM_XZ_THREADS", "4")
    monkeypatch.setenv("PM_XZ_BLOCK", "32768")
    good = str(tmp_path / "good.panman")
    write_panman(good, [c5_panmat(leaves=20, blocks=20, mean_len=4000, seed=2)])
    data = open(good, "rb").read()
    _, recs = _xz_index(data)
    assert len(recs) >= 3
    big = (1 << 63) - 1
    if attack == "wrap":       # out offsets wrap to a tiny total
        recs = [(recs[0][0], big), (recs[1][0], big)] + [(u, 2) for u, _ in recs[2:]]
    elif attack == "huge":
        recs = [(recs[0][0], 1 << 50)] + recs[1:]
    else:                      # first block claims the whole file
        recs = [(len(data), recs[0][1])] + recs[1:]
    bad = str(tmp_path / "bad.panman")
    open(bad, "wb").write(_with_index(data, recs))
    with pytest.raises(PanmanError) as e:
        PanmanFile(bad)
    assert "xz" in str(e.value)


def test_xz_blocks_depend_on_message_size_only(tmp_path, monkeypatch):
    """The writer cuts a message into >= 16 blocks of >= 64 KiB (1 MiB from 16 MiB up), whatever
    the host's thread count: the bytes written are the same with 1 and 8 encoder threads, and
    the stream holds the block count the size rule gives."""
    import lzma
    from panman_amd.synth import c5_panmat
    pm = c5_panmat(leaves=40, blocks=30, mean_len=3000, seed=9)
    monkeypatch.delenv("PM_XZ_BLOCK", raising=False)
    monkeypatch.delenv("PM_XZ_THREADS", raising=False)
    out = {}
    for threads in ("1", "8"):
        monkeypatch.setenv("PM_HOST_THREADS", threads)
        path = str(tmp_path / f"t{threads}.panman")
        write_panman(path, [pm])
        out[threads] = open(path, "rb").read()
    assert out["1"] == out["8"]
    n = len(lzma.decompress(out["1"]))
    block = 1 << 16
    while block < (1 << 20) and block * 16 < n:
        block <<= 1
    assert multi_blocks(out["1"]) == max(1, -(-n // block))
