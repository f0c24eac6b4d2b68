"""Independent check of the PanMAN wire format: a minimal Cap'n Proto decoder whose struct
layouts are derived here from panman.capnp with capnp's field-allocation rule (fields in
ordinal order; each data field takes the lowest-offset hole of its size, splitting larger
holes in halves; pointers take the next pointer slot).  Test infrastructure only."""
from __future__ import annotations

import lzma
import struct

SIZES = {"Bool": 1, "Int32": 32, "UInt32": 32, "Int64": 64}

# (struct, [(field, type)]) in ordinal order, from /root/reference/panman.capnp
SCHEMA = {
    "NucMut": [("nucPosition", "Int32"), ("nucGapPosition", "Int32"), ("nucGapExist", "Bool"),
               ("mutInfo", "UInt32")],
    "Mutation": [("blockId", "Int64"), ("blockGapExist", "Bool"), ("blockMutExist", "Bool"),
                 ("blockMutInfo", "Bool"), ("blockInversion", "Bool"), ("nucMutation", "ptr")],
    "Node": [("mutations", "ptr"), ("annotations", "ptr")],
    "ConsensusSeqToBlockIds": [("blockId", "ptr"), ("consensusSeq", "ptr"), ("blockGapExist", "ptr"),
                               ("chromosomeName", "ptr")],
    "GapList": [("blockId", "Int64"), ("blockGapExist", "Bool"), ("nucGapLength", "ptr"),
                ("nucPosition", "ptr")],
    "CircularOffset": [("sequenceId", "ptr"), ("offset", "Int32")],
    "RotationIndex": [("sequenceId", "ptr"), ("blockOffset", "Int32")],
    "SequenceInverted": [("sequenceId", "ptr"), ("inverted", "Bool")],
    "Tree": [(f, "ptr") for f in ("newick", "nodes", "consensusSeqMap", "gaps", "blockGaps",
                                  "circularSequences", "rotationIndexes", "sequencesInverted")],
    "TreeGroup": [("trees", "ptr"), ("complexMutations", "ptr")],
}


def layout(fields):
    """-> ({field: bit offset or ('ptr', index)}, data_words, ptr_count)"""
    holes = {}          # size -> sorted list of bit offsets
    words = 0
    ptrs = 0
    out = {}

    def take(size):
        nonlocal words
        for s in (size, 2 * size, 4 * size, 8 * size, 16 * size, 32 * size, 64 * size):
            if s > 64:
                break
            if holes.get(s):
                off = holes[s].pop(0)
                while s > size:      # split: keep the lower half, free the upper half
                    s //= 2
                    holes.setdefault(s, []).append(off + s)
                    holes[s].sort()
                return off
        off = words * 64
        words += 1
        s = 64
        while s > size:
            s //= 2
            holes.setdefault(s, []).append(off + s)
            holes[s].sort()
        return off

    for name, typ in fields:
        if typ == "ptr":
            out[name] = ("ptr", ptrs)
            ptrs += 1
        else:
            out[name] = take(SIZES[typ])
    return out, words, ptrs


LAYOUT = {k: layout(v) for k, v in SCHEMA.items()}


class Reader:
    def __init__(self, data: bytes):
        if data[:4] == b"\xfd7zX":
            data = lzma.decompress(data)
        n = struct.unpack_from("<I", data, 0)[0] + 1
        sizes = struct.unpack_from(f"<{n}I", data, 4)
        at = ((n + 1) * 4 + 7) // 8 * 8
        self.segs = []
        for s in sizes:
            self.segs.append(data[at:at + 8 * s])
            at += 8 * s

    def word(self, seg, pos):
        return struct.unpack_from("<Q", self.segs[seg], 8 * pos)[0]

    def ptr(self, seg, pos):
        w = self.word(seg, pos)
        if w == 0:
            return None
        kind = w & 3
        if kind == 2:
            assert not (w >> 2) & 1, "double-far not needed here"
            return self.ptr(w >> 32, (w >> 3) & 0x1FFFFFFF)
        off = ((w & 0xFFFFFFFF) >> 2)
        if off & (1 << 29):
            off -= 1 << 30
        return seg, pos + 1 + off, w

    def struct(self, seg, pos, name):
        p = self.ptr(seg, pos)
        return None if p is None else Struct(self, p[0], p[1], (p[2] >> 32) & 0xFFFF, p[2] >> 48, name)

    def list(self, seg, pos, name=None):
        p = self.ptr(seg, pos)
        if p is None:
            return []
        s, at, w = p
        esize, n = (w >> 32) & 7, w >> 35
        if esize == 7:
            tag = self.word(s, at)
            cnt, dw, pc = (tag & 0xFFFFFFFF) >> 2, (tag >> 32) & 0xFFFF, tag >> 48
            return [Struct(self, s, at + 1 + i * (dw + pc), dw, pc, name) for i in range(cnt)]
        raw = self.segs[s][8 * at:]
        if esize == 1:
            return [(raw[i // 8] >> (i % 8)) & 1 for i in range(n)]
        fmt = {2: "B", 3: "H", 4: "I", 5: "Q"}[esize]
        return list(struct.unpack_from(f"<{n}{fmt}", raw, 0))

    def text(self, seg, pos):
        b = self.list(seg, pos)
        return bytes(b[:-1]).decode() if b else ""


class Struct:
    def __init__(self, r, seg, pos, dwords, ptrs, name):
        self.r, self.seg, self.pos, self.dwords, self.ptrs, self.name = r, seg, pos, dwords, ptrs, name

    def _field(self, f):
        return LAYOUT[self.name][0][f]

    def bits(self, f, width, signed=False):
        off = self._field(f)
        if off // 64 >= self.dwords:
            return 0
        v = (self.r.word(self.seg, self.pos + off // 64) >> (off % 64)) & ((1 << width) - 1)
        if signed and v >> (width - 1):
            v -= 1 << width
        return v

    def pos_of(self, f):
        return self.pos + self.dwords + self._field(f)[1]

    def child(self, f, name):
        return self.r.struct(self.seg, self.pos_of(f), name)

    def items(self, f, name=None):
        return self.r.list(self.seg, self.pos_of(f), name)

    def text(self, f):
        return self.r.text(self.seg, self.pos_of(f))


def root(data: bytes) -> Struct:
    r = Reader(data)
    return r.struct(0, 0, "TreeGroup")
