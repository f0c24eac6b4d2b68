"""Independent Protobuf wire-format encoder for the older PanMAN format (panmanOld.treeGroup,
/root/reference/panman.proto) -- test infrastructure: builds .panman-old fixtures from a
loaded PanMAT, so the product's hand-written reader (pm_panman_load_old) can be checked
against the Cap'n Proto reader on the same trees.  No protobuf library exists offline."""
import lzma


def varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64          # int32 / int64 negatives: ten-byte two's complement
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def key(field: int, wire: int) -> bytes:
    return varint((field << 3) | wire)


def f_varint(field: int, v: int) -> bytes:
    return key(field, 0) + varint(int(v))


def f_bytes(field: int, b: bytes) -> bytes:
    return key(field, 2) + varint(len(b)) + b


def f_repeated(field: int, values, packed: bool) -> bytes:
    values = [int(x) for x in values]
    if packed:
        return f_bytes(field, b"".join(varint(x) for x in values)) if values else b""
    return b"".join(f_varint(field, x) for x in values)


def encode_tree(pm, newick: str, packed=True, shuffle=None, extra_unknown=False) -> bytes:
    """pm: a PanMAT with bulk arrays (PanmanFile.to_panmat), nodes indexed in pre-order of
    `newick` (the stored node order).  shuffle: a random.Random that permutes field order."""
    a = pm._arrays
    n = pm.num_nodes
    parts = [f_bytes(1, newick.encode())]
    bmo, nmo = a["block_mut_offsets"], a["nuc_mut_offsets"]
    for v in range(n):
        muts = []
        for k in range(int(bmo[v]), int(bmo[v + 1])):   # block mutations, list order
            m = f_varint(1, int(a["block_mut_primary"][k]) << 32) + f_varint(3, 1)
            m += f_varint(4, int(a["block_mut_info"][k])) + f_varint(5, int(a["block_mut_inversion"][k]))
            muts.append(m)
        for k in range(int(nmo[v]), int(nmo[v + 1])):   # one nucleotide mutation per message
            prim, sec = int(a["nuc_mut_primary"][k]), int(a["nuc_mut_secondary"][k])
            info, nucs = int(a["nuc_mut_info"][k]), int(a["nuc_mut_nucs"][k])
            ln = info >> 4
            nm = f_varint(1, int(a["nuc_mut_position"][k]))
            gap = int(a["nuc_mut_gap_position"][k])
            if gap >= 0:
                nm += f_varint(2, gap) + f_varint(3, 1)
            nm += f_varint(4, ((nucs >> (24 - 4 * ln)) << 8) + info)
            m = f_varint(1, (prim << 32) | (sec & 0xFFFFFFFF if sec >= 0 else 0))
            if sec >= 0:
                m += f_varint(2, 1)
            m += f_bytes(6, nm)
            muts.append(m)
        node = b"".join(f_bytes(1, m) for m in muts)
        if extra_unknown:
            node += f_bytes(2, b"an annotation") + f_varint(15, 7)
        parts.append(f_bytes(2, node))
    bso = a["block_seq_offsets"]
    for b in range(len(a["block_primary"])):
        seq = a["block_seq"][int(bso[b]):int(bso[b + 1])]
        c = f_repeated(1, [int(a["block_primary"][b]) << 32], packed) + f_repeated(2, seq, packed)
        c += f_repeated(3, [0], packed) + f_bytes(4, b"chr1")
        parts.append(f_bytes(4, c))
    go = a["gap_offsets"]
    for g in range(len(a["gap_primary"])):
        lo, hi = int(go[g]), int(go[g + 1])
        gl = f_varint(1, int(a["gap_primary"][g]) << 32)
        gl += f_repeated(3, a["gap_length"][lo:hi], packed) + f_repeated(4, a["gap_position"][lo:hi], packed)
        parts.append(f_bytes(5, gl))
    parts.append(f_bytes(6, b""))   # empty blockGaps
    for v in range(n):
        name = pm.names[v].encode()
        if pm.circular[v] >= 0:
            parts.append(f_bytes(7, f_bytes(1, name) + f_varint(2, int(pm.circular[v]))))
        if pm.rotation[v]:
            parts.append(f_bytes(8, f_bytes(1, name) + f_varint(2, int(pm.rotation[v]))))
        if pm.inverted[v]:
            parts.append(f_bytes(9, f_bytes(1, name) + f_varint(2, 1)))
    if shuffle is not None:   # fields in any order; each repeated field keeps its own order
        groups = {}
        for p in parts:
            groups.setdefault(p[0], []).append(p)
        queues = list(groups.values())
        merged = []
        while queues:
            q = shuffle.choice(queues)
            merged.append(q.pop(0))
            if not q:
                queues.remove(q)
        parts = merged
    return b"".join(parts)


def encode_tree_group(trees, compress=True) -> bytes:
    """trees: list of encoded tree messages."""
    raw = b"".join(f_bytes(1, t) for t in trees)
    raw += f_bytes(2, f_varint(1, 1) + f_varint(2, 0))   # one complexMutation (not on the path)
    return lzma.compress(raw, format=lzma.FORMAT_XZ) if compress else raw
