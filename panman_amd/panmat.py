"""In-memory PanMAT (the reference's Tree fields used by FASTA replay) as flat arrays,
and its C view `pm_panmat` (include/panman_gpu.h).  Reference types: Block
src/panman.hpp:520-534, GapList :537-543, BlockMut :429-517, NucMut :75-313, Tree
circularSequences / rotationIndexes / sequenceInverted (src/panman.hpp:634-983)."""
from __future__ import annotations

import ctypes as C

import numpy as np

CODE = {c: i for i, c in enumerate("-ACMGRSVTWYHKDBN")}


def encode_block(seq: str) -> list[int]:
    """Block(primaryBlockId, seq): 8 codes per uint32, MSB nibble first (src/panman.cpp:246-257)."""
    words = []
    for i in range(0, len(seq), 8):
        w = 0
        for j, ch in enumerate(seq[i:i + 8]):
            w ^= CODE.get(ch, 0) << (4 * (7 - j))
        words.append(w)
    return words


class PanmatStruct(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_int32), ("root", C.c_int32),
        ("child_offsets", C.c_void_p), ("child_index", C.c_void_p), ("names", C.c_void_p),
        ("num_blocks", C.c_int32), ("block_primary", C.c_void_p), ("block_seq_offsets", C.c_void_p),
        ("block_seq", C.c_void_p),
        ("num_gaps", C.c_int32), ("gap_primary", C.c_void_p), ("gap_offsets", C.c_void_p),
        ("gap_position", C.c_void_p), ("gap_length", C.c_void_p),
        ("block_mut_offsets", C.c_void_p), ("block_mut_primary", C.c_void_p), ("block_mut_info", C.c_void_p),
        ("block_mut_inversion", C.c_void_p),
        ("nuc_mut_offsets", C.c_void_p), ("nuc_mut_primary", C.c_void_p), ("nuc_mut_secondary", C.c_void_p),
        ("nuc_mut_position", C.c_void_p), ("nuc_mut_gap_position", C.c_void_p), ("nuc_mut_info", C.c_void_p),
        ("nuc_mut_nucs", C.c_void_p),
        ("circular_offset", C.c_void_p), ("rotation_index", C.c_void_p), ("sequence_inverted", C.c_void_p),
        ("branch_length", C.c_void_p),
    ]


class PanMAT:
    """Tree + blocks + gaps + per-node mutation lists, in list order."""

    def __init__(self, names, child_offsets, child_index, root):
        self.names = list(names)
        self.child_offsets = np.ascontiguousarray(child_offsets, np.int32)
        self.child_index = np.ascontiguousarray(child_index, np.int32)
        self.root = int(root)
        n = len(self.names)
        self.blocks: list[tuple[int, list[int]]] = []
        self.gaps: list[tuple[int, list[tuple[int, int]]]] = []
        self.block_muts: list[list[tuple[int, int, int]]] = [[] for _ in range(n)]
        self.nuc_muts: list[list[tuple[int, int, int, int, int, int]]] = [[] for _ in range(n)]
        self.circular = np.full(n, -1, np.int32)
        self.rotation = np.zeros(n, np.int32)
        self.inverted = np.zeros(n, np.uint8)
        self.branch_length = None   # optional float32 [n]; None = Newick defaults

    def set_arrays(self, **arrays):
        """Bulk form: block_primary, block_seq_offsets, block_seq, gap_primary, gap_offsets,
        gap_position, gap_length, block_mut_offsets/_primary/_info/_inversion,
        nuc_mut_offsets/_primary/_secondary/_position/_gap_position/_info/_nucs (numpy)."""
        self._arrays = arrays

    @property
    def num_nodes(self):
        return len(self.names)

    def index(self, name):
        return self.names.index(name)

    def add_block(self, primary: int, seq: str):
        self.blocks.append((primary, encode_block(seq)))

    def add_gaps(self, primary: int, slots: list[tuple[int, int]]):
        self.gaps.append((primary, list(slots)))

    def add_block_mut(self, node: int, primary: int, insertion: bool, inversion: bool):
        self.block_muts[node].append((primary, int(insertion), int(inversion)))

    def add_nuc_mut(self, node: int, primary: int, pos: int, gap: int, mtype: int, codes: list[int],
                    secondary: int = -1):
        info = (len(codes) << 4) + mtype
        nucs = 0
        for i, c in enumerate(codes):
            nucs += c << (4 * (5 - i))
        self.nuc_muts[node].append((primary, secondary, pos, gap, info, nucs))

    def add_nuc_mut_raw(self, node: int, primary: int, pos: int, gap: int, info: int, nucs: int):
        self.nuc_muts[node].append((primary, -1, pos, gap, info, nucs))

    def leaves(self):
        off = self.child_offsets
        return [i for i in range(self.num_nodes) if off[i] == off[i + 1]]

    def as_struct(self):
        """Returns (PanmatStruct, keepalive) -- keep the second alive while the struct is used."""
        keep = []

        def arr(a, dt):
            a = np.ascontiguousarray(np.asarray(a, dtype=dt))
            if a.size == 0:
                a = np.zeros(1, dt)
            keep.append(a)
            return a.ctypes.data

        blob = C.create_string_buffer(b"".join(n.encode() + b"\0" for n in self.names) or b"\0")
        keep.append(blob)
        blob = C.addressof(blob)
        a = getattr(self, "_arrays", None)
        if a is not None:
            return PanmatStruct(
                self.num_nodes, self.root, arr(self.child_offsets, np.int32), arr(self.child_index, np.int32), blob,
                len(a["block_primary"]), arr(a["block_primary"], np.int32), arr(a["block_seq_offsets"], np.int64),
                arr(a["block_seq"], np.uint32),
                len(a["gap_primary"]), arr(a["gap_primary"], np.int32), arr(a["gap_offsets"], np.int64),
                arr(a["gap_position"], np.uint32), arr(a["gap_length"], np.uint32),
                arr(a["block_mut_offsets"], np.int64), arr(a["block_mut_primary"], np.int32),
                arr(a["block_mut_info"], np.uint8), arr(a["block_mut_inversion"], np.uint8),
                arr(a["nuc_mut_offsets"], np.int64), arr(a["nuc_mut_primary"], np.int32),
                arr(a["nuc_mut_secondary"], np.int32), arr(a["nuc_mut_position"], np.int32),
                arr(a["nuc_mut_gap_position"], np.int32), arr(a["nuc_mut_info"], np.uint8),
                arr(a["nuc_mut_nucs"], np.uint32),
                arr(self.circular, np.int32), arr(self.rotation, np.int32), arr(self.inverted, np.uint8),
                self._lengths(arr)), keep
        seq_off = np.zeros(len(self.blocks) + 1, np.int64)
        seq = []
        for i, (_, w) in enumerate(self.blocks):
            seq += w
            seq_off[i + 1] = len(seq)
        g_off = np.zeros(len(self.gaps) + 1, np.int64)
        gpos, glen = [], []
        for i, (_, slots) in enumerate(self.gaps):
            for p, l in slots:
                gpos.append(p)
                glen.append(l)
            g_off[i + 1] = len(gpos)
        b_off = np.zeros(self.num_nodes + 1, np.int64)
        bm = []
        for i, lst in enumerate(self.block_muts):
            bm += lst
            b_off[i + 1] = len(bm)
        n_off = np.zeros(self.num_nodes + 1, np.int64)
        nm = []
        for i, lst in enumerate(self.nuc_muts):
            nm += lst
            n_off[i + 1] = len(nm)
        bm = np.array(bm, np.int64).reshape(-1, 3)
        nm = np.array(nm, np.int64).reshape(-1, 6)
        s = PanmatStruct(
            self.num_nodes, self.root, arr(self.child_offsets, np.int32), arr(self.child_index, np.int32), blob,
            len(self.blocks), arr([p for p, _ in self.blocks], np.int32), arr(seq_off, np.int64),
            arr(seq, np.uint32),
            len(self.gaps), arr([p for p, _ in self.gaps], np.int32), arr(g_off, np.int64), arr(gpos, np.uint32),
            arr(glen, np.uint32),
            arr(b_off, np.int64), arr(bm[:, 0], np.int32), arr(bm[:, 1], np.uint8), arr(bm[:, 2], np.uint8),
            arr(n_off, np.int64), arr(nm[:, 0], np.int32), arr(nm[:, 1], np.int32), arr(nm[:, 2], np.int32),
            arr(nm[:, 3], np.int32), arr(nm[:, 4], np.uint8), arr(nm[:, 5] & 0xFFFFFFFF, np.uint32),
            arr(self.circular, np.int32), arr(self.rotation, np.int32), arr(self.inverted, np.uint8),
            self._lengths(arr))
        return s, keep

    def _lengths(self, arr):
        return None if self.branch_length is None else arr(self.branch_length, np.float32)


def from_msa_dump(dump: str, names, child_offsets, child_index, root) -> PanMAT:
    """PanMAT built by the MSA drivers (canonical dump of pm_msa_build / oracle_msa_build)."""
    pm = PanMAT(names, child_offsets, child_index, root)
    index = {n: i for i, n in enumerate(pm.names)}
    for line in dump.splitlines():
        f = line.split("\t")
        if f[0] == "#error":
            raise ValueError(f[1])
        if f[0] == "#consensus":
            pm.add_block(0, f[1])
        elif f[0] == "#blockmut":
            pm.add_block_mut(index[f[1]], int(f[2]), bool(int(f[4])), bool(int(f[5])))
        else:
            pm.add_nuc_mut_raw(index[f[0]], 0, int(f[1]), int(f[2]), int(f[3]), int(f[4], 16))
    return pm


class PanmanFile:
    """A loaded .panman (libpanman_amd: xz + Cap'n Proto reader, host only); old=True reads
    the older Protobuf PanMAN (panmanOld.treeGroup) instead."""

    def __init__(self, path: str = None, handle: C.c_void_p = None, old: bool = False):
        from ._lib import PanmanError, load
        self.lib = load()
        self.h = C.c_void_p()
        if handle is not None:   # an owned pm_panman produced by the engine (e.g. pm_reroot)
            self.h = handle
            return
        err = C.create_string_buffer(512)
        fn = self.lib.pm_panman_load_old if old else self.lib.pm_panman_load
        rc = fn(path.encode(), C.byref(self.h), err, 512)
        if rc != 0:
            raise PanmanError(f"{'pm_panman_load_old' if old else 'pm_panman_load'}({path}): {err.value.decode()}")

    def __len__(self):
        return self.lib.pm_panman_tree_count(self.h)

    def view(self, i: int = 0) -> PanmatStruct:
        v = PanmatStruct()
        if self.lib.pm_panman_tree(self.h, i, C.byref(v)) != 0:
            raise IndexError(i)
        return v

    def newick(self, i: int = 0) -> str:
        return self.lib.pm_panman_newick(self.h, i).decode()

    def to_panmat(self, i: int = 0) -> PanMAT:
        """Copy tree i into a PanMAT (numpy arrays)."""
        v = self.view(i)
        n = v.num_nodes

        def a(ptr, dt, count):
            if count == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(count,)).copy()
        off = a(v.child_offsets, np.int32, n + 1)
        idx = a(v.child_index, np.int32, n - 1)
        blob = b""
        p = v.names
        for _ in range(n):
            s = C.string_at(p)
            blob += s + b"\0"
            p += len(s) + 1
        names = [x.decode() for x in blob.split(b"\0")[:n]]
        pm = PanMAT(names, off, idx, v.root)
        bo = a(v.block_seq_offsets, np.int64, v.num_blocks + 1)
        go = a(v.gap_offsets, np.int64, v.num_gaps + 1)
        bmo = a(v.block_mut_offsets, np.int64, n + 1)
        nmo = a(v.nuc_mut_offsets, np.int64, n + 1)
        pm.set_arrays(
            block_primary=a(v.block_primary, np.int32, v.num_blocks), block_seq_offsets=bo,
            block_seq=a(v.block_seq, np.uint32, int(bo[-1])), gap_primary=a(v.gap_primary, np.int32, v.num_gaps),
            gap_offsets=go, gap_position=a(v.gap_position, np.uint32, int(go[-1])),
            gap_length=a(v.gap_length, np.uint32, int(go[-1])), block_mut_offsets=bmo,
            block_mut_primary=a(v.block_mut_primary, np.int32, int(bmo[-1])),
            block_mut_info=a(v.block_mut_info, np.uint8, int(bmo[-1])),
            block_mut_inversion=a(v.block_mut_inversion, np.uint8, int(bmo[-1])), nuc_mut_offsets=nmo,
            nuc_mut_primary=a(v.nuc_mut_primary, np.int32, int(nmo[-1])),
            nuc_mut_secondary=a(v.nuc_mut_secondary, np.int32, int(nmo[-1])),
            nuc_mut_position=a(v.nuc_mut_position, np.int32, int(nmo[-1])),
            nuc_mut_gap_position=a(v.nuc_mut_gap_position, np.int32, int(nmo[-1])),
            nuc_mut_info=a(v.nuc_mut_info, np.uint8, int(nmo[-1])),
            nuc_mut_nucs=a(v.nuc_mut_nucs, np.uint32, int(nmo[-1])))
        pm.circular = a(v.circular_offset, np.int32, n)
        pm.rotation = a(v.rotation_index, np.int32, n)
        pm.inverted = a(v.sequence_inverted, np.uint8, n)
        if v.branch_length:
            pm.branch_length = a(v.branch_length, np.float32, n)
        return pm

    def write(self, path: str, compress: bool = True):
        """Write every tree of this file (pm_panman_write)."""
        from ._lib import PanmanError
        views = [self.view(i) for i in range(len(self))]
        arr = (C.c_void_p * max(1, len(views)))(*[C.addressof(v) for v in views])
        rc = self.lib.pm_panman_write(path.encode(), arr, len(views), int(compress))
        if rc != 0:
            raise PanmanError(f"pm_panman_write({path}) failed ({rc})")

    def close(self):
        if self.h:
            self.lib.pm_panman_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_panman(path: str, panmats: list, compress: bool = True):
    """TreeGroup::writeToFile + writePanMAN (xz level 9) for PanMATs."""
    from ._lib import PanmanError, load
    lib = load()
    structs, keep = [], []
    for pm in panmats:
        st, k = pm.as_struct()
        structs.append(st)
        keep.append(k)
    arr = (C.c_void_p * max(1, len(structs)))(*[C.cast(C.pointer(s), C.c_void_p) for s in structs])
    rc = lib.pm_panman_write(path.encode(), arr, len(structs), int(compress))
    del keep
    if rc != 0:
        raise PanmanError(f"pm_panman_write({path}) failed ({rc})")
