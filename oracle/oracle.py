"""ctypes wrapper around the CPU oracle (test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libpm_oracle.so")
_lib = None


def build() -> str:
    """Compile the oracle with g++ (seconds).  Returns the library path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def load() -> "Oracle":
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = C.CDLL(_LIB_PATH)
        lib.oracle_free.argtypes = [C.c_void_p]
        lib.oracle_msa_build.restype = C.c_void_p
        lib.oracle_msa_build.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int]
        lib.oracle_column.restype = C.c_void_p
        lib.oracle_column.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int]
        lib.oracle_csr_columns.restype = C.c_double
        lib.oracle_csr_columns.argtypes = [
            C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_char_p,
            C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
            C.c_int, C.c_int, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_int64), C.c_void_p]
        lib.oracle_fasta.restype = C.c_void_p
        lib.oracle_fasta.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]
        lib.oracle_pangraph.restype = C.c_void_p
        lib.oracle_pangraph.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        lib.oracle_pangraph_fasta.restype = C.c_void_p
        lib.oracle_pangraph_fasta.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int]
        lib.oracle_summary.restype = C.c_void_p
        lib.oracle_summary.argtypes = [C.c_void_p]
        lib.oracle_reroot.restype = C.c_void_p
        lib.oracle_reroot.argtypes = [C.c_void_p, C.c_char_p]
        _lib = lib
    return Oracle(_lib)


def _take_string(lib, ptr) -> str:
    try:
        return C.string_at(ptr).decode()
    finally:
        lib.oracle_free(ptr)


class Oracle:
    ALGO = {"fitch": 0, "sankoff": 1, "block_fitch": 2, "block_sankoff": 3}

    def __init__(self, lib):
        self.lib = lib

    def msa_build(self, newick: str, msa_text: str, reference: str = "", mode: int = 0,
                  threads: int = 1) -> str:
        """M1 (mode 0, Fitch) / M2 (mode 1, low-mem Sankoff) canonical dump."""
        p = self.lib.oracle_msa_build(newick.encode(), msa_text.encode(), reference.encode(),
                                      mode, threads)
        return _take_string(self.lib, p)

    def fasta(self, panmat, aligned: bool, leaf_limit: int = 0, timed: bool = False, threads: int = 1):
        """printFASTAUltraFast records of every leaf (or the first `leaf_limit` by name),
        sorted by name (panman_amd.panmat.PanMAT).  timed=True -> (text, seconds).
        threads > 1: leaves replayed in parallel (the reference's parallel_for_each)."""
        st, keep = panmat.as_struct()
        secs = C.c_double(0.0)
        p = self.lib.oracle_fasta(C.byref(st), int(aligned), int(leaf_limit), int(threads), C.byref(secs))
        del keep
        text = _take_string(self.lib, p)
        return (text, secs.value) if timed else text

    def pangraph(self, flat: str, newick: str, reference: str = "", tbb_order: bool = True) -> str:
        """Tree(PanGraph) dump (M3): blocks, then per node its block mutations and NucMuts.
        tbb_order=False iterates individualSequences as a std::unordered_map instead."""
        p = self.lib.oracle_pangraph(flat.encode(), newick.encode(), reference.encode(), int(tbb_order))
        return _take_string(self.lib, p)

    def pangraph_fasta(self, flat: str, newick: str, reference: str = "", tbb_order: bool = True,
                       aligned: bool = False) -> str:
        """M3 then printFASTAUltraFast on the built Tree: every leaf's record, by name."""
        p = self.lib.oracle_pangraph_fasta(flat.encode(), newick.encode(), reference.encode(), int(tbb_order),
                                           int(aligned))
        return _take_string(self.lib, p)

    def reroot(self, panmat, leaf: str) -> str:
        """Tree::reroot(leaf) dump: the new Newick, then per node (name order) its block
        mutations sorted by block and its NucMut records in list order."""
        st, keep = panmat.as_struct()
        p = self.lib.oracle_reroot(C.byref(st), leaf.encode())
        del keep
        return _take_string(self.lib, p)

    def summary(self, panmat) -> tuple[str, str]:
        """Tree::printSummary text (src/summary.cpp:257-273) and the block lines
        getBlockMutationsParallel prints to std::cout (:203-250)."""
        st, keep = panmat.as_struct()
        p = self.lib.oracle_summary(C.byref(st))
        del keep
        try:
            out = C.string_at(p).decode()
            rest = C.string_at(p + len(out) + 1).decode()
        finally:
            self.lib.oracle_free(p)
        return out, rest

    def column(self, newick: str, leaves: str, algo: str, forced: int, parent: int) -> dict:
        p = self.lib.oracle_column(newick.encode(), leaves.encode(), self.ALGO[algo], forced, parent)
        text = _take_string(self.lib, p)
        out = {"fwd": {}, "final": {}, "muts": {}}
        for line in text.splitlines():
            f = line.split("\t")
            if f[0] == "#error":
                raise ValueError(f[1])
            if f[0] == "F":
                out["fwd"][f[1]] = [int(x) for x in f[2].split(",")] if "," in f[2] else int(f[2])
            elif f[0] == "B":
                out["final"][f[1]] = int(f[2])
            elif f[0] == "M":
                out["muts"][f[1]] = [int(f[2]), f[3]]
        return out

    def csr_columns(self, child_off, child_idx, root, names, leaf_codes, node_row, cons,
                    ref=None, algo=0, threads=1, with_root=False):
        """Faithful per-column loop on a CSR tree.  Returns (seconds, records[n,4]) or, with
        with_root, (seconds, records, root_code[S]) -- root final code per site, 255 = none."""
        child_off = np.ascontiguousarray(child_off, dtype=np.int32)
        child_idx = np.ascontiguousarray(child_idx, dtype=np.int32)
        leaf_codes = np.ascontiguousarray(leaf_codes, dtype=np.uint8)
        node_row = np.ascontiguousarray(node_row, dtype=np.int32)
        cons = np.ascontiguousarray(cons, dtype=np.uint8)
        n = child_off.shape[0] - 1
        sites = leaf_codes.shape[1]
        blob = b"".join(s.encode() + b"\0" for s in names)
        refp = None
        if ref is not None:
            ref = np.ascontiguousarray(ref, dtype=np.uint8)
            refp = ref.ctypes.data
        recs = C.POINTER(C.c_uint32)()
        cnt = C.c_int64(0)
        root_codes = np.zeros(sites, np.uint8)
        secs = self.lib.oracle_csr_columns(
            n, child_off.ctypes.data, child_idx.ctypes.data, int(root), blob,
            leaf_codes.ctypes.data, leaf_codes.strides[0], node_row.ctypes.data, sites,
            cons.ctypes.data, refp, algo, threads, C.byref(recs), C.byref(cnt), root_codes.ctypes.data)
        k = cnt.value
        out = np.ctypeslib.as_array(recs, shape=(max(k, 1) * 4,))[: k * 4].reshape(k, 4).copy()
        self.lib.oracle_free(C.cast(recs, C.c_void_p))
        if with_root:
            return secs, out, root_codes
        return secs, out
