"""ctypes binding of libpanman_amd.so (the HIP engine's C-ABI, include/panman_gpu.h).

There is no CPU fallback: if the library is missing or a call fails, this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PANMAN_AMD_LIB") or os.path.join(_HERE, "libpanman_amd.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "panman_gpu.h")

PM_OK = 0
MODE_FITCH = 0
MODE_SANKOFF = 1
MODE_BLOCK_FITCH = 2
MODE_BLOCK_SANKOFF = 3

_lib = None


class PanmanError(RuntimeError):
    pass


class Mut(C.Structure):
    _fields_ = [("node", C.c_uint32), ("site_info", C.c_uint32)]


class Summary(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("nodes", "samples", "substitutions", "insertions", "deletions",
                                          "inversions", "max_depth")] + [("mean_depth", C.c_float)] + \
               [(n, C.c_int64) for n in ("block_insertions", "block_deletions", "block_inversions",
                                          "block_duplications", "block_translocations")]


class Tree(C.Structure):
    _fields_ = [("num_nodes", C.c_int32), ("root", C.c_int32),
                ("child_offsets", C.c_void_p), ("child_index", C.c_void_p)]


_SIGS = {
    "pm_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "pm_destroy": (None, [C.c_void_p]),
    "pm_last_error": (C.c_char_p, [C.c_void_p]),
    "pm_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pm_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "pm_set_option": (C.c_int, [C.c_void_p, C.c_int, C.c_int64]),
    "pm_tree_upload": (C.c_int, [C.c_void_p, C.POINTER(Tree)]),
    "pm_leaves_upload": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p,
                                   C.c_void_p, C.c_int64]),
    "pm_sites_upload": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "pm_run": (C.c_int, [C.c_void_p, C.c_int]),
    "pm_mutation_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "pm_mutations_fetch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
    "pm_site_results": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "pm_site_results_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "pm_kernel_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "pm_synth_tree_sars_like": (C.c_int, [C.c_int64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p]),
    "pm_synth_tree_random_join": (C.c_int, [C.c_int64, C.c_uint64, C.c_void_p, C.c_void_p,
                                            C.POINTER(C.c_int32)]),
    "pm_synth_columns": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_uint64]),
    "pm_leaf_codes_fetch": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]),
    "pm_consensus_fetch": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]),
    "pm_msa_build": (C.c_void_p, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int]),
    "pm_free": (None, [C.c_void_p]),
    "pm_msa_to_panman": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_char_p,
                                   C.c_char_p, C.c_int64]),
    "pm_fasta": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    "pm_fasta_multi": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_void_p),
                                 C.POINTER(C.c_int64), C.c_char_p, C.c_int64]),
    "pm_msa_to_panman_multi": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_void_p, C.c_int,
                                         C.c_char_p, C.c_char_p, C.c_int64]),
    "pm_replay_prepare_range": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64]),
    "pm_replay_prepare": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pm_replay_run": (C.c_int, [C.c_void_p]),
    "pm_replay_format": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    "pm_replay_format_fd": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int64)]),
    "pm_fasta_fd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int64)]),
    "pm_fasta_multi_fd": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int64),
                                    C.c_char_p, C.c_int64]),
    "pm_panman_load": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_int64]),
    "pm_panman_load_old": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_int64]),
    "pm_panman_tree_count": (C.c_int, [C.c_void_p]),
    "pm_panman_tree": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "pm_panman_newick": (C.c_char_p, [C.c_void_p, C.c_int]),
    "pm_panman_free": (None, [C.c_void_p]),
    "pm_panman_write": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "pm_reroot": (C.c_int, [C.c_void_p, C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p)]),
    "pm_pangraph_build": (C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]),
    "pm_comm_unique_id": (C.c_int, [C.c_void_p, C.c_int64]),
    "pm_comm_init_rank": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    "pm_comm_init_all": (C.c_int, [C.c_void_p, C.c_int]),
    "pm_run_gather": (C.c_int, [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]),
    "pm_multi_run": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]),
    "pm_shard_range": (C.c_int, [C.c_int, C.c_int, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "pm_pack_site_results": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]),
    "pm_unpack_site_results": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int64, C.c_void_p,
                                         C.c_void_p]),
    "pm_chunk_entries": (C.c_int, [C.c_int64, C.c_int, C.POINTER(C.c_int64)]),
    "pm_chunk_pack": (C.c_int, [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]),
    "pm_chunk_unpack": (C.c_int, [C.c_void_p, C.c_int64, C.c_int, C.c_int64, C.c_void_p, C.c_void_p]),
    "pm_summary_compute": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(Summary)]),
    "pm_design_bytes": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "pm_build_id": (C.c_char_p, []),
    "pm_phase_reset": (None, []),
    "pm_memory_footprint": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "pm_gather_probe": (C.c_int, [C.c_int, C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "pm_phase_report": (C.c_int64, [C.c_char_p, C.c_int64]),
    "pm_stream_copy_rate": (C.c_int, [C.c_int, C.c_int64, C.c_int, C.POINTER(C.c_double)]),
    "pm_stream_write_rate": (C.c_int, [C.c_int, C.c_int64, C.c_int, C.POINTER(C.c_double)]),
    "pm_warmup": (C.c_int, [C.c_int]),
    "pm_replay_shape": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
}


def build_id() -> str:
    """Hash of the loaded library's sources (pm_build_id)."""
    lib = load()
    return lib.pm_build_id().decode() if hasattr(lib, "pm_build_id") else "unknown"


def phase_reset() -> None:
    """Empty the library's phase log (pm_phase_reset; a no-op on an older experiment build)."""
    lib = load()
    if hasattr(lib, "pm_phase_reset"):
        lib.pm_phase_reset()


def phase_report() -> list[tuple[str, float]]:
    """(phase, seconds) the library's drivers logged since the last phase_reset."""
    lib = load()
    if not hasattr(lib, "pm_phase_report"):
        return []
    need = lib.pm_phase_report(None, 0)
    buf = C.create_string_buffer(int(need))
    lib.pm_phase_report(buf, need)
    out = []
    for line in buf.value.decode().splitlines():
        name, _, secs = line.rpartition("\t")
        out.append((name, float(secs)))
    return out


def header_symbols() -> list[str]:
    """Every function the public header declares."""
    text = re.sub(r"/\*.*?\*/", " ", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(pm_[a-z_0-9]+)\s*\(", text)))


def load():
    """Load the HIP engine.  Raises if the extension was not built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PanmanError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            # an experiment build given by PANMAN_AMD_LIB may predate newer entry points
            if os.environ.get("PANMAN_AMD_LIB") and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib
