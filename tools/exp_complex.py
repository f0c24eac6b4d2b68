"""Experiment: fraction of (materialised node, word) Fitch sets with a non-singleton site
at the bench workload (needs the PM_EXP_COUNT_COMPLEX variant via PANMAN_AMD_LIB)."""
import ctypes as C
import sys

import torch  # noqa: F401  (HIP runtime first)

import panman_amd

L = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
S = int(sys.argv[2]) if len(sys.argv) > 2 else 30_000
off, idx, root = panman_amd.random_join_tree(L, seed=1)
e = panman_amd.Engine(0)
e.tree_upload(off, idx, root)
e.synth_columns(0, S, seed=2)
e.run(panman_amd.MODE_FITCH)
print("mutations", e.mutation_count())
out = (C.c_ulonglong * 4)()
e.lib.pm_exp_counters(out)
print(f"complex words {out[0]} of {out[1]} = {out[0] / max(1, out[1]):.4f}")
print(f"simple words {out[2]} = {out[2] / max(1, out[1]):.4f}; of them ACGT-only {out[3]} = {out[3] / max(1, out[2]):.4f}")
