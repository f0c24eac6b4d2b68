"""Experiment: k_tail lane classes at the bench workload (PM_EXP_TAILSTAT variant via
PANMAN_AMD_LIB): how many tail lanes load leaves (dirty), how many of those have a
non-uniform subtree, how many a uniform subtree whose code differs from the parent's final."""
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
out = (C.c_ulonglong * 8)()
e.lib.pm_exp_tail(out)
tot = out[0] + out[1] + out[2]
dirty = out[3] + out[4] + out[5]
print(f"tail lanes: leaf-parent {out[0]} S2 {out[1]} S3 {out[2]}; dirty {out[3]} {out[4]} {out[5]} "
      f"({dirty / max(1, tot):.3f} of all)")
print(f"dirty & non-uniform {out[6]} ({out[6] / max(1, dirty):.3f} of dirty); dirty & uniform & != parent final {out[7]} "
      f"({out[7] / max(1, dirty):.3f})")
