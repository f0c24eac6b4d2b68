"""CPU oracle for the panman small-parsimony path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  It wraps oracle/_build/libpm_oracle.so (built from
oracle/pm_oracle.cpp by `make -C oracle`), a restatement of the reference's
src/fitchSankoff.cpp + MSA drivers in src/panman.cpp.  The product library
(panman_amd) never imports it.
"""
from .oracle import (  # noqa: F401
    Oracle,
    load,
)
