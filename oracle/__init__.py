"""oracle — CPU restatement of the reference (ShuoyiHU/pyqed) hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package, and only as the checker / the timed
CPU baseline — never as the product path (pyqed_amd has no CPU fallback).

Each function restates a reference function with NumPy and cites the
reference file:line it follows.  The restatement is pinned against golden
vectors produced by importing the real reference in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz; see tests/test_oracle_golden.py).
"""
