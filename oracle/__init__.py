"""CPU oracle for DAG-Rider's reachability hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker.  The product (dag_rider_amd/) never uses it.

Parity pinning: the reference is Go and cannot run here (no Go toolchain, see
DESIGN.md s5).  The restatement is pinned against the reference's own known
answers (TestPath, process/process_internal_test.go:20-83, on the Figure-1 DAG
of :86-283) plus SURVEY.md s4's hand-derived answers, both committed in
tests/golden/figure1.json.
"""
from .pyoracle import *  # noqa: F401,F403
from . import setweak  # noqa: F401,E402  (setWeakEdges, process.go:298-310)
from . import buffer  # noqa: F401,E402  (buffer loop + present(), process.go:200-234, :374-384)
