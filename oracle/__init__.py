"""CPU oracle for the dmdqn hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  It is the checker: a plain-C restatement (liboracle.so) of the
reference algorithm, each function citing the reference file:line it follows,
pinned against tests/golden/ fixtures produced by the reference's own Python.
The product (dmdqn_amd) never imports it and fails loudly without its HIP
library.
"""
from .oracle import *  # noqa: F401,F403
