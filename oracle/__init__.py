"""CPU oracle (TEST INFRASTRUCTURE ONLY): ctypes binding of oracle/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this package.
See mimic_oracle.h for what it restates and how it is pinned.
"""
from .pyoracle import OracleVM, OracleError, load  # noqa: F401
