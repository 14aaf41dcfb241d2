"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the sender-recovery path.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by
the product package (eges_amd). Two components:

  liboracle.so        this repo's C restatement of the reference path (oracle/oracle.c)
  _ref/libeges_ref.so the reference libsecp256k1 compiled in place by oracle/Makefile
                      (present wherever it was built; travels to the GPU box as a file)
"""
from .pyoracle import Oracle, RefLib, have_ref  # noqa: F401
