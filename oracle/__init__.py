"""ORACLE package -- test infrastructure only (CPU restatements of the
reference algorithms).  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package."""
