"""ORACLE — test infrastructure only (see oracle/oracle.c).  Importable by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by raytracing_test_amd/."""
