"""ORACLE package — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline)."""
