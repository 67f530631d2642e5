"""ORACLE package — test infrastructure only (see climsr_ref.py header)."""
