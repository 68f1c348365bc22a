"""ORACLE -- test infrastructure only (CPU restatement + reference bindings).  See oracle/oracle.py."""
