"""CPU restatement of the bithash codec path -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package (bitalosdb_amd) never imports it.
"""
