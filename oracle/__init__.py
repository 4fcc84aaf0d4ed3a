"""CPU ORACLE package -- test infrastructure only (see bsm_oracle.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package. The product package basic_sparse_matrix_amd never does.
"""
