"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference MMSBM EM path used as the parity checker for
the HIP engine.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package; the product path never does.
"""
