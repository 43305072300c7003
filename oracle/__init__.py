"""TEST INFRASTRUCTURE ONLY -- the parity oracle for the Paillier hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import anything
under oracle/, and only as the checker / CPU baseline.  The product (fate_amd) never does.
  paillier_oracle.py : pure-Python restatement of rust/fate_utils (paillier, fixedpoint_paillier)
  gmp_ref.c          : the same call sequence on libgmp (the library rug wraps) -- cross-check
                       of the restatement and the timed CPU baseline (cpu_baseline.kind="port")
"""
