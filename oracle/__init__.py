"""oracle -- CPU restatement of the Cocytus EC hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it,
as the checker / timed CPU baseline.  Parity unpinned (see gf8_ref.h).
"""
