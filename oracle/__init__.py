"""CPU oracle for chunkio's CRC-32 path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker.  chunkio_amd/ never does.
"""
