#!/bin/bash
# A/B: top priority while a stream-kernel wave waits for its slot and issues
# its refill (-DCIO_PRIO_ISSUE=1) against the kept per-step rotation.
set -u
OUT=gpurun_out/${1:-r03z}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 500 python tools/ab_lib.py --libs $A/crc_base.so,$A/crc_prio_issue.so,$A/crc_base.so,$A/crc_prio_issue.so --cfg cfg2,big --iters 200 --rounds 4 > $OUT/ab_prio_issue.txt 2>&1 || { tail -20 $OUT/ab_prio_issue.txt; exit 1; }
tail -12 $OUT/ab_prio_issue.txt
