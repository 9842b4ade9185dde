#!/bin/bash
# Round 4: fused OTR A/B — the current generated Spec vs round 3's, against the current headers and
# those of round 3 (fdb4cbc) and 4c8fbe0.
OUT=gpurun_out/r4o; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/probe_fused.py otr build/fab/otr_new.co build/fab/otr_old_cur.co build/fab/otr_old_h3.co build/fab/otr_old_h4c.co > $OUT/fused_otr.log 2>&1; rc=$?
cat $OUT/fused_otr.log; exit $rc
