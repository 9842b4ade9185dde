#!/bin/bash
# Round 4: fused OTR header bisect — round 3's generated Spec against the headers of each round-4
# commit (and the working tree without the v_mad_u64_u32 Philox products).
OUT=gpurun_out/r4q; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/probe_fused.py otr build/fab/otr_old_h3.co build/fab/otr_old_fbe0722.co build/fab/otr_old_101efaf.co build/fab/otr_old_4c8fbe0.co build/fab/otr_old_cur.co build/fab/otr_old_cur_nomad.co > $OUT/fused_otr.log 2>&1; rc=$?
cat $OUT/fused_otr.log; exit $rc
