#!/bin/bash
# Round 4: Philox products — inline v_mad_u64_u32 with an SGPR-pair carry (default), with the
# carry in VCC (PSG_PHILOX_MAD64=2), and the compiler's mul_lo / mul_hi (0), on the headline,
# LV C3, C4 KSet / FloodMin and the fused OTR module.
OUT=gpurun_out/r4r; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in otr lv kset fm; do run libpsg $W; run mad2 $W; run nomad $W; done
timeout -k 10 400 python3 scripts/probe_fused.py otr build/fab/otr_old_cur.co build/fab/otr_old_cur_mad2.co build/fab/otr_old_cur_nomad.co > $OUT/fused_otr.log 2>&1 || exit $?
cat $OUT/fused_otr.log
