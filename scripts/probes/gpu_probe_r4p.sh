#!/bin/bash
# Round 4: sender-keyed crash-round survival for n > 64 (SurvW, lane-parallel) — full -m gpu suite,
# then A/B against the last commit on the crash configurations, and the fused OTR module A/B.
OUT=gpurun_out/r4p; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in kset fm kses lv; do run head $W; run libpsg $W; done
timeout -k 10 400 python3 scripts/probe_fused.py otr build/fab/otr_new.co build/fab/otr_old_cur.co build/fab/otr_old_h3.co > $OUT/fused_otr.log 2>&1 || exit $?
cat $OUT/fused_otr.log
