#!/bin/bash
# Round 4: full -m gpu suite (survival calls skipped for crash-free words, scratch-free digest),
# then A/Bs: KSet / FloodMin / KSetES vs the last commit; LV / SLV / Epsilon at the scratch-free
# occupancy targets; OTR at 8 waves/SIMD.
OUT=gpurun_out/r4i; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in kset fm kses; do run head $W; run libpsg $W; done
for W in lv slv eps; do run libpsg $W; run wpe_a $W; done
run libpsg otr; run otr8 otr; run libpsg otr; run otr8 otr
