#!/bin/bash
# Round 4: full -m gpu suite on the scratch-free LV / SLV / Epsilon build (opaque per-lane
# hash and init-address terms, Epsilon at 6 waves/SIMD), then an A/B against the last commit.
OUT=gpurun_out/r4j; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in lv slv eps otr benor kset; do run head $W; run libpsg $W; done
PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1 timeout -k 10 300 python3 scripts/probe_phases.py otr > $OUT/timers_otr.log 2>&1 || exit $?
grep -E "kernel ms|phase cycles" $OUT/timers_otr.log
