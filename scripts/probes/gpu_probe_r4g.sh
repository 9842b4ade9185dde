#!/bin/bash
# Round 4: sender-keyed crash survival — full -m gpu suite on the new build, then an A/B against
# the previous commit (receiver-keyed survival words) on the crash-stop configurations.
OUT=gpurun_out/r4g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
for L in prev libpsg; do
  for W in kset fm lv kses; do
    PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py $W > $OUT/${L}_$W.log 2>&1 || exit $?
    echo "== $L $W"; cat $OUT/${L}_$W.log
  done
done
