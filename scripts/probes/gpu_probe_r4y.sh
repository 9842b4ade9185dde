#!/bin/bash
# Round 4: EpsilonConsensus rank-based member selection — its GPU parity tests, then A/B.
OUT=gpurun_out/r4y; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -k "epsilon or Epsilon or eps" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for L in head libpsg head libpsg; do run $L eps; done
