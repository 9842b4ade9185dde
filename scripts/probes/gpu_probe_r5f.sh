#!/bin/bash
# Round 4: loss-free draw path — in every loss-free round (lossfree.so) vs only in crash rounds
# (lossfree2.so) vs the committed build: C4 KSet / KSetES, repeated.
OUT=gpurun_out/r5f; mkdir -p $OUT; export TMPDIR=/tmp
PSG_LIB=round_amd/lossfree2.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -k "kset or KSet or floodmin or FloodMin or schedule" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2_$3.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2_$3.log; }
for rep in 1 2; do for L in libpsg lossfree lossfree2; do run $L kset $rep; done; done
for L in libpsg lossfree lossfree2; do run $L kses 1; done
