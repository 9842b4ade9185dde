#!/bin/bash
# Round 4: loss-free (drop_log2 = 0) draw path for W > 1 (round_amd/lossfree.so) — KSet / KSetES /
# FloodMin parity on that library, then A/B against the committed build.
OUT=gpurun_out/r5e; mkdir -p $OUT; export TMPDIR=/tmp
PSG_LIB=round_amd/lossfree.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -k "kset or KSet or floodmin or FloodMin or schedule" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in kset kses fm otr; do run libpsg $W; run lossfree $W; done
