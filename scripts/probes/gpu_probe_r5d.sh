#!/bin/bash
# Round 4: Philox round keys formed per call (PSG_PHILOX_OPAQUE_KEYS) vs hoisted into SGPRs, and
# the draw-free ablation, on every probe row.
OUT=gpurun_out/r5d; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in kset fm kses otr lv benor slv; do run libpsg $W; run opk $W; done
