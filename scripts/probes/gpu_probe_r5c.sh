#!/bin/bash
# Round 4: packed KSet attribution at f = 0 / 1 — HO sets (every alive sender heard) and the check
# points skipped (probe builds, wrong results).
OUT=gpurun_out/r5c; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for L in libpsg abl_nodraw abl_noho; do run $L kset; done
