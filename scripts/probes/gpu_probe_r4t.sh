#!/bin/bash
# Round 4 vs round 3: the final round-3 kernels (fdb4cbc, built from that commit's sources) and
# the round-4 tree on the same box, every probe row.
OUT=gpurun_out/r4t; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in benor otr lv kset fm kses slv eps; do run r3final $W; run libpsg $W; done
