#!/bin/bash
# Round 4: BenOr C5 regression bisect (round-4 commits, and the tree without the inline Philox
# products), Epsilon alongside.
OUT=gpurun_out/r4u; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for L in r3final b_fbe0722 b_101efaf b_4c8fbe0 libpsg nomad; do run $L benor; done
for L in r3final libpsg nomad; do run $L eps; done
