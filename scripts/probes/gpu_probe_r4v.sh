#!/bin/bash
# Round 4: BenOr C5 regression — the opaque digest pid and the survival-call skip, each removed.
OUT=gpurun_out/r4v; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for L in b_101efaf libpsg nodig nocw; do run $L benor; done
for L in libpsg nodig nocw; do run $L kset; run $L fm; done
