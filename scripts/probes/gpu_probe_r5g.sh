#!/bin/bash
# Round 4: the loss-free draw branch marked unlikely (round_amd/expect.so) vs the committed build.
OUT=gpurun_out/r5g; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2_$3.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2_$3.log; }
for rep in 1 2; do for L in libpsg expect; do run $L kset $rep; done; done
for L in libpsg expect; do run $L kses 1; run $L fm 1; done
