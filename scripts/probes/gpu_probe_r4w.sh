#!/bin/bash
# Round 4: the survival-call skip confined to crash rounds — BenOr C5 / KSet / FloodMin vs the last commit.
OUT=gpurun_out/r4w; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in benor kset fm otr lv; do run head $W; run libpsg $W; done
