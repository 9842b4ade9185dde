#!/bin/bash
# Round 4: fused LastVoting with the compiler's Philox products (the fused-module default now) vs
# the inline v_mad_u64_u32 form; the G1 rows on the final generator.
OUT=gpurun_out/r4s; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/probe_fused.py lv build/fab/lv_cur.co build/fab/lv_mad2.co > $OUT/fused_lv.log 2>&1 || exit $?
cat $OUT/fused_lv.log
timeout -k 10 400 python3 bench_configs.py --only G1_lv_n64_fused,G1_otr_n64_fused > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d = json.loads(l); print(d['config'], d['value'], d['kernel_ms'])
"
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in otr kset lv; do run head $W; run libpsg $W; done
