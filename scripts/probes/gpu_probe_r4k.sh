#!/bin/bash
# Round 4: FloodMin / KSet crash-round survival cost (Philox replaced by a hash), the packed
# KSet check without deciders, and the fused OTR / LastVoting rows on the current build.
OUT=gpurun_out/r4k; mkdir -p $OUT; export TMPDIR=/tmp
run() { PSG_LIB=round_amd/$1.so timeout -k 10 240 python3 scripts/probe_ab.py $2 > $OUT/$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; cat $OUT/$1_$2.log; }
for W in fm kset kses; do run libpsg $W; run abl_surv $W; done
timeout -k 10 400 python3 bench_configs.py --only G1_otr_n64_fused,G1_lv_n64_fused,C4_kset > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d = json.loads(l); print(d.get('config', {}).get('workload', d.get('metric')), d.get('value'), d.get('ms_per_step'))
"
