#!/bin/bash
# A/B of two library builds on config rows (same box, same call).
# usage: bash scripts/gpu_ab.sh TAG "prefixes" libA libB ...
TAG=$1; ONLY=$2; shift 2
mkdir -p gpurun_out/$TAG
for L in "$@"; do
  echo "== $L"
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 bench_configs.py --only "$ONLY" --steps 2 --warmup 1 > gpurun_out/$TAG/$L.log 2>&1 || exit 1
  grep "^{" gpurun_out/$TAG/$L.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(d["config"], round(d["kernel_ms"], 2), "%.3g" % d["value"])
'
done
