#!/bin/bash
# A/B of library builds on the headline bench (same box, same call); V = 64 line + V = 2 / 4 variants.
# usage: bash scripts/gpu_ab_bench.sh TAG libA libB ...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for L in "$@"; do
  echo "== $L"
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/$L.log 2>&1 || exit 1
  grep "^{" gpurun_out/$TAG/$L.log | python3 -c '
import json, sys
d = json.loads(sys.stdin.read()); print("V=64", round(d["roofline"]["kernel_ms"], 2), "%.4g" % d["value"], {k: round(v["kernel_ms"], 2) for k, v in d["variants"].items()})
'
done
