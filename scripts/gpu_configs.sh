#!/bin/bash
# Throughput of configuration rows C3-C5 / W2 (bench_configs.py) + kernel-trace stats.
# usage: scripts/gpu_configs.sh TAG [comma-separated name prefixes]
TAG=${1:-cfg}
ONLY=${2:-}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 bench_configs.py --only "$ONLY" --out "$OUT/configs.json" > "$OUT/configs.log" 2>&1
rc=$?; echo "configs rc=$rc"; tail -14 "$OUT/configs.log" | cut -c1-400
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 $ROOT/bench_configs.py --only "$ONLY" --steps 1 --warmup 0 --scale 0.5 > "$OUT/kt.log" 2>&1
echo "kt rc=$?"
