#!/bin/bash
# Parity subset (pytest -k EXPR) on the current libpsg.so, then an A/B of library builds on
# bench_configs.py rows.  usage: bash scripts/gpu_ab_cfg.sh TAG "pytest -k expr" "config prefixes" libA libB ...
TAG=$1; K=$2; ONLY=$3; shift 3
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q -x -k "$K" -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log; [ $rc -le 1 ] || exit $rc
for L in "$@"; do
  PSG_LIB=round_amd/$L.so timeout -k 10 300 python3 bench_configs.py --only "$ONLY" --steps 2 --warmup 1 \
    > gpurun_out/$TAG/$L.log 2>&1 || exit 1
  python3 - "$L" gpurun_out/$TAG/$L.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[1], d["config"], round(d["kernel_ms"], 2), "%.4g" % d["value"], d["violations"])
PY
done
