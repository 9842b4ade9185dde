#!/bin/bash
# Parity subset on the in-tree libpsg.so, then headline (OTR C2) / C3 / config-row A/B of builds.
# usage: bash scripts/gpu_ab_probe.sh TAG "pytest -k expr" "config prefixes" libA libB ...
TAG=$1; K=$2; ONLY=$3; shift 3
mkdir -p gpurun_out/$TAG
if [ -n "$K" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -k "$K" -p no:cacheprovider --timeout 200 \
    --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/$TAG/pytest.log; [ $rc -le 1 ] || exit $rc
fi
for rep in 1 2; do
for L in "$@"; do
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py otr > gpurun_out/$TAG/$L.otr$rep.log 2>&1 || exit 1
  sed "s/^/$L /" gpurun_out/$TAG/$L.otr$rep.log
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py lv > gpurun_out/$TAG/$L.lv$rep.log 2>&1 || exit 1
  sed "s/^/$L /" gpurun_out/$TAG/$L.lv$rep.log
  if [ -n "$ONLY" ] && [ $rep = 1 ]; then
    PSG_LIB=round_amd/$L.so timeout -k 10 300 python3 bench_configs.py --only "$ONLY" --steps 2 --warmup 1 \
      > gpurun_out/$TAG/$L.cfg.log 2>&1 || exit 1
    python3 - "$L" gpurun_out/$TAG/$L.cfg.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[1], d["config"], round(d["kernel_ms"], 2), "%.4g" % d["value"], d["violations"])
PY
  fi
done
done
