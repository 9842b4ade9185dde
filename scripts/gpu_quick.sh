#!/bin/bash
# Quick GPU iteration: full -m gpu suite, one bench line, one SQ-counter pass.
TAG=${1:-quick}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
  case $rc in 0|1|2) return 0 ;; *) echo "fatal rc=$rc in $name, stopping"; exit $rc ;; esac
}
step pytest 900 python3 -m pytest tests -q -m gpu -p no:cacheprovider
step bench 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --variants= --no-cpu-baseline
echo done
