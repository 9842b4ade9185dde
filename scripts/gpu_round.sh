#!/bin/bash
# One GPU iteration: full -m gpu suite, smoke(), one bench line (no PMC).
# Usage (on the box, from the repo root): bash scripts/gpu_round.sh [tag] [pytest args...]
TAG=${1:-round}; shift
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
  tail -5 "$OUT/$name.log"
  case $rc in 0|1|2) return 0 ;; *) echo "fatal rc=$rc in $name, stopping"; exit $rc ;; esac
}
step pytest 900 python3 -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread "$@"
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python3 bench.py --steps 3 --warmup 1
echo done
