#!/bin/bash
# GPU-box profiling run: full bench, rocprofv3 kernel-trace stats, PMC passes.
# Usage (on the box, from the repo root): bash scripts/profile.sh [tag]
# A step that faults / aborts / times out ends the script (no further GPU work).
TAG=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 lim=$2
  shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  case $rc in
    0|1|2) return 0 ;;
    *) echo "fatal rc=$rc in $name, stopping" | tee -a "$OUT/steps.log"; exit $rc ;;
  esac
}

sha256sum "$ROOT/round_amd/libpsg.so" | cut -d' ' -f1 > "$OUT/lib_sha256.txt"
B="python3 $ROOT/bench.py"
SMALL="--steps 2 --warmup 1 --variants= --no-cpu-baseline"

step bench_default 500 $B
step kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- $B $SMALL
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- $B $SMALL
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- $B $SMALL
step pmc_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o run -- $B $SMALL
step pmc_sq2 400 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_COUNT --kernel-trace --output-format csv -d "$OUT/pmc_sq2" -o run -- $B $SMALL
echo done | tee -a "$OUT/steps.log"
