#!/bin/bash
# PMC passes over the multi-wave kernels (FloodMin n=256 f=8, KSet n=256 k=2, BenOr n=128)
# plus a kernel-trace pass; each pass is its own rocprofv3 run (no counter splitting).
# usage (on the box, repo root): bash scripts/pmc_wide.sh TAG [only-prefixes] [scale]
TAG=${1:-pmcw}
ONLY=${2:-C4_floodmin_n256_f8,C4_kset_n256_k2,C5_benor_n128}
SCALE=${3:-0.25}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
RUN="python3 $ROOT/bench_configs.py --only $ONLY --steps 1 --warmup 0 --scale $SCALE"

step() {  # step <name> <timeout-s> <cmd...>; a signal/time limit ends the script
  local name=$1 lim=$2
  shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 -s KILL "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name, stopping" | tee -a "$OUT/steps.log"; exit $rc; fi
  return 0
}

step list 60 rocprofv3 -L
step kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- $RUN
step pmc_a 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_a" -o run -- $RUN
step pmc_b 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_COUNT --kernel-trace --output-format csv -d "$OUT/pmc_b" -o run -- $RUN
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- $RUN
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- $RUN
echo done | tee -a "$OUT/steps.log"
