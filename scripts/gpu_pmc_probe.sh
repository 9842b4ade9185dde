#!/bin/bash
# Phase timers (profiling build round_amd/libpsg_timers.so) + instruction-mix PMC of one probe
# workload on the in-tree libpsg.so.  usage: bash scripts/gpu_pmc_probe.sh TAG otr|lv|fm|kset|benor
TAG=$1; W=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout-s> <cmd...>; a signal/time limit ends the script
  local name=$1 lim=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 -s KILL "$lim" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name" | tee -a $OUT/steps.log; exit $rc; fi
  tail -4 $OUT/$name.log
}
if [ -f round_amd/libpsg_timers.so ]; then
  PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1 step timers 200 python3 scripts/probe_phases.py $W
fi
step pmc_a 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_a -o run -- python3 scripts/probe_phases.py $W
step pmc_b 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_COUNT --kernel-trace --output-format csv -d $OUT/pmc_b -o run -- python3 scripts/probe_phases.py $W
echo done
