#!/bin/bash
# Round 4: phase split of the packed KSet (C4 f = 0 / 1 / 32 / 64) and of LastVoting C3 on the current tree.
OUT=gpurun_out/r4z; mkdir -p $OUT; export TMPDIR=/tmp
for W in kset4 lv; do
  PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1 timeout -k 10 300 python3 scripts/probe_phases.py $W > $OUT/timers_$W.log 2>&1 || exit $?
  grep -E "kernel ms|phase cycles" $OUT/timers_$W.log
done
