#!/bin/bash
# LastVoting occupancy variants (round_amd/lv5.so, lv7.so vs the in-tree build) and the phase split
# of the fused OTR / LastVoting Spec modules (profiling build). usage: bash scripts/gpu_ab_lv_fused.sh TAG
TAG=${1:-ablf}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for L in libpsg lv5 lv7; do
  [ -f round_amd/$L.so ] || continue
  PSG_LIB=round_amd/$L.so timeout -k 10 150 python3 scripts/probe_ab.py lv >> $OUT/lv_ab.log 2>&1 || exit $?
done
cat $OUT/lv_ab.log
for A in otr lv; do
  PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1 timeout -k 10 200 python3 scripts/fused_breakdown.py --timers --alg $A \
    > $OUT/fused_timers_$A.log 2>&1 || exit $?
  grep -E "phase cycles|variant" $OUT/fused_timers_$A.log
done
