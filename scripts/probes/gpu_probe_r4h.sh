#!/bin/bash
# Round 4: packed KSet attribution — path counts per round (event-count build), then the C4 rows
# with the crash-round survival draws replaced by a hash and with the check points skipped.
OUT=gpurun_out/r4h; mkdir -p $OUT; export TMPDIR=/tmp
PSG_LIB=round_amd/kset_stats.so PSG_PHASE_TIMERS=1 timeout -k 10 300 python3 scripts/probe_phases.py kset4 > $OUT/stats_kset.log 2>&1 || exit $?
grep -E "kernel ms|phase cycles" $OUT/stats_kset.log
for L in libpsg abl_surv abl_nocheck; do
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py kset > $OUT/${L}_kset.log 2>&1 || exit $?
  echo "== $L"; cat $OUT/${L}_kset.log
done
for L in libpsg abl_surv; do
  for W in fm lv kses; do
    PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py $W > $OUT/${L}_$W.log 2>&1 || exit $?
    echo "== $L $W"; cat $OUT/${L}_$W.log
  done
done
