#!/bin/bash
# Round 4: packed KSet probe — finer phase timers (t2 = HO draws, t5 = rest of the slot updates),
# then an A/B of the uniform-t fast path on the C4 rows (f = 1, 16, 64).
OUT=gpurun_out/r4e; mkdir -p $OUT; export TMPDIR=/tmp
PSG_LIB=round_amd/kset_tprobe.so PSG_PHASE_TIMERS=1 timeout -k 10 300 python3 scripts/probe_phases.py kset4 > $OUT/timers_kset.log 2>&1 || exit $?
grep -E "kernel ms|phase cycles" $OUT/timers_kset.log
for L in libpsg kset_uni libpsg kset_uni; do
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py kset > $OUT/$L.log 2>&1 || exit $?
  echo "== $L"; cat $OUT/$L.log
done
