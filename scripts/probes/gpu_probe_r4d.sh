#!/bin/bash
# Round 4: full -m gpu suite on the current build (frozen tail + mad64 Philox), then the packed
# KSet probe: phase timers (profiling build) and PMC of the C4 rows at f = 0 / 64.
OUT=gpurun_out/r4d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1 timeout -k 10 300 python3 scripts/probe_phases.py kset4 > $OUT/timers_kset.log 2>&1 || exit $?
cat $OUT/timers_kset.log
bash scripts/pmc_wide.sh r4d/pmc C4_kset_n256_k2_f0,C4_kset_n256_k2_f64 0.25 > /dev/null 2>&1 || exit $?
python3 scripts/summarize_pmc.py gpurun_out/r4d/pmc gpurun_out/r4d/pmc_sum --kernel 'kset_packed_kernel#0=50000,16,256' --kernel 'kset_packed_kernel#1=50000,16,256' > /dev/null
python3 -c "
import json; d=json.load(open('gpurun_out/r4d/pmc_sum/pmc_summary.json'))
for k,v in d.items(): print(k, v.get('kernel_trace_avg_ns'), v.get('clock_GHz'), v.get('issue_utilization'), v.get('wave_cycle_split'), v.get('dispatch'))"
