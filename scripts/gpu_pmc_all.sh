#!/bin/bash
# Spec GPU tests, then PMC of every non-headline kernel on the in-tree build (LastVoting C3,
# OTR2, the lane-packed / wide kernels). usage: bash scripts/gpu_pmc_all.sh TAG
TAG=${1:-pmcall}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_spec.py tests/test_spec_native_text.py -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $OUT/pytest_spec.log 2>&1
rc=$?; tail -3 $OUT/pytest_spec.log; [ $rc -ge 124 ] && exit $rc
bash scripts/pmc_wide.sh ${TAG}_pmc C3_lastvoting_n64,W2_otr2_n64,C4_floodmin_n256_f8,C4_kset_n256_k2_f1,C5_benor_n128,W2_kset_es,W2_epsilon,W2_slv 0.25
# phase split (profiling build: s_memtime per phase) of the packed KSet and the headline OTR
for W in kset4 otr lv; do
  PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1 timeout -k 10 200 python3 scripts/probe_phases.py $W \
    > $OUT/phases_$W.log 2>&1 || exit $?
  tail -12 $OUT/phases_$W.log
done
