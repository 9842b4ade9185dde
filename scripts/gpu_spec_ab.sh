#!/bin/bash
# Generic-Spec GPU tests, the fused-Spec cost breakdown (OTR, LastVoting) and the G1 rows.
# usage: bash scripts/gpu_spec_ab.sh TAG
TAG=${1:-specab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_spec.py tests/test_spec_native_text.py -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $OUT/pytest_spec.log 2>&1
rc=$?; tail -3 $OUT/pytest_spec.log; [ $rc -ne 0 ] && exit $rc
for A in otr lv; do
  timeout -k 10 300 python3 scripts/fused_breakdown.py --alg $A > $OUT/breakdown_$A.log 2>&1 || exit $?
  grep '^{' $OUT/breakdown_$A.log | cut -c1-120
done
timeout -k 10 400 python3 bench_configs.py --only G1_otr_n64_fused,G1_lv_n64_fused --out $OUT/configs.json > $OUT/configs.log 2>&1 || exit $?
grep '^{' $OUT/configs.log | cut -c1-200
