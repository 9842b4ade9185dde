#!/bin/bash
# OTR parity subset on the current libpsg.so, then an A/B of library builds on the headline bench.
# usage: bash scripts/gpu_ab_otr.sh TAG libA libB ...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_sampled.py \
  tests/test_gpu_spec.py tests/test_gpu_schedule.py -m gpu -q -x -k "otr or c2 or 2_32 or batch_rows" \
  -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_ab_bench.sh $TAG "$@"
