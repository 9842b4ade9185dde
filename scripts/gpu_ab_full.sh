#!/bin/bash
# Full -m gpu suite on the current libpsg.so, then an A/B of library builds on the headline bench.
# usage: bash scripts/gpu_ab_full.sh TAG libA libB ...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_ab_bench.sh $TAG "$@"
