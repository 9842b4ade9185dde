#!/bin/bash
# Round 4 probe: integer-multiply / Philox issue costs, the counter list, the new pin tests.
OUT=gpurun_out/r4a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 build/mb_philox > $OUT/mb_philox.log 2>&1 || exit $?
cat $OUT/mb_philox.log
timeout -k 10 120 rocprofv3 -L > $OUT/counters.log 2>&1; echo "counters rc=$?"
timeout -k 10 300 python3 -u -m pytest tests/test_reference_pins.py tests/test_reference_kset.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pins.log 2>&1; echo "pins rc=$?"; tail -3 $OUT/pins.log
