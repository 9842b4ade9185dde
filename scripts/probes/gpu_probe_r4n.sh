#!/bin/bash
# Round 4: the symmetric-check-point lowering's membership rewrite and old == current shortcut —
# every generic-Spec GPU test, then the G1 fused rows.
OUT=gpurun_out/r4n; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_spec.py tests/test_spec_native_text.py tests/test_gpu_schedule.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench_configs.py --only G1_lv_n64_fused,G1_otr_n64_fused > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d = json.loads(l); print(d['config'], d['value'], d['kernel_ms'])
"
