mkdir -p gpurun_out/split3 && export TMPDIR=/tmp
for a in otr lv; do for m in "" --nosplit "" --nosplit; do
  timeout -k 10 150 python3 scripts/fused_breakdown.py --alg $a $m >> gpurun_out/split3/$a.jsonl 2>&1 || exit $?
done; done
grep -E '"(full|inv0|inv1|inv2|Integrity)"' gpurun_out/split3/*.jsonl
timeout -k 10 900 python3 -u -m pytest tests/test_formula.py tests/test_spec_native_text.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/split3/tests.log 2>&1; rc=$?; tail -3 gpurun_out/split3/tests.log; exit $rc
