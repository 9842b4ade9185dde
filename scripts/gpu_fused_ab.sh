#!/bin/bash
# Fused-Spec cost breakdown with and without the symmetric-check-point lowering (OTR, LastVoting),
# then the G1 / C4 KSet config rows. usage: bash scripts/gpu_fused_ab.sh TAG
TAG=${1:-fab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout-s> <cmd...>; a signal / time limit ends the script
  local name=$1 lim=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$lim" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  cat $OUT/$name.log | grep '^{' | cut -c1-200
  if [ $rc -ge 124 ] || [ $rc -eq 1 ] || [ $rc -eq 2 ]; then [ $rc -ge 124 ] && exit $rc; fi
  return 0
}
step otr_sym 300 python3 scripts/fused_breakdown.py
step otr_nosym 300 python3 scripts/fused_breakdown.py --nosym
step lv_sym 300 python3 scripts/fused_breakdown.py --alg lv
step lv_nosym 300 python3 scripts/fused_breakdown.py --alg lv --nosym
step cfg 400 python3 bench_configs.py --only G1_otr_n64_fused,G1_lv_n64_fused,C4_kset_n256_k2_f1,C3_lastvoting --out $OUT/configs.json
echo done
