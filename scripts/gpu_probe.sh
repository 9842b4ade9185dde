#!/bin/bash
TAG=${1:-probe}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc" -o run -- python3 $ROOT/scripts/otr_rounds_probe.py > "$OUT/probe.log" 2>&1
echo "rc=$?"; tail -2 "$OUT/probe.log"
