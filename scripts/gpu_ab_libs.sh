#!/bin/bash
# A/B of library builds on probe rows: bash scripts/gpu_ab_libs.sh TAG "ROWS" LIB...
# (ROWS: scripts/probe_ab.py row names, e.g. "eps otr"); one line per (row, library)
TAG=$1; ROWS=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for w in $ROWS; do
  for L in round_amd/libpsg.so "$@"; do
    echo "-- $L" >> gpurun_out/$TAG/ab.log
    PSG_LIB=$L timeout -k 10 200 python3 scripts/probe_ab.py $w >> gpurun_out/$TAG/ab.log 2>&1 || exit 1
  done
done
