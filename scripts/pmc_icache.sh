#!/bin/bash
# Instruction-cache PMC pass (one rocprofv3 run per library build) over scripts/probe_ab.py WHICH.
# usage (on the box): bash scripts/pmc_icache.sh TAG WHICH libA libB ...
TAG=$1; WHICH=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for L in "$@"; do
  PSG_LIB=round_amd/$L.so timeout -k 10 -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/$L -o run -- python3 scripts/probe_ab.py $WHICH > $OUT/$L.log 2>&1 || exit $?
  echo "== $L"; cat $OUT/$L.log
done
