#!/bin/bash
# A/B of library builds (scripts/build_variant.sh NAME ...) on one box in one call:
# scripts/probe_ab.py WHICH (otr | lv | kset | fm | kses | benor | slv | eps) per build, min kernel
# ms over 5 launches. A failing step ends the script (no further GPU work).
# usage: bash scripts/gpu_ab.sh TAG WHICH[,WHICH...] libA libB ...   (libpsg = the in-tree build)
TAG=$1; WHICH=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for w in ${WHICH//,/ }; do
  for L in "$@"; do
    PSG_LIB=round_amd/$L.so timeout -k 10 240 python3 scripts/probe_ab.py $w > $OUT/${L}_$w.log 2>&1 || exit $?
    echo "== $L $w"; cat $OUT/${L}_$w.log
  done
done
