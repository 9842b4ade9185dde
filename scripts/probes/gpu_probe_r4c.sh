#!/bin/bash
# Round 4 probe: frozen-tail loop variants of the headline kernel (A/B, same box).
OUT=gpurun_out/r4c; mkdir -p $OUT; export TMPDIR=/tmp
for L in libpsg tail1 tail2 tail4 tail2m mad64 libpsg; do
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py otr > $OUT/$L.log 2>&1 || exit $?
  echo "== $L"; cat $OUT/$L.log
done
