#!/bin/bash
# Round 4: how much of packed KSet / FloodMin (C4) is the crash-round survival draw: the same
# kernels with the HO draws' Philox replaced by a cheap hash (ablation build, wrong schedule).
OUT=gpurun_out/r4f; mkdir -p $OUT; export TMPDIR=/tmp
for L in libpsg abl_cheaprng; do
  for W in kset fm; do
    PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py $W > $OUT/${L}_$W.log 2>&1 || exit $?
    echo "== $L $W"; cat $OUT/${L}_$W.log
  done
done
