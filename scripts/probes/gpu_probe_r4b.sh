#!/bin/bash
# Round 4 probe: ablation builds of the headline kernel (where the time goes) + exact variants.
OUT=gpurun_out/r4b; mkdir -p $OUT; export TMPDIR=/tmp
for L in libpsg abl_nofrozen abl_cheaprng abl_nodigest mad64; do
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py otr > $OUT/$L.log 2>&1 || exit $?
  echo "== $L"; cat $OUT/$L.log
done
timeout -k 10 300 python3 -u -m pytest tests/test_reference_pins.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k bitset > $OUT/pins.log 2>&1; echo "pins rc=$?"; tail -2 $OUT/pins.log
