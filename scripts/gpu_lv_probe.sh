#!/bin/bash
# LastVoting C3 probe: phase timers + PMC on the in-tree build, then the kernel time of variants.
bash scripts/gpu_pmc_probe.sh $1 lv || exit $?
shift
for L in "$@"; do
  PSG_LIB=round_amd/$L.so timeout -k 10 200 python3 scripts/probe_ab.py lv 2>&1 | sed "s/^/$L /" || exit 1
done
