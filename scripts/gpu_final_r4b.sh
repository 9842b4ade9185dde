#!/bin/bash
# Round 4, second final call: every configuration row (bench_configs.py) with kernel-trace stats,
# then PMC passes over the non-headline kernels (LastVoting C3, packed KSet f=1 / f=64, packed
# FloodMin f=8, ShortLastVoting, Epsilon, KSetEarlyStopping). usage: bash scripts/gpu_final_r4b.sh TAG
TAG=${1:-r4}
bash scripts/gpu_configs.sh ${TAG}_configs || exit $?
bash scripts/pmc_wide.sh ${TAG}_pmc C3_lastvoting_n64,C4_kset_n256_k2_f1,C4_kset_n256_k2_f64,C4_floodmin_n256_f8,W2_slv,W2_epsilon,W2_kset_es 0.25 || exit $?
