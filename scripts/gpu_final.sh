#!/bin/bash
# Round-end verification of the current build in one GPU call:
#   1. -m gpu suite + smoke() + default bench line (gpu_round.sh)
#   2. headline profile (profile.sh: kernel trace + PMC) summarized into profiles/TAG_otr_n64,
#      and the default bench line re-run against it (bench_matched.json)
#   3. (full) every configuration row with kernel-trace stats (gpu_configs.sh) and PMC passes over
#      the non-headline kernels (pmc_wide.sh)
# usage: bash scripts/gpu_final.sh TAG [full]
TAG=${1:-final}
bash scripts/gpu_round.sh ${TAG}_verify || exit $?
bash scripts/profile.sh ${TAG}_otr_n64 || exit $?
python3 scripts/summarize_profile.py gpurun_out/${TAG}_otr_n64 profiles/${TAG}_otr_n64 > /dev/null || exit $?
cp -r profiles/${TAG}_otr_n64 gpurun_out/${TAG}_otr_n64/summary
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_otr_n64/bench_matched.log 2>&1 || exit $?
grep '^{' gpurun_out/${TAG}_otr_n64/bench_matched.log | cut -c1-300
[ "$2" = full ] || exit 0
bash scripts/gpu_configs.sh ${TAG}_configs || exit $?
bash scripts/pmc_wide.sh ${TAG}_pmc C3_lastvoting_n64,C4_kset_n256_k2_f1,C4_kset_n256_k2_f64,C4_floodmin_n256_f8,W2_slv,W2_epsilon,W2_kset_es 0.25
