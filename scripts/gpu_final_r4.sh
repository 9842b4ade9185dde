#!/bin/bash
# Round-end verification of the current build in one call: -m gpu suite + smoke + bench line
# (gpu_round.sh), the headline profile (profile.sh: kernel trace + PMC), its summary written
# into profiles/TAG_otr_n64 on the box and the default bench line re-run against it
# (bench_matched.json: roofline achieved / frac from this build's own counters).
# usage: bash scripts/gpu_final_r4.sh TAG
TAG=${1:-final}
bash scripts/gpu_round.sh ${TAG}_verify || exit $?
bash scripts/profile.sh ${TAG}_otr_n64 || exit $?
python3 scripts/summarize_profile.py gpurun_out/${TAG}_otr_n64 profiles/${TAG}_otr_n64 > /dev/null || exit $?
cp -r profiles/${TAG}_otr_n64 gpurun_out/${TAG}_otr_n64/summary
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_otr_n64/bench_matched.log 2>&1 || exit $?
grep '^{' gpurun_out/${TAG}_otr_n64/bench_matched.log | cut -c1-300
