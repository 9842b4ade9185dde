#!/bin/bash
# Round 4 final: verification + matched headline profile, then every configuration row and the
# non-headline PMC, on the same build in one call. usage: bash scripts/gpu_final_r4c.sh TAG
TAG=${1:-r4}
bash scripts/gpu_final_r4.sh $TAG || exit $?
bash scripts/gpu_final_r4b.sh $TAG || exit $?
