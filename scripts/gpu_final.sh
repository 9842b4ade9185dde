#!/bin/bash
# Round-end verification of the current build: -m gpu suite, smoke(), bench line, headline
# profile (kernel trace + PMC), config rows.  usage: bash scripts/gpu_final.sh TAG
TAG=${1:-final}
bash scripts/gpu_round.sh ${TAG}_verify && bash scripts/profile.sh ${TAG}_otr_n64 && bash scripts/gpu_configs.sh ${TAG}_configs
