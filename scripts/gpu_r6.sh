#!/bin/bash
# round + PMC passes
TAG=${1:-r}
bash scripts/gpu_round.sh $TAG && bash scripts/gpu_pmc.sh pmc_$TAG
