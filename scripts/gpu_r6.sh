#!/bin/bash
bash scripts/gpu_round.sh r6 && bash scripts/gpu_pmc.sh pmc6
