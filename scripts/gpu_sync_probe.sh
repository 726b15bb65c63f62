#!/bin/bash
# host round trip of one sync point: memcpy + stream sync vs a post kernel + host spin
set -o pipefail
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/sync_probe scripts/sync_probe.hip && \
timeout -k 10 60 gpurun_out/sync_probe | tee gpurun_out/sync_probe.txt && \
timeout -k 10 60 gpurun_out/sync_probe spin | tee -a gpurun_out/sync_probe.txt
